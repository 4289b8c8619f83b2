"""Static instruction mix of kernels in a device assembly file (hipcc --cuda-device-only -S):

    python tools/isa_mix.py file.s <substring>...   (every kernel whose name contains one)"""
import re
import sys
from collections import Counter


def main():
    text = open(sys.argv[1]).read()
    for m in re.finditer(r"^(_Z\S+):\s*; @", text, re.M):
        name = m.group(1)
        if not any(k in name for k in sys.argv[2:]):
            continue
        end = text.index(".Lfunc_end", m.end())
        ins = [ln.split()[0] for ln in text[m.end():end].split("\n")
               if ln.strip() and not ln.strip().startswith((".", ";")) and not ln.strip().endswith(":")]
        c = Counter(ins)
        grp = lambda *p: sum(n for k, n in c.items() if k.startswith(p))  # noqa: E731
        print(f"{name[:90]}\n  total {len(ins)}  valu {grp('v_')}  salu {grp('s_') - grp('s_load', 's_waitcnt', 's_barrier', 's_cbranch', 's_branch')}"
              f"  vmem {grp('global_', 'buffer_', 'flat_')}  lds {grp('ds_')}  waitcnt {grp('s_waitcnt')}")
        print("  " + ", ".join(f"{k} {n}" for k, n in c.most_common(16)))


if __name__ == "__main__":
    main()
