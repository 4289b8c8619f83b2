"""Summarise a rocprofv3 kernel trace (sqlite .db or kernel_stats/kernel_trace CSV) into a
per-kernel table: calls, total ms, avg us, % of total.  Usage:
    python tools/prof_summary.py <run_results.db | *_kernel_trace.csv> [--top N]
"""
import csv
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = name.replace("retr::", "")
    name = re.sub(r"__hip_bfloat16|__bf16", "bf16", name)
    return name[:160]


def from_db(path):
    c = sqlite3.connect(path)
    q = ("select s.kernel_name, d.start, d.end, s.arch_vgpr_count, s.accum_vgpr_count, "
         "s.group_segment_size from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
         "on d.kernel_id = s.id")
    for name, st, en, vg, ag, lds in c.execute(q):
        yield name, (en - st) * 1e-3, (vg, ag, lds)


def from_csv(path):
    with open(path) as f:
        for r in csv.DictReader(f):
            yield r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3, \
                (r.get("VGPR_Count"), r.get("Accum_VGPR_Count"), r.get("LDS_Block_Size"))


def main():
    path = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    rows = from_db(path) if path.endswith(".db") else from_csv(path)
    agg = defaultdict(lambda: [0, 0.0, None])
    for name, us, res in rows:
        a = agg[short(name)]
        a[0] += 1
        a[1] += us
        a[2] = res
    tot = sum(v[1] for v in agg.values())
    print(f"total kernel time {tot / 1e3:.3f} ms over {sum(v[0] for v in agg.values())} "
          "dispatches")
    print(f"{'calls':>6} {'total_ms':>9} {'avg_us':>8} {'pct':>6}  vgpr/agpr/lds  kernel")
    for k, (n, us, res) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{n:6d} {us / 1e3:9.3f} {us / n:8.1f} {100 * us / tot:6.2f}  {res}  {k}")


if __name__ == "__main__":
    main()
