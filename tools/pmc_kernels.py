"""Mean rocprofv3 ``--pmc`` counter values per dispatch, per kernel, from one or more
counter_collection CSVs (one pass each; see pmc_traffic.py for the slot limits):

    python tools/pmc_kernels.py <counter_collection.csv>... [--match dec_] [--top 12]

FETCH_SIZE is printed doubled (the gfx950 correction, MI355X_MICROARCH.md §HBM)."""
import csv
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    match = args[args.index("--match") + 1] if "--match" in args else ""
    top = int(args[args.index("--top") + 1]) if "--top" in args else 12
    paths = [a for i, a in enumerate(args) if not a.startswith("--")
             and (i == 0 or args[i - 1] not in ("--match", "--top"))]
    per = defaultdict(lambda: defaultdict(lambda: [0, 0.0]))
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                k = r.get("Kernel_Name", "")
                if match not in k:
                    continue
                c = per[k][r["Counter_Name"]]
                c[0] += 1
                c[1] += float(r["Counter_Value"])
    rows = sorted(per.items(), key=lambda kv: -max(v[0] for v in kv[1].values()))[:top]
    for k, cs in rows:
        print(k[:110])
        for name, (n, tot) in sorted(cs.items()):
            v = tot / n
            if name == "FETCH_SIZE":
                name, v = "FETCH_SIZE x2 (KiB)", 2 * v
            print(f"    {name:28s} {v:14.1f}   ({n} dispatches)")


if __name__ == "__main__":
    main()
