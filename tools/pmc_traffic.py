"""HBM traffic per launch, per kernel family, from rocprofv3 ``--pmc`` passes.

FETCH_SIZE (3 TCC slots) and WRITE_SIZE (2 slots) do not fit one pass on gfx950, so they come
from two runs (MI355X_MICROARCH.md "rocprofv3 PMC slots").  Both are in KiB.  On gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads, so it is doubled
(MI355X_MICROARCH.md §HBM); WRITE_SIZE is exact for 16-B streaming stores and float atomics.

    python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> \
        --out profiles/pmc_traffic.json --source "<what was run>" [--steps N]

``--steps``: training steps the profiled program ran (bench.py --eager --steps 1 --warmup 1: 2),
so ``dispatches_per_step`` can be set against bench.py's API calls per step (one retr_* call
may dispatch several kernels of a family: the attention backward's dQ and dK/dV kernels, the
two grouped conv weight-gradient kinds).
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd.probe import family_of_symbol  # noqa: E402


def read(path, counter):
    """{family: [dispatches, summed counter]} from a counter_collection CSV."""
    per = defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            fam = family_of_symbol(r.get("Kernel_Name", ""))
            if fam is None:
                continue
            per[fam][0] += 1
            per[fam][1] += float(r["Counter_Value"])
    return per


def main():
    fetch, write = sys.argv[1], sys.argv[2]
    out = sys.argv[sys.argv.index("--out") + 1]
    src = sys.argv[sys.argv.index("--source") + 1] if "--source" in sys.argv else ""
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else None
    fr, wr = read(fetch, "FETCH_SIZE"), read(write, "WRITE_SIZE")
    fams = {}
    for fam in sorted(set(fr) | set(wr)):
        nf, f_kib = fr.get(fam, (0, 0.0))
        nw, w_kib = wr.get(fam, (0, 0.0))
        if not nf or not nw:
            continue
        rd = 2.0 * f_kib * 1024 / nf           # gfx950 FETCH_SIZE x2 correction
        wb = w_kib * 1024 / nw
        fams[fam] = {"bytes_per_launch": round(rd + wb), "read_bytes_per_launch": round(rd),
                     "write_bytes_per_launch": round(wb), "dispatches": [nf, nw]}
        if steps:
            fams[fam]["dispatches_per_step"] = nf / steps
    with open(out, "w") as f:
        json.dump({"source": src, "steps": steps, "correction": "read = 2 x FETCH_SIZE KiB (gfx950), "
                   "write = WRITE_SIZE KiB", "families": fams}, f, indent=1)
    for k, v in fams.items():
        print(f"{k:15s} {v['bytes_per_launch'] / 1e6:10.2f} MB/launch")


if __name__ == "__main__":
    main()
