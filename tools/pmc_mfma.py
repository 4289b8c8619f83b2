"""MFMA utilisation and instruction mix per kernel family / kernel from one rocprofv3 --pmc pass.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA \
        SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d <dir> -o run -- python3 <program>
    python tools/pmc_mfma.py <dir>/.../run_counter_collection.csv --out profiles/pmc_mfma.json \
        --source "<what was run>" [--by-kernel 25]

Per dispatch (rocprofv3 sums each counter over its hardware instances):
  * mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs), cycles per dispatch =
    min(GRBM_GUI_ACTIVE / 8, duration x 2.4 GHz): rocprof's own MfmaUtil
    (counter_defs.yaml: sum(MFMA_BUSY) / (max(GRBM_GUI_ACTIVE) x SIMD_NUM); GRBM_GUI_ACTIVE
    is summed over the 8 XCDs, MI355X_MICROARCH.md "DVFS give-back"), except that on short
    dispatches GRBM_GUI_ACTIVE spans more than the dispatch (its quotient by the duration
    reads above the 2.4 GHz maximum clock): there the dispatch's own duration at the maximum
    clock is the denominator (a lower bound on the busy fraction).  ``mfma_busy_grbm`` keeps
    the uncorrected figure and ``clock_ghz`` the raw GRBM quotient;
  * mfma_flop = SQ_VALU_MFMA_BUSY_CYCLES x 1024: the FLOPs the busy cycles correspond to for
    bf16 (a 32x32x16 bf16 MFMA = 32 busy cycles = 32768 FLOP; MI355X_MICROARCH.md), to compare
    with the algorithmic FLOPs (padding and recomputation show as a surplus);
  * valu_per_mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA (wave instructions; SQ_INSTS_VALU includes
    the MFMAs).  Families are aggregated busy-cycle-weighted (sums of counters).
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd.probe import family_of_symbol  # noqa: E402

SIMDS = 1024
XCDS = 8


MAX_CLOCK_GHZ = 2.4


def read(path):
    """{dispatch id: (kernel name, {counter: value}, duration ns)}."""
    rows = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = rows.setdefault(r["Dispatch_Id"], [r["Kernel_Name"], {}, 0])
            d[1][r["Counter_Name"]] = d[1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            try:
                d[2] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            except (KeyError, ValueError):
                pass
    return rows


def short(name):
    """Kernel name without the return type, anonymous-namespace prefix and argument list."""
    for pre in ("void ", "(anonymous namespace)::"):
        if name.startswith(pre):
            name = name[len(pre):]
    return name.split("(")[0][:110]


def summarise(groups):
    out = {}
    for key, (n, c, ns) in groups.items():
        busy, grbm = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), c.get("GRBM_GUI_ACTIVE", 0.0)
        valu, mfma = c.get("SQ_INSTS_VALU", 0.0), c.get("SQ_INSTS_MFMA", 0.0)
        cyc = c.get("_cycles", 0.0)
        e = {"dispatches": n, "mfma_busy": round(busy / (cyc * SIMDS), 4) if cyc else None,
             "mfma_busy_grbm": round(busy / (grbm / XCDS * SIMDS), 4) if grbm else None,
             "clock_corrected_dispatches": int(c.get("_clamped", 0)),
             "mfma_flop_per_dispatch": round(busy * 1024 / n),
             "valu_per_mfma": round(valu / mfma, 2) if mfma else None,
             "insts_per_dispatch": {k: round(v / n) for k, v in sorted(c.items())
                                    if k.startswith("SQ_INSTS")},
             "clock_ghz": round(grbm / XCDS / ns, 3) if ns else None,
             "us_per_dispatch": round(ns / n / 1e3, 2)}
        out[key] = e
    return out


def main():
    path = sys.argv[1]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    src = sys.argv[sys.argv.index("--source") + 1] if "--source" in sys.argv else ""
    nk = int(sys.argv[sys.argv.index("--by-kernel") + 1]) if "--by-kernel" in sys.argv else 25
    rows = read(path)
    fam = defaultdict(lambda: [0, defaultdict(float), 0])
    ker = defaultdict(lambda: [0, defaultdict(float), 0])
    for name, c, ns in rows.values():
        # per-dispatch cycle denominator: GRBM_GUI_ACTIVE / 8, clamped to the dispatch's own
        # duration at the maximum clock when GRBM spans more than the dispatch
        g8 = c.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        cap = ns * MAX_CLOCK_GHZ if ns else g8
        c = dict(c)
        c["_cycles"] = min(g8, cap) if ns else g8
        c["_clamped"] = 1.0 if (ns and g8 > cap) else 0.0
        f = family_of_symbol(name) or "(other)"
        for g, k in ((fam, f), (ker, short(name))):
            g[k][0] += 1
            g[k][2] += ns
            for cn, v in c.items():
                g[k][1][cn] += v
    fams = summarise(fam)
    top = sorted(ker.items(), key=lambda kv: -kv[1][2])[:nk]
    kers = summarise(dict(top))
    res = {"source": src, "formula": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (min(GRBM_GUI_ACTIVE "
           "/ 8 XCDs, duration x 2.4 GHz) x 1024 SIMDs) per dispatch (rocprof MfmaUtil, clamped "
           "where GRBM spans more than the dispatch); mfma_busy_grbm = the unclamped figure; "
           "mfma_flop = busy cycles x 1024 (bf16); valu_per_mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA", "families": fams, "kernels": kers}
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
    def ghz(e):
        # GRBM_GUI_ACTIVE / 8 / duration reads above the 2.4 GHz maximum clock when the counter
        # spans more than the dispatch (short kernels): that quotient is not a clock -- print
        # "clamp" (the busy fraction used the dispatch duration at 2.4 GHz instead)
        g = e["clock_ghz"]
        return "  n/a" if g is None else (f"{g:6.2f}" if g <= 2.4 else " clamp")
    print(f"{'family / kernel':60s} {'n':>5} {'us/disp':>9} {'mfma_busy':>9} {'VALU/MFMA':>9} "
          f"{'GHz':>6}")
    for k, e in sorted(fams.items(), key=lambda kv: -kv[1]["us_per_dispatch"] * kv[1]["dispatches"]):
        print(f"{k:60s} {e['dispatches']:5d} {e['us_per_dispatch']:9.2f} "
              f"{e['mfma_busy'] if e['mfma_busy'] is not None else 0:9.3f} "
              f"{e['valu_per_mfma'] or 0:9.2f} {ghz(e)}")
    print()
    for k, e in kers.items():
        print(f"{k[:60]:60s} {e['dispatches']:5d} {e['us_per_dispatch']:9.2f} "
              f"{e['mfma_busy'] if e['mfma_busy'] is not None else 0:9.3f} "
              f"{e['valu_per_mfma'] or 0:9.2f} {ghz(e)}")


if __name__ == "__main__":
    main()
