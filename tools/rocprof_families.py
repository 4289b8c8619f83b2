"""Per-family totals of a rocprofv3 kernel trace, in the families bench.py's roofline uses
(retr_amd.probe.family_of_symbol): launches, total and average device time per launch.

    python tools/rocprof_families.py <run_results.db | *_kernel_trace.csv> [--steps N]

Totals are also divided by the number of training steps in the trace so they compare directly
with bench.py's ``kernel_families`` (ms per step) and its ``roofline.avg_launch_us``.  That
count is read from the trace itself: the fused stem (``stem_pool_kernel``) runs exactly once
per training step (warm-up, captured and probe steps alike; decode runs its own stem
launches only when the trace holds decode, so pass ``--steps N`` explicitly there).
``--steps N`` overrides; the header line says which count was used and where it came from.
"""
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd.probe import family_of_symbol  # noqa: E402
from tools.prof_summary import from_csv, from_db  # noqa: E402


def main():
    path = sys.argv[1]
    rows = list(from_db(path) if path.endswith(".db") else from_csv(path))   # read twice below
    if "--steps" in sys.argv:
        steps = int(sys.argv[sys.argv.index("--steps") + 1])
        src = "--steps"
    else:
        steps = sum(1 for name, _, _ in rows if "stem_pool_kernel" in name)
        src = "stem_pool_kernel launches in the trace (one per training step)"
        if steps == 0:
            steps, src = 1, "no stem_pool_kernel in the trace: totals per trace"
    print(f"# steps in trace: {steps} ({src})")
    agg = defaultdict(lambda: [0, 0.0])
    other = [0, 0.0]
    for name, us, _ in rows:
        fam = family_of_symbol(name)
        a = agg[fam] if fam else other
        a[0] += 1
        a[1] += us
    print(f"{'family':15s} {'launches':>9} {'total_ms':>10} {'ms/step':>9} {'avg_us':>9}")
    for fam, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{fam:15s} {n:9d} {us / 1e3:10.3f} {us / 1e3 / steps:9.3f} {us / n:9.2f}")
    print(f"{'(other)':15s} {other[0]:9d} {other[1] / 1e3:10.3f} {other[1] / 1e3 / steps:9.3f}")


if __name__ == "__main__":
    main()
