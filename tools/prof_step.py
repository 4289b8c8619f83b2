"""Per-step kernel breakdown of a rocprofv3 trace of bench.py.

Splits the dispatch stream into training steps at the stem's NCHW->NHWC kernel (one launch per
step), takes one step window (default: the 7th) and prints (a) per-kernel totals inside it and
(b) the GEMM launches grouped by instantiation and grid size.

    python tools/prof_step.py gpurun_out/prof/run_results.db [--step N]
"""
import os
import re
import sqlite3
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from retr_amd.probe import family_of_symbol  # noqa: E402

# kernels outside the roofline families, by name fragment (first match wins)
CATEGORIES = [("slab_sum_group", "linear wgrad slab sums"), ("table_put", "wgrad batch tables"),
              ("slab_epilogue", "split-K slab epilogues"),
              ("wgrad_unpack", "conv wgrad slab sums + OIHW"),
              ("adamw", "clip + AdamW"), ("ln_", "LayerNorm"), ("embed", "embeddings"),
              ("ce_", "cross-entropy"), ("pos_grad", "position gradients"),
              ("conv_pack", "conv weight packing"), ("cat_rows", "conv weight packing"),
              ("dropout", "dropout"), ("phase_fill", "dgrad phase fill"),
              ("nchw_to", "input layout"), ("mask", "masks"), ("seed", "dropout seed"),
              ("fill", "fills / copies"), ("copy", "fills / copies"), ("cast", "casts")]


def category(name):
    f = family_of_symbol(name)
    if f:
        return f
    for frag, cat in CATEGORIES:
        if frag in name:
            return cat
    return "other"


def main():
    path = sys.argv[1]
    step = int(sys.argv[sys.argv.index("--step") + 1]) if "--step" in sys.argv else 6
    c = sqlite3.connect(path)
    q = ("select s.kernel_name, d.start, d.end, d.grid_size_x, d.grid_size_y, d.grid_size_z, "
         "d.workgroup_size_x from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
         "on d.kernel_id = s.id order by d.start")
    rows = list(c.execute(q))
    marks = [i for i, r in enumerate(rows) if "nchw_to_nhwc" in r[0] or "nchw_to_s2d" in r[0]]
    w = rows[marks[step]:marks[step + 1]]
    span = (w[-1][2] - w[0][1]) / 1e6
    busy = sum(r[2] - r[1] for r in w) / 1e6
    print(f"step window {step}: {len(w)} dispatches, span {span:.3f} ms, kernel busy {busy:.3f} ms")
    cat = defaultdict(lambda: [0, 0.0])
    for r in w:
        c = category(r[0])
        cat[c][0] += 1
        cat[c][1] += (r[2] - r[1]) / 1e3
    print(f"\n{'category':32s} {'calls':>5} {'ms':>7} {'share':>6}")
    for c, (n, us) in sorted(cat.items(), key=lambda kv: -kv[1][1]):
        print(f"{c:32s} {n:5d} {us / 1e3:7.3f} {us / 1e3 / busy:6.1%}")
    agg = defaultdict(lambda: [0, 0.0])
    for r in w:
        k = re.sub(r"^_ZN\d*", "", r[0])[:110]
        agg[k][0] += 1
        agg[k][1] += (r[2] - r[1]) / 1e3
    print(f"\n{'calls':>5} {'total_us':>9}  kernel")
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"{n:5d} {us:9.1f}  {k}")
    g = defaultdict(lambda: [0, 0.0])
    for r in w:
        if "gemm" not in r[0]:
            continue
        key = (re.sub(r"^_ZN\d*", "", r[0])[:100], r[3] // r[6], r[4], r[5])
        g[key][0] += 1
        g[key][1] += (r[2] - r[1]) / 1e3
    print(f"\nGEMM launches by instantiation and grid (blocks x splits):")
    for k, (n, us) in sorted(g.items(), key=lambda kv: -kv[1][1])[:50]:
        print(f"{n:4d} {us:8.1f} us {us / n:7.1f} us/launch grid={k[1]}x{k[2]}  {k[0]}")


if __name__ == "__main__":
    main()
