"""In-process kernel timing with HIP events (used by bench.py for the roofline figure).

When a ``Probe`` is installed, every C-ABI call whose name it tracks is bracketed by two
``torch.cuda.Event``s recorded on torch's current stream — the stream every retr kernel is
launched on — and its algorithmic FLOPs are computed from the call's shape arguments.
A short device-side spin (``retr_spin_us``) is queued in front of the start event, so by the
time the event executes the host has already queued the kernel: the event pair brackets the
kernel's device execution, not the host's launch latency (which a plain eager re-run would
add to every launch).

Family keys match the GEMM kernel's family tag (``gemm_kernel<FAM, ...>`` in csrc/gemm.hpp:
0 linear_fwd, 1 linear_dgrad, 2 linear_wgrad, 3 conv_fwd, 4 conv_dgrad, 5 conv_wgrad) and the
attention kernels, so a family's time here and its rows in a rocprofv3 summary agree.
"""
import torch

from . import _lib

PEAK_FLOPS = 2.5e15    # MI355X dense bf16 MFMA (MI355X_MICROARCH.md), FLOP/s
PEAK_BYTES = 8.0e12    # HBM3E, B/s
RIDGE = PEAK_FLOPS / PEAK_BYTES   # 312.5 FLOP/B: below it a launch is HBM-bound


def _conv_out(h, k, s, p, d):
    return (h + 2 * p - d * (k - 1) - 1) // s + 1


def _conv_variant(k, s, p):
    return "1x1s1" if (k == 1 and s == 1 and p == 0) else f"{k}x{k}"


def flops_of(name, a):
    """(family key, algorithmic FLOPs) of one C-ABI call (2 FLOP per MAC)."""
    name = _ALIAS.get(name, name)
    if name in ("retr_conv2d_fwd", "retr_conv2d_fwd_out"):
        _, _, n, h, w, c, _, _, _, _, co, kh, kw, s, p, d = a[:16]
        oh, ow = _conv_out(h, kh, s, p, d), _conv_out(w, kw, s, p, d)
        if name == "retr_conv2d_fwd_out":
            oh, ow = a[16], a[17]
        return "conv_fwd", 2.0 * n * oh * ow * co * kh * kw * c
    if name == "retr_conv1x1_fwd_cat":
        c1, c2, m, co = a[2], a[4], a[5] * a[6] * a[7], a[14]
        return "conv_fwd", 2.0 * m * co * (c1 + c2)
    if name == "retr_bottleneck_s1_fwd":
        m, cin, ds = a[2] * a[3] * a[4], a[5], a[12]
        k3 = 64 + (cin if ds else 0)
        return "conv_fwd", 2.0 * m * (cin * 64 + 9 * 64 * 64 + k3 * 256)
    if name == "retr_stem_pool_fwd":           # the conv's own pixels (halo recompute excluded)
        return "conv_fwd", 2.0 * a[2] * a[3] * a[4] * a[8] * 256
    if name == "retr_conv2d_dgrad":
        _, _, n, h, w, c, _, _, co, kh, kw, s, p, d = a[:14]
        oh, ow = _conv_out(h, kh, s, p, d), _conv_out(w, kw, s, p, d)
        return "conv_dgrad", 2.0 * n * oh * ow * co * kh * kw * c
    if name == "retr_conv2d_wgrad":
        _, _, _, n, h, w, c, _, co, kh, kw, s, p, d = a[:14]
        oh, ow = _conv_out(h, kh, s, p, d), _conv_out(w, kw, s, p, d)
        return "conv_wgrad", 2.0 * n * oh * ow * co * kh * kw * c
    if name in ("retr_linear_fwd", "retr_linear_fwd_splitk"):
        m, n, k = a[9], a[10], a[11]
        return "linear_fwd", 2.0 * m * n * k
    if name == "retr_linear_fwd_splitk_ln":     # the LayerNorm in its epilogue: no MFMA work
        m, n, k = a[8], a[9], a[10]
        return "linear_fwd", 2.0 * m * n * k
    if name in ("retr_linear_dgrad", "retr_linear_dgrad_splitk"):
        m, n, k = a[8], a[9], a[10]
        return "linear_dgrad", 2.0 * m * n * k
    if name == "retr_linear_wgrad":
        m, n, k = a[7], a[8], a[9]
        return "linear_wgrad", 2.0 * m * n * k
    if name in _GROUPS:
        fam, ia = _GROUPS[name]
        n, arr = a[ia - 1], a[ia]
        return fam, sum(2.0 * arr[i].M * arr[i].N * arr[i].K for i in range(n))
    if name == "retr_linear_wgrad_batch":
        n, arr = a[0], a[1]
        return "linear_wgrad", sum(2.0 * arr[i].M * arr[i].N * arr[i].K for i in range(n))
    if name == "retr_conv2d_wgrad_group":
        n, arr = a[1], a[2]
        fl = 0.0
        for d in (arr[i] for i in range(n)):
            if d.kind >= 0:
                oh = _conv_out(d.H, d.KH, d.stride, d.pad, d.dil)
                ow = _conv_out(d.W, d.KW, d.stride, d.pad, d.dil)
                fl += 2.0 * d.Nb * oh * ow * d.Co * d.KH * d.KW * d.C
        return "conv_wgrad", fl
    if name == "retr_attention_fwd":
        b, h, lq, lk, hd, causal = a[9], a[10], a[11], a[12], a[13], a[15]
        return "attention_fwd", 4.0 * b * h * lq * lk * hd * (0.5 if causal else 1.0)
    if name == "retr_attention_bwd":
        b, h, lq, lk, hd, causal = a[18], a[19], a[20], a[21], a[22], a[24]
        return "attention_bwd", 10.0 * b * h * lq * lk * hd * (0.5 if causal else 1.0)
    return name, 0.0


# entry points measured as another one (same leading arguments; extras are tiny sums)
_ALIAS = {"retr_linear_wgrad_group2": "retr_linear_wgrad_group",
          "retr_attention_fwd_dm": "retr_attention_fwd", "retr_attention_bwd_dm": "retr_attention_bwd"}

# grouped launches: name -> (family, index of the descriptor array in the call's arguments)
_GROUPS = {"retr_linear_fwd_group": ("linear_fwd", 3), "retr_linear_dgrad_group": ("linear_dgrad", 5),
           "retr_linear_wgrad_group": ("linear_wgrad", 2),
           "retr_linear_wgrad_group2": ("linear_wgrad", 2)}


def _esz(dtype):
    return 2 if dtype == 1 else 4


def bytes_of(name, a):
    """Algorithmic (compulsory) HBM bytes of one C-ABI call: every operand read once and every
    output written once in its storage type (bf16 operands, fp32 weight gradients / fp32
    outputs where the call says so).  Split-K slabs, re-reads and padding are implementation
    traffic and are NOT counted here -- the rocprofv3 --pmc passes measure those."""
    name = _ALIAS.get(name, name)
    if name == "retr_conv2d_wgrad_group":      # bf16 dY and X once, fp32 slab-free dW once
        n, arr = a[1], a[2]
        by = 0
        for d in (arr[i] for i in range(n)):
            if d.kind >= 0:
                oh = _conv_out(d.H, d.KH, d.stride, d.pad, d.dil)
                ow = _conv_out(d.W, d.KW, d.stride, d.pad, d.dil)
                by += 2 * (d.Nb * oh * ow * d.Co + d.Nb * d.H * d.W * d.C) \
                    + 4 * d.Co * d.KH * d.KW * d.C
        return by
    if name == "retr_linear_wgrad_batch":      # bf16 operands, fp32 dW / db
        cnt, arr = a[0], a[1]
        return sum(2 * (d.M * d.N + d.M * d.K) + 4 * (d.N * d.K + (d.N if d.db else 0))
                   * (2 if d.accumulate else 1) for d in (arr[i] for i in range(cnt)))
    e = _esz(a[0])
    if name in ("retr_conv2d_fwd", "retr_conv2d_fwd_out"):
        _, _, n, h, w, c, _, _, res, _, co, kh, kw, s, p, d = a[:16]
        oh, ow = _conv_out(h, kh, s, p, d), _conv_out(w, kw, s, p, d)
        if name == "retr_conv2d_fwd_out":
            oh, ow = a[16], a[17]
        out = n * oh * ow * co * e
        return e * (n * h * w * c + co * kh * kw * c) + out * (2 if res else 1)
    if name == "retr_conv1x1_fwd_cat":
        c1, c2, n, oh, ow, co = a[2], a[4], a[5], a[6], a[7], a[14]
        m = n * oh * ow
        return e * (m * (c1 + c2) + co * (c1 + c2) + m * co)
    if name == "retr_bottleneck_s1_fwd":
        m, cin, ds = a[2] * a[3] * a[4], a[5], a[12]
        k3 = 64 + (cin if ds else 0)
        return e * (m * (cin + 256) + 64 * cin + 9 * 64 * 64 + 256 * k3)
    if name == "retr_stem_pool_fwd":           # s2d input once, pooled output once, weights
        n, h2, w2, co = a[2], a[3], a[4], a[8]
        return e * (n * h2 * w2 * 16 + co * 256 + n * ((h2 + 1) // 2) * ((w2 + 1) // 2) * co)
    if name == "retr_conv2d_dgrad":
        _, _, n, h, w, c, _, _, co, kh, kw, s, p, d, addend, gate = a[:16]
        oh, ow = _conv_out(h, kh, s, p, d), _conv_out(w, kw, s, p, d)
        dx = n * h * w * c * e
        return e * (n * oh * ow * co + co * kh * kw * c) + dx * (1 + bool(addend) + bool(gate))
    if name == "retr_conv2d_wgrad":
        _, _, _, n, h, w, c, _, co, kh, kw, s, p, d = a[:14]
        oh, ow = _conv_out(h, kh, s, p, d), _conv_out(w, kw, s, p, d)
        return e * (n * oh * ow * co + n * h * w * c) + 4 * co * kh * kw * c
    if name in ("retr_linear_fwd", "retr_linear_fwd_splitk"):
        yf32, m, n, k, res = a[8], a[9], a[10], a[11], a[13]
        return e * (m * k + n * k) + m * n * (4 if yf32 else e) + (4 * m * n if res else 0)
    if name == "retr_linear_fwd_splitk_ln":     # fp32 out + the LayerNorm's bf16 outputs
        m, n, k, res = a[8], a[9], a[10], a[12]
        ln = getattr(a[18], "_obj", None)
        nout = (bool(ln.y) + bool(ln.y2)) if ln is not None else 1
        return e * (m * k + n * k) + 4 * m * n + (4 * m * n if res else 0) + 2 * m * n * nout
    if name in ("retr_linear_dgrad", "retr_linear_dgrad_splitk"):
        dxf32, m, n, k, addend, af32, gate = a[7], a[8], a[9], a[10], a[11], a[12], a[14]
        return (e * (m * n + n * k) + m * k * (4 if dxf32 else e)
                + (m * k * (4 if af32 else e) if addend else 0) + (m * k * e if gate else 0))
    if name == "retr_linear_wgrad":
        m, n, k, acc = a[7], a[8], a[9], a[11]
        return e * (m * n + m * k) + 4 * n * k * (2 if acc else 1)
    if name == "retr_linear_fwd_group":
        yf32, cnt, arr = a[1], a[2], a[3]
        return sum(e * (d.M * d.K + d.N * d.K) + d.M * d.N * (4 if yf32 else e)
                   + (4 * d.M * d.N if d.residual else 0) for d in (arr[i] for i in range(cnt)))
    if name == "retr_linear_dgrad_group":
        dxf32, af32, cnt, arr = a[1], a[2], a[4], a[5]
        return sum(e * (d.M * d.N + d.N * d.K) + d.M * d.K * (4 if dxf32 else e)
                   + (d.M * d.K * (4 if af32 else e) if d.addend else 0)
                   + (d.M * d.K * e if d.gate else 0) for d in (arr[i] for i in range(cnt)))
    if name == "retr_linear_wgrad_group":
        cnt, arr = a[1], a[2]
        return sum(e * (d.M * d.N + d.M * d.K) + 4 * d.N * d.K * (2 if d.accumulate else 1)
                   for d in (arr[i] for i in range(cnt)))
    if name == "retr_attention_fwd":
        b, h, lq, lk, hd = a[9], a[10], a[11], a[12], a[13]
        return e * b * h * hd * (2 * lq + 2 * lk) + 4 * b * h * lq
    if name == "retr_attention_bwd":
        b, h, lq, lk, hd = a[18], a[19], a[20], a[21], a[22]
        # read q k v o dO (+lse), write dq dk dv
        return e * b * h * hd * (3 * lq + 2 * lk + lq + 2 * lk) + 4 * b * h * lq
    return 0


def shape_of(name, a):
    """Short shape tag of a call (for the per-shape breakdown)."""
    name = _ALIAS.get(name, name)
    if name in _GROUPS:
        n, arr = a[_GROUPS[name][1] - 1], a[_GROUPS[name][1]]
        return "group " + " + ".join(f"M{arr[i].M} N{arr[i].N} K{arr[i].K}" for i in range(n))
    if name == "retr_linear_wgrad_batch":
        return f"batch of {a[0]} (+{a[2]} partial-row sums)"
    if name == "retr_conv2d_wgrad_group":
        return f"group of {a[1]} conv weight gradients"
    if name in ("retr_conv2d_fwd", "retr_conv2d_fwd_out"):
        return f"N{a[2]} {a[3]}x{a[4]}x{a[5]} ->{a[10]} k{a[11]} s{a[13]} d{a[15]}"
    if name == "retr_conv1x1_fwd_cat":
        return f"N{a[5]} {a[6]}x{a[7]} [{a[2]}|{a[4]} s{a[10]}] ->{a[14]} k1 cat"
    if name == "retr_bottleneck_s1_fwd":
        return f"N{a[2]} {a[3]}x{a[4]}x{a[5]} bottleneck ds{a[12]}"
    if name == "retr_stem_pool_fwd":
        return f"N{a[2]} {a[3]}x{a[4]}x16 ->{a[8]} k4 stem+maxpool"
    if name == "retr_conv2d_dgrad":
        return f"N{a[2]} {a[3]}x{a[4]}x{a[5]} <-{a[8]} k{a[9]} s{a[11]} d{a[13]}"
    if name == "retr_conv2d_wgrad":
        return f"N{a[3]} {a[4]}x{a[5]}x{a[6]} ->{a[8]} k{a[9]} s{a[11]} d{a[13]}"
    if name == "retr_linear_fwd":
        return f"M{a[9]} N{a[10]} K{a[11]} relu{a[12]} res{int(bool(a[13]))}"
    if name == "retr_linear_dgrad":
        return f"M{a[8]} N{a[9]} K{a[10]} add{int(bool(a[11]))} gate{int(bool(a[14]))}"
    if name == "retr_linear_dgrad_splitk":
        return f"M{a[8]} N{a[9]} K{a[10]} add{int(bool(a[11]))} gate{int(bool(a[14]))} split{a[18]}"
    if name == "retr_linear_fwd_splitk":
        return f"M{a[9]} N{a[10]} K{a[11]} relu{a[12]} res{int(bool(a[13]))} split{a[18]}"
    if name == "retr_linear_fwd_splitk_ln":
        return f"M{a[8]} N{a[9]} K{a[10]} relu{a[11]} res{int(bool(a[12]))} split{a[17]} +LN"
    if name == "retr_linear_wgrad":
        return f"M{a[7]} N{a[8]} K{a[9]} db{int(bool(a[10]))} acc{a[11]}"
    if name == "retr_attention_fwd":
        return f"B{a[9]} H{a[10]} Lq{a[11]} Lk{a[12]} hd{a[13]} c{a[15]}"
    if name == "retr_attention_bwd":
        return f"B{a[18]} H{a[19]} Lq{a[20]} Lk{a[21]} hd{a[22]} c{a[24]}"
    return ""


TRACKED = ("retr_conv2d_fwd", "retr_conv2d_fwd_out", "retr_conv1x1_fwd_cat",
           "retr_bottleneck_s1_fwd", "retr_stem_pool_fwd", "retr_conv2d_dgrad", "retr_conv2d_wgrad", "retr_linear_fwd",
           "retr_linear_fwd_splitk", "retr_linear_fwd_splitk_ln",
           "retr_linear_dgrad", "retr_linear_dgrad_splitk", "retr_linear_wgrad",
           "retr_linear_fwd_group", "retr_linear_dgrad_group", "retr_linear_wgrad_group",
           "retr_linear_wgrad_group2", "retr_linear_wgrad_batch", "retr_conv2d_wgrad_group",
           "retr_attention_fwd",
           "retr_attention_bwd",
           "retr_attention_fwd_dm", "retr_attention_bwd_dm")


FAMILY_SYMBOL = {"linear_fwd": "gemm{,2,2_group,_short}_kernel<0,",
                 "linear_dgrad": "gemm{,2,2_group,_short}_kernel<1,",
                 "linear_wgrad": "gemm{,2,2_group}_kernel<2, + wgrad_batch_kernel",
                 "conv_fwd": "gemm{,2}_kernel<3, + conv3x3_kernel<..., false> + bottleneck_s1_kernel + stem_pool_kernel",
                 "conv_dgrad": "gemm{,2}_kernel<4, + conv3x3_kernel<..., true>",
                 "conv_wgrad": "gemm{,2}_kernel<5, + conv_wgrad_group_kernel",
                 "attention_fwd": "attn_fwd{,2,2s}_kernel + attn_keep_bits_kernel",
                 "attention_bwd": "attn_bwd_"}


def family_of_symbol(name):
    """Family key of a rocprof kernel name (mangled ``_ZN4retr11gemm_kernelILi3E...`` or
    demangled ``retr::gemm_kernel<3, ...>``), or None."""
    import re
    m = re.search(r"gemm(?:2|_short)?(?:_group)?_kernelILi(\d+)E", name) or \
        re.search(r"gemm(?:2|_short)?(?:_group)?_kernel<(\d+),", name)
    if m:
        return ("linear_fwd", "linear_dgrad", "linear_wgrad", "conv_fwd", "conv_dgrad",
                "conv_wgrad")[int(m.group(1))]
    m = re.search(r"conv3x3_kernelI(?:Li\d+E){5,7}Lb([01])E", name) or \
        re.search(r"conv3x3_kernel<(?:\d+, ){5,7}(false|true)", name)
    if m:                                         # direct 3x3 conv (csrc/conv3x3.hip)
        return "conv_dgrad" if m.group(1) in ("1", "true") else "conv_fwd"
    if "wgrad_batch_kernel" in name:
        return "linear_wgrad"
    if "conv_wgrad_group_kernel" in name:
        return "conv_wgrad"
    if "bottleneck_s1_kernel" in name or "stem_pool_kernel" in name:
        return "conv_fwd"
    if re.search(r"attn_fwd\d*s?_kernel", name) or "attn_keep_bits_kernel" in name:
        return "attention_fwd"
    if "attn_bwd_" in name:
        return "attention_bwd"
    return None


class Probe:
    def __init__(self, names=TRACKED, detail=False, spin_us=40.0):
        self.names = set(names)
        self.detail = detail
        self.spin_us = spin_us
        self.records = []     # (key, flops, bytes, ev0, ev1)
        self.active = False

    def wrap(self, name, args, fn):
        if not self.active:
            return fn()
        key, fl = flops_of(name, args)
        by = bytes_of(name, args)
        if self.detail:
            key = f"{key} | {shape_of(name, args)}"
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        if self.spin_us > 0:
            _lib._raw_call("retr_spin_us", (float(self.spin_us), _lib.stream()))
        e0.record()
        fn()
        e1.record()
        self.records.append((key, fl, by, e0, e1))

    def summary(self, peak_flops=PEAK_FLOPS, peak_bytes=PEAK_BYTES):
        """{key: {launches, ms_total, ms_avg, tflops, flops, bytes, attainable_ms}} (call after
        synchronising).  ``attainable_ms`` = sum over launches of max(FLOP / MFMA peak,
        algorithmic bytes / HBM peak): the time each launch would take at its own roofline."""
        out = {}
        for key, fl, by, e0, e1 in self.records:
            ms = e0.elapsed_time(e1)
            d = out.setdefault(key, {"launches": 0, "ms_total": 0.0, "flops": 0.0,
                                     "bytes": 0.0, "attainable_ms": 0.0})
            d["launches"] += 1
            d["ms_total"] += ms
            d["flops"] += fl
            d["bytes"] += by
            d["attainable_ms"] += max(fl / peak_flops, by / peak_bytes) * 1e3
        for d in out.values():
            finish(d)
        return out

    def __enter__(self):
        _lib.set_probe(self)
        self.active = True
        return self

    def __exit__(self, *exc):
        self.active = False
        _lib.set_probe(None)


def finish(d):
    """Derived rates of a summary entry (after its sums changed)."""
    d["ms_avg"] = d["ms_total"] / max(1, d["launches"])
    t = d["ms_total"] * 1e-3
    d["tflops"] = d["flops"] / t / 1e12 if t else 0.0
    d["gbs"] = d["bytes"] / t / 1e9 if t else 0.0
    d["intensity"] = d["flops"] / d["bytes"] if d["bytes"] else float("inf")
    d["attainable_frac"] = d["attainable_ms"] / d["ms_total"] if d["ms_total"] else 0.0
    return d
