"""ctypes binding of ``libretr_hip.so`` (the gfx950 kernels; C-ABI in ``include/retr_hip.h``).

The product path has no fallback: if the library is missing or a CUDA/HIP device is absent,
every op raises.  Build the library with ``make`` (or ``__graft_entry__.build()``).
"""
import ctypes
import os
import warnings

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libretr_hip.so")
# A/B measurements only (tools/*_micro.py, tools/ab_step.py): time a baseline build of the same
# C-ABI.  Never silent: a stray setting would swap every kernel of the process.
if os.environ.get("RETR_AB_LIB"):
    LIB_PATH = os.environ["RETR_AB_LIB"]
    import sys as _sys
    print(f"retr_amd: RETR_AB_LIB is set -- loading kernels from {LIB_PATH} instead of the "
          f"in-tree libretr_hip.so (A/B tooling only)", file=_sys.stderr)

F32, BF16 = 0, 1
TUNE_COUNT = 40          # include/retr_hip.h RETR_TUNE_COUNT

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float
_D = ctypes.c_double
_U64 = ctypes.c_ulonglong
_SZ = ctypes.c_size_t



class LinearFwdDesc(ctypes.Structure):
    """retr_linear_fwd_desc (include/retr_hip.h)"""
    _fields_ = [("x", _P), ("ldx", _L), ("w", _P), ("ldw", _L), ("bias", _P), ("y", _P),
                ("ldy", _L), ("residual", _P), ("ldr", _L), ("drop_p", _F), ("seed", _U64),
                ("M", _I), ("N", _I), ("K", _I), ("relu", _I)]


class LinearDgradDesc(ctypes.Structure):
    """retr_linear_dgrad_desc"""
    _fields_ = [("dy", _P), ("lddy", _L), ("w", _P), ("ldw", _L), ("dx", _P), ("lddx", _L),
                ("addend", _P), ("lda", _L), ("gate", _P), ("ldg", _L), ("M", _I), ("N", _I),
                ("K", _I), ("pad", _I)]


class LinearWgradDesc(ctypes.Structure):
    """retr_linear_wgrad_desc"""
    _fields_ = [("dy", _P), ("lddy", _L), ("x", _P), ("ldx", _L), ("dw", _P), ("lddw", _L),
                ("db", _P), ("M", _I), ("N", _I), ("K", _I), ("accumulate", _I)]


class ConvWgradDesc(ctypes.Structure):
    """retr_conv_wgrad_desc"""
    _fields_ = [("dy", _P), ("x", _P), ("ws", _P), ("Nb", _I), ("H", _I), ("W", _I), ("C", _I),
                ("Co", _I), ("KH", _I), ("KW", _I), ("stride", _I), ("pad", _I), ("dil", _I),
                ("splits", _I), ("kind", _I)]


class ConvUnpackDesc(ctypes.Structure):
    """retr_conv_unpack_desc"""
    _fields_ = [("ws", _P), ("scale", _P), ("grad", _P), ("Co", _I), ("Ci", _I), ("Cp", _I),
                ("KH", _I), ("KW", _I), ("splits", _I), ("accumulate", _I), ("pad", _I)]


class PosItem(ctypes.Structure):
    """retr_pos_item"""
    _fields_ = [("d", _P), ("ld", _L), ("M", _I), ("pad", _I)]


class LnOut(ctypes.Structure):
    """retr_ln_out"""
    _fields_ = [("gamma", _P), ("beta", _P), ("eps", _F), ("y_bf16", _I), ("y", _P), ("y2", _P),
                ("ldy", _L), ("pos", _P), ("period", _I), ("mean", _P), ("rstd", _P)]


class ConvPackDesc(ctypes.Structure):
    """retr_conv_pack_desc"""
    _fields_ = [("w", _P), ("bn_w", _P), ("bn_b", _P), ("bn_rm", _P), ("bn_rv", _P),
                ("conv_bias", _P), ("w_out", _P), ("wt_out", _P), ("bias_out", _P),
                ("scale_out", _P), ("Co", _I), ("Ci", _I), ("KH", _I), ("KW", _I), ("Cp", _I),
                ("pad", _I)]


class CatRowsDesc(ctypes.Structure):
    """retr_cat_rows_desc"""
    _fields_ = [("a", _P), ("b", _P), ("dst", _P), ("bias_a", _P), ("bias_b", _P),
                ("bias_dst", _P), ("rows", _I), ("ka", _I), ("kb", _I)]


class SlabSumDesc(ctypes.Structure):
    """retr_slab_sum_desc"""
    _fields_ = [("parts", _P), ("stride", _L), ("nparts", _I), ("cols", _I), ("dst", _P),
                ("accumulate", _I)]


_PFD = ctypes.POINTER(LinearFwdDesc)
_PDD = ctypes.POINTER(LinearDgradDesc)
_PWD = ctypes.POINTER(LinearWgradDesc)

# name -> argtypes (all functions return int unless listed in _RESTYPE)
_SIGS = {
    "retr_abi_version": [],
    "retr_last_error": [],
    "retr_set_seed_base": [_P],
    "retr_seed_bump": [_P, _U64, _P],
    "retr_spin_us": [_F, _P],
    "retr_linear_fwd": [_I, _P, _L, _P, _L, _P, _P, _L, _I, _I, _I, _I, _I, _P, _L, _F, _U64, _P],
    "retr_linear_dgrad": [_I, _P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _P, _I, _L, _P, _L, _I,
                          _P],
    "retr_transpose_cast": [_I, _P, _P, _I, _I, _I, _P],
    "retr_linear_splits": [_I, _I, _I, _I],
    "retr_ffn_splits": [_I, _I, _I],
    "retr_ffn_fwd": [_P, _L, _P, _P, _P, _P, _P, _L, _P, _L, _P, _L, _I, _I, _I, _F, _U64, _P,
                     _I, _P],
    "retr_ffn_bwd_data": [_P, _L, _P, _P, _L, _P, _P, _L, _P, _L, _I, _I, _I, _P, _I, _P],
    "retr_linear_fwd_splitk": [_I, _P, _L, _P, _L, _P, _P, _L, _I, _I, _I, _I, _I, _P, _L, _F,
                               _U64, _P, _I, _P],
    "retr_linear_fwd_splitk_ln": [_I, _P, _L, _P, _L, _P, _P, _L, _I, _I, _I, _I, _P, _L, _F,
                                  _U64, _P, _I, ctypes.POINTER(LnOut), _P],
    "retr_linear_dgrad_splitk": [_I, _P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _P, _I, _L, _P, _L,
                                 _I, _P, _I, _P],
    "retr_linear_dgrad_slabs": [_I, _P, _L, _P, _L, _I, _I, _I, _I, _P, _I, _P],
    "retr_linear_wgrad": [_I, _P, _L, _P, _L, _P, _L, _I, _I, _I, _P, _I, _P],
    "retr_bias_grad": [_I, _P, _L, _I, _I, _P, _P],
    "retr_linear_fwd_group": [_I, _I, _I, _PFD, _P],
    "retr_linear_dgrad_group": [_I, _I, _I, _I, _I, _PDD, _P],
    "retr_linear_wgrad_group_workspace": [_I, _PWD],
    "retr_linear_wgrad_group": [_I, _I, _PWD, _P, _P],
    "retr_linear_wgrad_group2": [_I, _I, _PWD, _P, _I, ctypes.POINTER(SlabSumDesc), _P],
    "retr_linear_wgrad_batch_table_bytes": [_I, _I],
    "retr_linear_wgrad_batch": [_I, _PWD, _I, ctypes.POINTER(SlabSumDesc), _P, _SZ, _P],
    "retr_conv_pack": [_I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P],
    "retr_conv_pack_group": [_I, _I, ctypes.POINTER(ConvPackDesc), _P],
    "retr_cat_rows_group": [_I, ctypes.POINTER(CatRowsDesc), _P],
    "retr_conv2d_fwd": [_I, _P, _I, _I, _I, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    "retr_conv2d_dgrad": [_I, _P, _I, _I, _I, _I, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P],
    "retr_conv2d_wgrad": [_I, _P, _P, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _I, _P],
    "retr_conv_wgrad_unpack": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    "retr_conv2d_wgrad_group_table_bytes": [_I],
    "retr_conv2d_wgrad_group_plan": [_I, _I, ctypes.POINTER(ConvWgradDesc)],
    "retr_conv2d_wgrad_group": [_I, _I, ctypes.POINTER(ConvWgradDesc), _P, _SZ, _P],
    "retr_conv_wgrad_unpack_group_table_bytes": [_I],
    "retr_conv_wgrad_unpack_group": [_I, ctypes.POINTER(ConvUnpackDesc), _P, _SZ, _P],
    "retr_conv2d_wgrad_splits": [_I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I],
    "retr_nchw_to_nhwc": [_I, _P, _P, _I, _I, _I, _I, _I, _P],
    "retr_nchw_to_s2d16": [_P, _P, _I, _I, _I, _I, _P],
    "retr_pipe_run": [_P, _P, _I, _P, _P, _P, _I, _P, _P, _P, _I, _P, _P, _P],
    "retr_stem_s2d_weights": [_P, _P, _I, _I, _P],
    "retr_conv2d_fwd_out": [_I, _P, _I, _I, _I, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I,
                            _I, _I, _P],
    "retr_bottleneck_s1_fwd": [_I, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P, _P],
    "retr_conv1x1_fwd_cat": [_I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _I,
                             _P],
    "retr_maxpool3x3s2": [_I, _P, _P, _I, _I, _I, _I, _I, _I, _P],
    "retr_stem_pool_fwd": [_I, _P, _I, _I, _I, _P, _P, _P, _I, _P],
    "retr_mask_nearest": [_P, _P, _I, _I, _I, _I, _I, _P],
    "retr_layernorm_fwd": [_I, _P, _L, _P, _P, _F, _I, _I, _P, _L, _P, _P, _I, _P, _P, _P],
    "retr_layernorm_bwd": [_I, _P, _P, _L, _P, _L, _P, _P, _P, _I, _I, _P, _L, _P, _P, _P, _P,
                           _P],
    "retr_layernorm_bwd_workspace": [_I, _I],
    "retr_layernorm_bwd2": [_I, _P, _P, _L, _P, _L, _P, _P, _P, _I, _I, _P, _L, _P, _P, _P, _P,
                            _P, _L, _F, _U64, _P, _P],
    "retr_layernorm_bwd_slabs": [_P, _I, _P, _L, _P, _P, _P, _I, _I, _P, _L, _P, _P, _P, _P, _P,
                                 _L, _F, _U64, _P, _P],
    "retr_embed_ln_fwd": [_P, _I, _I, _I, _P, _P, _P, _P, _F, _F, _U64, _P, _P, _P, _P],
    "retr_embed_ln_bwd": [_P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _F, _U64, _P, _P, _P, _P, _I,
                          _P, _P],
    "retr_embed_ln_bwd_workspace": [_I, _I, _I],
    "retr_set_deterministic": [_I],
    "retr_get_deterministic": [],
    "retr_tune": [_I, _I],
    "retr_attention_fwd": [_I, _P, _L, _P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _I, _P, _I, _F,
                           _U64, _P, _P, _P],
    "retr_attention_bwd": [_I, _P, _L, _P, _L, _P, _L, _P, _L, _P, _L, _P, _P, _L, _P, _L, _P,
                           _L, _I, _I, _I, _I, _I, _P, _I, _F, _U64, _P, _P],
    "retr_attention_bwd_workspace": [_I, _I, _I],
    "retr_attention_fwd_dm": [_I, _P, _L, _P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _I, _P, _I, _F,
                              _U64, _P, _P, _P, _P],
    "retr_attention_bwd_dm": [_I, _P, _L, _P, _L, _P, _L, _P, _L, _P, _L, _P, _P, _L, _P, _L,
                              _P, _L, _I, _I, _I, _I, _I, _P, _I, _F, _U64, _P, _P, _P],
    "retr_attention_dropout_mask_bytes": [_I, _I, _I, _I],
    "retr_attention_decode": [_I, _P, _L, _P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _I, _P, _I,
                              _P, _P],
    "retr_topk_rows": [_I, _P, _L, _I, _I, _I, _P, _P, _P],
    "retr_beam_select": [_P, _P, _I, _I, _I, _I, ctypes.c_longlong, _P, _P, _P, _P, _P, _P, _P,
                         _P],
    "retr_greedy_update": [_P, _I, _I, _I, ctypes.c_longlong, _P, _P, _P, _P, _P],
    "retr_ce_fwd": [_I, _P, _L, _I, _I, _P, _P, _P, _P, _P],
    "retr_ce_bwd": [_I, _P, _L, _I, _I, _P, _P, _P, _F, _P, _L, _P],
    "retr_ce_fwd_bwd": [_I, _P, _L, _I, _I, _P, _P, _P, _P, _F, _P, _L, _P],
    "retr_ce_bwd_rescale": [_I, _P, _L, _I, _I, _P, _P, _P, _F, _P, _L, _P],
    "retr_argmax_rows": [_I, _P, _L, _I, _I, _P, _P],
    "retr_argmax_workspace": [_I],
    "retr_argmax_rows_ws": [_I, _P, _L, _I, _I, _P, _P, _P],
    "retr_dropout_apply": [_I, _P, _L, _P, _L, _I, _I, _F, _U64, _P],
    "retr_cast": [_I, _P, _P, _L, _P],
    "retr_add_pos_fwd": [_I, _P, _L, _I, _I, _P, _I, _P, _P, _L, _P],
    "retr_sum2": [_I, _P, _P, _L, _P, _P],
    "retr_pos_grad": [_I, _P, _L, _I, _I, _I, _P, _P],
    "retr_pos_grad_set": [_I, _P, _L, _I, _I, _I, _P, _P],
    "retr_pos_grad_multi": [_I, _I, ctypes.POINTER(PosItem), _I, _I, _P, _I, _P],
    "retr_dec_gemm": [_P, _P, _I, _I, _P, _P, _I, _P, _L, _I, _P, _L, _I, _P, _L, _I, _I, _I, _P],
    "retr_dec_rows": [_P, _P, _I, _P, _I, _I, _P, _P, _P, _F, _P, _P, _P, _P],
    "retr_dec_embed_rows": [_P, _I, _I, _P, _P, _P, _P, _F, _P, _P, _P, _F, _P, _P, _P],
    "retr_greedy_select": [_I, _P, _L, _I, _I, _P, _I, _I, ctypes.c_longlong, _P, _P, _P, _P, _P,
                           _P],
    "retr_greedy_select2": [_I, _P, _L, _I, _I, _P, _I, _I, ctypes.c_longlong, _P, _P, _P, _P, _P,
                            _I, _P],
    "retr_dec_attn_row": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _F,
                          _P, _P, _P, _P, _P],
    "retr_dec_ffn": [_P, _I, _I, _P, _P, _P, _I, _P, _P],
    "retr_dec_ffn_ln": [_P, _P, _I, _P, _P, _P, _F, _P, _I, _I, _P, _P, _P, _I, _P, _P],
    "retr_dec_linear_bf16": [_P, _L, _P, _L, _P, _P, _L, _I, _I, _I, _I, _P],
    "retr_dec_linear_f32": [_P, _L, _P, _L, _P, _P, _L, _I, _I, _I, _I, _P, _L, _P],
    "retr_dec_linear3_f32": [_I, _P, _L, _P, _L, _P, _P, _L, _I, _I, _P, _L, _P, _L, _P, _L, _P, _P, _L, _I, _I, _P, _L, _P, _L, _P, _L, _P, _P, _L, _I, _I, _P, _L, _I, _I, _P],
    "retr_dec_self_f32": [_I, _I, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P,
                          _P, _P, _F, _P, _P, _F, _P, _P, _P],
    "retr_dec_cross_f32": [_I, _I, _I, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _P, _I, _I, _P,
                           _P, _P, _P],
    "retr_dec_ffn_f32": [_P, _P, _I, _P, _P, _P, _F, _P, _I, _I, _P, _P, _P, _I, _P, _P],
    "retr_dec_rows_f32": [_P, _P, _I, _P, _I, _I, _P, _P, _P, _F, _P, _P],
    "retr_dec_ffn_ln64": [_P, _P, _I, _P, _P, _P, _F, _P, _I, _I, _P, _P, _P, _I, _P, _P],
    "retr_dec_ffn_ln128": [_P, _P, _I, _P, _P, _P, _F, _P, _I, _I, _P, _P, _P, _I, _P, _P],
    "retr_dec_self_heads_ln": [_P, _P, _I, _I, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _I,
                               _P, _P, _P, _F, _P, _P, _P],
    "retr_dec_self_heads": [_P, _P, _I, _I, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P],
    "retr_dec_cross_heads": [_P, _P, _P, _P, _I, _I, _I, _P, _P, _F, _P, _P, _P, _P, _P, _I, _I,
                             _P, _P, _P, _P],
    "retr_dec_self_heads_embed": [_P, _P, _P, _P, _F, _I, _I, _I, _P, _P, _P, _P, _I, _I, _P,
                                  _P, _P, _P, _P, _F, _P, _P, _P],
    "retr_dec_self_heads_mr": [_P, _P, _I, _I, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _I,
                               _P, _P, _P, _F, _P, _P, _I, _P],
    "retr_dec_cross_heads_mr": [_P, _P, _P, _P, _I, _I, _I, _P, _P, _F, _P, _P, _P, _P, _P, _I, _I,
                                _P, _P, _P, _I, _P],
    "retr_adamw_sumsq": [_P, _L, _P, _I, _P, _P],
    "retr_adamw_update": [_P, _P, _P, _P, _L, _P, _D, _D, _F, _P, _F, _P, _I, _F, _P, _P],
    "retr_adamw_update2": [_P, _P, _P, _P, _L, _P, _D, _D, _F, _P, _F, _P, _I, _F, _P, _I, _P],
}
_RESTYPE = {"retr_last_error": ctypes.c_char_p, "retr_attention_bwd_workspace": _SZ,
            "retr_attention_dropout_mask_bytes": _SZ,
            "retr_layernorm_bwd_workspace": _SZ, "retr_embed_ln_bwd_workspace": _SZ,
            "retr_linear_wgrad_group_workspace": _SZ, "retr_linear_wgrad_batch_table_bytes": _SZ, "retr_conv2d_wgrad_group_table_bytes": _SZ, "retr_conv_wgrad_unpack_group_table_bytes": _SZ, "retr_argmax_workspace": _SZ,
            "retr_set_deterministic": None,
            "retr_set_seed_base": None}

_lib = None


def load():
    """Load the kernel library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"retr_amd: native library {LIB_PATH} is missing; build it with `make` "
                "(there is no CPU fallback)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, ctypes.c_int)
        # RETR_TUNE_<knob>=<value> in the environment presets a tuning knob (A/B runs)
        # (a malformed value or an unknown knob number is reported and skipped: it must not
        # break every import of the package)
        for k, v in os.environ.items():
            if k.startswith("RETR_TUNE_") and k[10:].isdigit():
                try:
                    val = int(v)
                except ValueError:
                    warnings.warn(f"retr_amd: ignoring {k}={v!r} (not an integer)")
                    continue
                if not 0 <= int(k[10:]) < TUNE_COUNT:
                    warnings.warn(f"retr_amd: ignoring {k}={v!r} (no tuning knob {k[10:]})")
                    continue
                lib.retr_tune(int(k[10:]), val)     # (returns the knob's previous value)
        _lib = lib
    return _lib


def exported_symbols():
    return list(_SIGS)


_probe = None


def set_probe(p):
    """Install (or remove with None) a retr_amd.probe.Probe that times selected calls."""
    global _probe
    _probe = p


def _raw_call(name, args):
    rc = getattr(load(), name)(*args)
    if rc is not None and rc != 0:   # void functions return None
        msg = load().retr_last_error()
        raise RuntimeError(f"{name} failed ({rc}): {msg.decode() if msg else ''}")


def call(name, *args):
    if _probe is not None and name in _probe.names:
        return _probe.wrap(name, args, lambda: _raw_call(name, args))
    _raw_call(name, args)


def ptr(t):
    """Device pointer of a tensor (or None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


def require_device(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("retr_amd ops run on the MI355X (HIP) device only; got a "
                               f"{t.device} tensor (no CPU fallback)")
