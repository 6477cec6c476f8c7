"""ctypes binding of libvqx.so (the C ABI declared in include/vqx.h).

The product path has no fallback: if the shared library is missing or was
built for another ABI, importing the ops raises.  Build it with
``python -m vae_npvc_amd.csrc.build`` (``__graft_entry__.build()`` does).

torch must be imported before the library is loaded so that libvqx.so binds
to the HIP runtime torch already loaded (same SONAME, one runtime per
process, shared streams and allocations).
"""
import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (loads the HIP runtime first; see module docstring)

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libvqx.so"
ABI_VERSION = 128  # include/vqx.h VQX_ABI_VERSION

VQX_F32, VQX_BF16 = 0, 1
PRO_NONE, PRO_LRELU, PRO_RELU, PRO_SCALE_RELU = 0, 1, 2, 3
(EPI_BIAS, EPI_ROWBIAS, EPI_MASK, EPI_RES, EPI_GNADD, EPI_SPLIT, EPI_OUTF32, EPI_ACT, EPI_ACT2, EPI_COLSUM, EPI_GNSTATS,
 EPI_GNBWD) = (1 << i for i in range(12))
CONV_TILE_ROWS = 128

c_void_p, c_int32, c_int64, c_float, c_double = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                                 ctypes.c_float, ctypes.c_double)


class ConvArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("w", c_void_p), ("y", c_void_p), ("bias", c_void_p), ("rowbias", c_void_p),
        ("res", c_void_p), ("mask", c_void_p), ("gn_h", c_void_p), ("gn_mean_rstd", c_void_p),
        ("gn_gamma", c_void_p), ("gn_beta", c_void_p), ("out2", c_void_p),
        ("n_rows", c_int64), ("T", c_int32), ("cin", c_int32), ("cout", c_int32), ("ntaps", c_int32),
        ("pad", c_int32), ("ldx", c_int32), ("ldy", c_int32), ("ldres", c_int32), ("ldmask", c_int32),
        ("ldgn", c_int32), ("ldo2", c_int32), ("dtype", c_int32), ("prologue", c_int32),
        ("epilogue", c_int32), ("split_col", c_int32), ("out2_accumulate", c_int32),
        ("pro_scale", c_float), ("mask_slope", c_float), ("mask_scale", c_float),
        ("y2", c_void_p), ("ldy2", c_int32), ("epi_act", c_int32), ("colsum_part", c_void_p),
        ("stat_part", c_void_p), ("gn_groups", c_int32), ("gn_glu", c_int32),
        ("gn_stat_tiles", c_void_p), ("gn_eps", c_float), ("dil", c_int32), ("kernel_policy", c_int32),
    ]


class WgradArgs(ctypes.Structure):
    _fields_ = [
        ("p", c_void_p), ("q", c_void_p), ("slabs", c_void_p), ("n_rows", c_int64), ("T", c_int32),
        ("r_dim", c_int32), ("c_dim", c_int32), ("ntaps", c_int32), ("pad", c_int32),
        ("shift_sign", c_int32), ("ldp", c_int32), ("ldq", c_int32), ("dtype", c_int32),
        ("q_prologue", c_int32), ("splits", c_int32), ("pro_scale", c_float), ("dil", c_int32),
        ("slab_dtype", c_int32), ("kernel_policy", c_int32), ("fixup_dw", c_void_p), ("fixup_counters", c_void_p),
    ]


class WNLayer(ctypes.Structure):
    _fields_ = [
        ("v", c_void_p), ("g", c_void_p), ("w_packed", c_void_p), ("norm", c_void_p), ("dv", c_void_p),
        ("dg", c_void_p), ("slabs", c_void_p), ("kind", c_int32), ("cout", c_int32), ("cin", c_int32),
        ("k", c_int32), ("splits", c_int32), ("dtype", c_int32), ("stride", c_int32), ("pad", c_int32),
        ("slab_dtype", c_int32),
    ]


class LinearLayer(ctypes.Structure):
    _fields_ = [("W", c_void_p), ("bias", c_void_p), ("out", c_void_p), ("dout", c_void_p), ("dW", c_void_p),
                ("dbias", c_void_p)]


class StepClose(ctypes.Structure):  # include/vqx.h vqx_step_close
    _fields_ = [("parts", c_void_p * 2), ("n", c_int32 * 2), ("scale", c_float * 2), ("out", c_void_p * 2),
                ("pub_src", c_void_p), ("pub_n", c_int32), ("pub_copy", c_void_p), ("pub_box", c_void_p),
                ("pub_slot", c_int32), ("pub_slots", c_int32), ("pub_floats", c_int32), ("pub_seq", ctypes.c_uint32),
                ("rows_src", c_void_p), ("rows_ld", c_int32), ("n_rows", c_int32), ("rows_host", c_void_p)]


WN_COLREDUCE = 2
WN_RESAMPLE, WN_RESAMPLE_T = 3, 4  # strided Conv1d / ConvTranspose1d (include/vqx.h)

# name -> argtypes (restype is int for every entry point except the two below)
_SIGS = {
    "vqx_conv1d_fwd": [ctypes.POINTER(ConvArgs), c_void_p],
    "vqx_conv1d_dgrad": [ctypes.POINTER(ConvArgs), c_void_p],
    "vqx_conv1d_wgrad": [ctypes.POINTER(WgradArgs), c_void_p],
    "vqx_conv1d_dgrad_wgrad": [ctypes.POINTER(ConvArgs), ctypes.POINTER(WgradArgs), ctypes.POINTER(ctypes.c_int32),
                               c_void_p],
    "vqx_weight_norm_fwd": [c_void_p, c_void_p, c_int32, c_void_p],
    "vqx_weight_norm_bwd": [c_void_p, c_void_p, c_int32, c_void_p],
    "vqx_weight_norm_fwd_flags": [c_void_p, c_void_p, c_int32, c_int32, c_void_p],
    "vqx_adam_step_wn": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_float, c_void_p,
                         c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_void_p],
    "vqx_weight_norm_bwd_partials": [c_void_p, c_int32, c_void_p],
    "vqx_weight_norm_bwd_sq": [c_void_p, c_void_p, c_int32, c_void_p, c_int64, c_void_p],
    "vqx_sq_norm_finish": [c_void_p, c_int64, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p],
    "vqx_sq_norm_finish_adam": [c_void_p, c_int64, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p,
                                c_double, c_double, c_int32, c_double, c_double, c_double, c_void_p, c_void_p],
    "vqx_groupnorm_stats": [c_void_p, c_int32, c_int32, c_int64, c_int32, c_int32, c_int32, c_float, c_void_p,
                            c_void_p, c_void_p],
    "vqx_gn_lrelu_fwd": [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_int64, c_int32, c_int32, c_void_p,
                         c_void_p, c_void_p, c_void_p],
    "vqx_gn_glu_fwd": [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_int64, c_int32, c_int32, c_void_p,
                       c_void_p, c_void_p, c_void_p],
    "vqx_gn_glu_fwd_tiles": [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_int64, c_int32, c_int32, c_void_p,
                             c_float, c_void_p, c_void_p, c_void_p, c_void_p],
    "vqx_gn_bwd": [c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_int32, c_int32, c_int64, c_int32, c_int32,
                   c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p,
                   c_void_p],
    "vqx_gn_finalize_tiles": [c_void_p, c_int64, c_int32, c_int32, c_int32, c_float, c_void_p, c_void_p],
    "vqx_colsum": [c_void_p, c_int32, c_int32, c_int64, c_int32, c_void_p, c_void_p, c_int32, c_void_p],
    "vqx_colsum_parts": [c_int64, c_int32, c_int32, c_void_p],
    "vqx_colsum_partials": [c_void_p, c_int32, c_int32, c_int64, c_int32, c_void_p, c_void_p],
    "vqx_nct_to_ntc": [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_int32, c_int32, c_void_p],
    "vqx_ntc_to_nct": [c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p],
    "vqx_logloss_fwd_bwd": [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_float, c_void_p, c_int32,
                            c_int32, c_void_p, c_void_p, c_void_p],
    "vqx_logloss_fwd_bwd_x": [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_float, c_void_p, c_int32,
                              c_int32, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p],
    "vqx_logloss_parts": [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_float, c_void_p, c_int32, c_int32,
                          c_void_p, c_void_p, c_void_p],
    "vqx_vq_forward": [c_void_p, c_int64, c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_int32,
                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "vqx_vq_workspace": [c_int64, c_int32, c_int32, c_int32, c_void_p],
    "vqx_vq_stats": [c_void_p, c_int64, c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p],
    "vqx_vq_ema_update": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_float,
                          c_float, c_void_p, c_void_p, c_void_p],
    "vqx_vq_ema_update_clear": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_float,
                                c_float, c_void_p, c_void_p, c_void_p],
    "vqx_vq_ema_update_close": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_float,
                                c_float, c_void_p, c_void_p, c_void_p, c_void_p],
    "vqx_gather_rows": [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_void_p, c_void_p],
    "vqx_gather_rows_host": [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_void_p, c_void_p],
    "vqx_vq_commit_bwd": [c_void_p, c_void_p, c_int64, c_float, c_void_p, c_int32, c_void_p],
    "vqx_vq_commit_bwd_cs": [c_void_p, c_void_p, c_int64, c_int32, c_float, c_void_p, c_int32, c_void_p, c_void_p],
    "vqx_time_gather": [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_int32, c_void_p],
    "vqx_embedding_fwd": [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p],
    "vqx_embedding_bwd": [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p],
    "vqx_embedding_bwd_rows": [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_int32, c_void_p],
    "vqx_linear_f32": [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p],
    "vqx_linear_bwd_f32": [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p],
    "vqx_grad_sq_norm": [c_void_p, c_int64, c_void_p, c_void_p, c_void_p],
    "vqx_adam_hyper": [c_void_p, c_double, c_double, c_int32, c_double, c_double, c_double, c_void_p, c_void_p],
    "vqx_linear_batched_fwd": [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_int32, c_void_p],
    "vqx_linear_batched_bwd": [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p],
    "vqx_linear_batched_fwd_ids": [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p],
    "vqx_step_prologue": [c_void_p, c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32,
                          c_int32, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_int32, c_int32, c_void_p],
    "vqx_linear_batched_bwd_ids": [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p,
                                   c_void_p, c_void_p],
    "vqx_wgrad_tiles": [c_int64, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                        ctypes.POINTER(c_int32)],
    "vqx_wgrad_fixup_ok": [c_int64, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                           c_int32, ctypes.POINTER(c_int32)],
    "vqx_vq_normalize": [c_void_p, c_int64, c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_void_p],
    "vqx_vq_perplexity": [c_void_p, c_int32, c_int64, c_void_p, c_void_p],
    "vqx_vq_plain_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int64, c_int32,
                         c_int32, c_float, c_float, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_int32, c_void_p, c_void_p],
    "vqx_stream_create_cu_mask": [c_int32, ctypes.POINTER(c_void_p), ctypes.POINTER(c_int32)],
    "vqx_mailbox_create": [c_int32, c_int32, ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p)],
    "vqx_mailbox_destroy": [c_void_p],
    "vqx_mailbox_publish": [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32, c_int32, ctypes.c_uint32,
                            c_void_p],
    "vqx_stream_destroy": [c_void_p],
    "vqx_probe_enable": [c_int32],
    "vqx_probe_select": [c_void_p],
    "vqx_probe_clear": [],
    "vqx_probe_count": [ctypes.POINTER(c_int64)],
    "vqx_probe_read": [c_int64, ctypes.POINTER(c_int32), ctypes.POINTER(c_double), ctypes.POINTER(c_float)],
    "vqx_scale_act_2d": [c_void_p, c_int32, c_int32, c_void_p, c_int32, c_int32, c_int64, c_int32, c_float, c_int32,
                         c_void_p],
    "vqx_convert_2d": [c_void_p, c_int32, c_int32, c_void_p, c_int32, c_int32, c_int64, c_int32, c_void_p],
    "vqx_convert_2d_zero2": [c_void_p, c_int32, c_int32, c_void_p, c_int32, c_int32, c_int64, c_int32, c_void_p,
                             c_int32, c_int64, c_int32, c_void_p],
    "vqx_adam_step": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_float, c_void_p],
    "vqx_radam_hyper": [c_void_p, c_double, c_double, c_int32, c_double, c_double, c_double, c_void_p, c_void_p],
    "vqx_radam_step": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_float, c_void_p],
}
EXPORTS = tuple(_SIGS) + ("vqx_last_error", "vqx_version")


class VqxError(RuntimeError):
    pass


_lib = None


def load(path: os.PathLike = None):
    """Load libvqx.so once (env VQX_LIB overrides the in-tree path, for A/B
    builds); raise if it is absent (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(path or os.environ.get("VQX_LIB") or LIB_PATH)
    if not path.exists():
        raise VqxError(f"libvqx.so not found at {path}; build it with `python -m vae_npvc_amd.csrc.build` "
                       "(the HIP kernels are the only implementation of this path)")
    lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
    for name, argtypes in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    lib.vqx_last_error.restype = ctypes.c_char_p
    lib.vqx_last_error.argtypes = []
    lib.vqx_version.restype = ctypes.c_int
    lib.vqx_version.argtypes = []
    if lib.vqx_version() != ABI_VERSION:
        raise VqxError(f"libvqx ABI {lib.vqx_version()} != expected {ABI_VERSION}; rebuild")
    _lib = lib
    return lib


_post_call = None  # debug.py's guard check (EngineOptions.debug_checks); None in normal runs


def set_post_call(fn):
    """fn(name) after every successful entry point (None removes it)."""
    global _post_call
    _post_call = fn


def call(name: str, *args):
    """Invoke an entry point and turn a non-zero status into VqxError."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise VqxError(f"{name} failed ({rc}): {lib.vqx_last_error().decode(errors='replace')}")
    if _post_call is not None:
        _post_call(name)
    return rc


def stream_ptr() -> int:
    """hipStream_t of torch's current stream on the current device."""
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()
