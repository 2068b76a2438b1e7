"""ctypes binding of libzonos_hip.so (the C ABI declared in include/zonos_hip.h).

The library is built in-tree (zonos_vibes_amd/build.py). There is no fallback: if the
shared object is missing or a call fails, a RuntimeError is raised.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# ZMI_LIB_PATH selects a diagnostic build (tools/stamps.py); the product path is libzonos_hip.so
LIB_PATH = os.environ.get("ZMI_LIB_PATH") or os.path.join(HERE, "libzonos_hip.so")

c_int, c_int64, c_float, c_void_p, c_uint64 = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, \
    ctypes.c_uint64
c_int_p = ctypes.POINTER(ctypes.c_int)

EPI_STORE, EPI_RESIDUAL, EPI_QKV, EPI_SWIGLU, EPI_LOGITS, EPI_F32 = range(6)
OPT_GEMV_SPREAD = 0  # zmi_set_option knobs
OPT_GEMM_ROWS = 1
OPT_XC_HANDOFF = 2  # 0: chunk-split attention hand-offs through the XCD's L2; 1: write-through
# 3..9: reserved (the removed diagnostic forms' knobs)
OPT_DAC_WIDE = 10
OPT_DAC_WIDE_MIN = 11
OPT_ATTNBLK_SPREAD = 12
OPT_DAC_STAGE = 13
OPT_DAC_STAGE_MIN = 14
OPT_SCAN_PQ = 15
OPT_SPLITK_WGS = 16
OPT_SPLITK_STAGE = 17
ATTNBLK_SELF, ATTNBLK_SPLIT = 256, 512  # zmi_attn_block slices flags: self-scoring / chunk-split forms
PACK_IDENTITY, PACK_SWIGLU = 0, 1
PRO_AUTO, PRO_ADDLN, PRO_GRMS, PRO_GRMS_G = 0, 2, 3, 4


class GemvArgs(ctypes.Structure):
    _fields_ = [
        ("W", c_void_p), ("X", c_void_p),
        ("M", c_int), ("N", c_int), ("K", c_int), ("ldx", c_int),
        ("groups", c_int), ("reserved", c_int),
        ("ln_w", c_void_p), ("ln_b", c_void_p), ("eps", c_float),
        ("out", c_void_p), ("ldo", c_int), ("n_valid", c_int),
        ("row_kv", c_void_p), ("row_pos", c_void_p),
        ("k_cache", c_void_p), ("v_cache", c_void_p),
        ("smax", c_int), ("hq", c_int), ("hkv", c_int), ("hd", c_int),
        ("rope", c_void_p), ("diag", c_void_p),
        ("pro", c_int), ("ld_aux", c_int), ("aux", c_void_p), ("res_out", c_void_p),
    ]


class Prefetch(ctypes.Structure):
    _fields_ = [("ptr", c_void_p * 2), ("bytes", c_int64 * 2), ("sink", c_void_p), ("blocks", c_int),
                ("reserved", c_int)]


class Sampling(ctypes.Structure):
    _fields_ = [
        ("temperature", c_float), ("top_p", c_float), ("min_p", c_float), ("linear", c_float),
        ("conf", c_float), ("quad", c_float), ("rep_penalty", c_float), ("cfg_scale", c_float),
        ("top_k", c_int), ("rep_window", c_int), ("seed", c_uint64),
    ]


class Slots(ctypes.Structure):
    _fields_ = [
        ("active", c_void_p), ("pos", c_void_p), ("offset", c_void_p), ("remaining", c_void_p),
        ("stopping", c_void_p), ("step", c_void_p), ("delayed", c_void_p), ("params", c_void_p),
        ("total_len", c_void_p), ("tcap", c_int), ("n_slots", c_int),
    ]


class CondParam(ctypes.Structure):
    _fields_ = [("table", c_void_p), ("weight", c_void_p), ("bias", c_void_p), ("in_dim", c_int), ("pad", c_int),
                ("min_val", c_float), ("max_val", c_float)]


class CondRow(ctypes.Structure):
    _fields_ = [("param", c_int), ("kind", c_int), ("index", c_int), ("x_off", c_int)]


class Mamba2Args(ctypes.Structure):
    _fields_ = [
        ("zxbcdt", c_void_p), ("ld_zx", c_int), ("M", c_int),
        ("d_ssm", c_int), ("nheads", c_int), ("headdim", c_int), ("d_state", c_int), ("d_conv", c_int),
        ("ngroups", c_int),
        ("conv_w", c_void_p), ("conv_b", c_void_p), ("dt_bias", c_void_p), ("A", c_void_p), ("D", c_void_p),
        ("conv_ring", c_void_p), ("ssm", c_void_p), ("y", c_void_p), ("ldy", c_int), ("gz_g", c_int),
        ("row_pos", c_void_p), ("row_kv", c_void_p), ("gz", c_void_p),
    ]


COND_EMBED, COND_VECTOR, COND_FOURIER, COND_LINEAR, COND_PASSTHROUGH = range(5)


_SIGS = {
    "zmi_pack_weight": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "zmi_gemv_launch": (c_int, [ctypes.POINTER(GemvArgs), c_int, c_void_p]),
    "zmi_layernorm_rows": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_int,
                                   c_void_p]),
    "zmi_attention": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                              c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "zmi_attention_variant": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                      c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                      c_void_p]),
    "zmi_attention_pf": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                 c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                 ctypes.POINTER(Prefetch), c_void_p]),
    "zmi_attention_max_keys_whole": (c_int, []),
    "zmi_attention_pick": (c_int, [c_int, c_int, c_int]),
    "zmi_attn_block_max_pos": (c_int, [c_int]),
    "zmi_attn_block": (c_int, [ctypes.POINTER(GemvArgs), c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "zmi_attn_block_gran_words": (c_int64, [c_int, c_int]),
    "zmi_gemv_splitk": (c_int, [ctypes.POINTER(GemvArgs), c_int, c_void_p, c_int64, c_void_p]),
    "zmi_gemv_splitk_floats": (c_int64, [c_int, c_int]),
    "zmi_gemv_splitk_ln": (c_int, [ctypes.POINTER(GemvArgs), c_int, c_void_p, c_int64, c_void_p, c_void_p, c_float,
                                   c_void_p, c_int, c_void_p]),
    "zmi_attn_block_pf": (c_int, [ctypes.POINTER(GemvArgs), c_void_p, c_void_p, c_void_p, c_int, c_int,
                                  ctypes.POINTER(Prefetch), c_void_p]),
    "zmi_attn_block_oproj": (c_int, [ctypes.POINTER(GemvArgs), ctypes.POINTER(GemvArgs), c_void_p, c_void_p, c_void_p,
                                     c_int, c_int, ctypes.POINTER(Prefetch), c_void_p]),
    "zmi_attention_work_bytes": (c_int64, [c_int, c_int, c_int, c_int, c_int]),
    "zmi_attention_partial_floats": (c_int64, [c_int, c_int, c_int, c_int, c_int]),
    "zmi_attention_chunk": (c_int, []),
    "zmi_sample_step": (c_int, [ctypes.POINTER(Slots), c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "zmi_sample_step_greedy": (c_int, [ctypes.POINTER(Slots), c_void_p, c_void_p, c_int, c_int, c_void_p, c_int,
                                       c_void_p, c_void_p, c_void_p, c_void_p]),
    "zmi_sample_logits": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "zmi_apply_delay_pattern": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int64, c_void_p]),
    "zmi_revert_delay_pattern": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "zmi_embed_step": (c_int, [ctypes.POINTER(Slots), c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "zmi_embed_codes": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "zmi_delay_init": (c_int, [ctypes.POINTER(Slots), c_int, c_void_p, c_int, c_int, c_void_p]),
    "zmi_delay_revert": (c_int, [ctypes.POINTER(Slots), c_int, c_void_p, c_int, c_void_p]),
    "zmi_dac_from_codes": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "zmi_dac_conv": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                             c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "zmi_dac_im2col7": (c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    "zmi_dac_vq": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_void_p]),
    "zmi_dac_conv_t": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                c_void_p, c_void_p]),
    "zmi_dac_conv_out": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "zmi_prefix_condition": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_float,
                                     c_void_p, c_void_p]),
    "zmi_mamba2_step": (c_int, [ctypes.POINTER(Mamba2Args), c_void_p]),
    "zmi_mamba2_scan": (c_int, [ctypes.POINTER(Mamba2Args), c_int, c_void_p]),
    "zmi_mamba2_scan_ws": (c_int, [ctypes.POINTER(Mamba2Args), c_int, c_void_p, ctypes.c_int64, c_void_p]),
    "zmi_mamba2_scan_ws_bytes": (ctypes.c_int64, [c_int, c_int, c_int]),
    "zmi_add_layernorm": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_float,
                                  c_void_p, c_int, c_int, c_void_p]),
    "zmi_mamba_block": (c_int, [ctypes.POINTER(GemvArgs), ctypes.POINTER(Mamba2Args), c_void_p, c_void_p, c_void_p]),
    "zmi_mamba_block_pf": (c_int, [ctypes.POINTER(GemvArgs), ctypes.POINTER(Mamba2Args), c_void_p, c_void_p,
                                   ctypes.POINTER(Prefetch), c_void_p]),
    "zmi_mamba_block_gran_words": (c_int64, [c_int, c_int]),
    "zmi_gated_rmsnorm": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_float, c_void_p, c_int,
                                  c_void_p]),
    "zmi_fill_uniform": (c_int, [c_void_p, c_int64, c_uint64, c_float, c_float, c_int, c_void_p]),
    "zmi_graph_begin": (c_int, [c_void_p]),
    "zmi_graph_end": (c_int, [c_void_p, ctypes.POINTER(c_void_p)]),
    "zmi_graph_launch": (c_int, [c_void_p, c_int, c_void_p]),
    "zmi_graph_destroy": (c_int, [c_void_p]),
    "zmi_last_error": (ctypes.c_char_p, []),
    "zmi_version": (c_int, []),
    "zmi_xcd_dealing": (c_int, [c_void_p]),
    "zmi_set_option": (c_int, [c_int, c_int]),
    "zmi_get_option": (c_int, [c_int]),
}

EXPORTED = sorted(_SIGS)
_lib = None
ABI_VERSION = 6  # zmi_version() of the library this binding (and its weight packers) is written for


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load the library (torch is imported first so its HIP runtime is the one in use)."""
    import torch  # noqa: F401  -- libamdhip64.so.7 from torch must be resident before the dlopen
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `python -m zonos_vibes_amd.build` "
                           "(the HIP path has no CPU fallback)")
    lib_ = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib_, name)
        fn.restype = res
        fn.argtypes = args
    if lib_.zmi_version() != ABI_VERSION:  # weight layouts and option meanings change with the version
        raise RuntimeError(f"{path} has ABI version {lib_.zmi_version()}, this binding expects {ABI_VERSION}: rebuild it")
    return lib_


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        _lib = load()
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().zmi_last_error().decode(errors="replace")
        raise RuntimeError(f"libzonos_hip {what} failed (status {rc}): {msg}")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None for None)."""
    return None if t is None else t.data_ptr()
