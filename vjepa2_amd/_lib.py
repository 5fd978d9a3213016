"""ctypes binding of libvjepa_hip.so (include/vjepa_hip.h).

The product path has no CPU fallback: if the library is missing or a call fails, a RuntimeError
is raised. PyTorch is imported first so that its HIP runtime (libamdhip64.so.7) is the one the
library binds to.
"""

import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime our library links against)

# VJ_LIB: an alternative build of the same library (A/B timing of kernel variants, tools/)
LIB_PATH = os.environ.get("VJ_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libvjepa_hip.so")

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float
_U = ctypes.c_uint

# name -> argtypes (restype is always int)
SIGNATURES = {
    "vj_version": [],
    "vj_header_crc": [],
    "vj_get_last_error": [ctypes.c_char_p, ctypes.c_size_t],
    "vj_device_sync": [],
    "vj_gemm_bf16": [_I, _I, _I, _P, _L, _I, _P, _L, _I, _I, _P, _P, _L, _P, _L, _P, _L, _P],
    "vj_gemm_bf16_splitk": [_I, _I, _I, _P, _L, _I, _P, _L, _I, _I, _P, _P, _L, _P, _L, _P, _L, _I, _P, _L, _P],
    "vj_gemm_bf16_wgrad": [_I, _I, _I, _P, _L, _P, _L, _P, _L, _I, _P, _I, _I, _P, _L, _P],
    "vj_attn_fwd": [_I, _I, _I, _P, _L, _I, _I, _I, _P, _L, _P, _F, _I, _P, _P, _P],
    "vj_attn_bwd": [_I, _I, _I, _P, _L, _I, _I, _I, _P, _L, _P, _L, _P, _P, _L, _F, _I, _P, _P, _P, _I, _I, _I, _P,
                    _P, _P],
    "vj_attn_fwd_fc": [_I, _I, _I, _P, _L, _I, _I, _I, _P, _L, _P, _F, _I, _P, _P, _I, _P],
    "vj_attn_bwd_fc": [_I, _I, _I, _P, _L, _I, _I, _I, _P, _L, _P, _L, _P, _P, _L, _F, _I, _P, _P, _P, _I, _I, _I, _P,
                       _P, _I, _P],
    "vj_attn_fwd_ex": [_I, _I, _I, _P, _L, _I, _I, _I, _P, _L, _P, _F, _I, _P, _P, _I, _F, _U, _P],
    "vj_attn_bwd_ex": [_I, _I, _I, _P, _L, _I, _I, _I, _P, _L, _P, _L, _P, _P, _L, _F, _I, _P, _P, _P, _I, _I, _I, _P,
                       _P, _I, _F, _U, _P],
    "vj_qkv_rope_gemm": [_I, _I, _P, _L, _P, _L, _P, _P, _L, _I, _I, _P, _I, _I, _I, _P, _P, _I, _P],
    "vj_layernorm_fwd": [_I, _I, _P, _I, _L, _P, _P, _F, _P, _I, _L, _P, _P, _P],
    "vj_gemm_fp8": [_I, _I, _I, _P, _L, _P, _P, _L, _P, _I, _P, _P, _L, _P, _L, _P, _L, _P],
    "vj_qkv_rope_gemm_fp8": [_I, _I, _P, _L, _P, _P, _L, _P, _P, _P, _L, _I, _I, _P, _I, _I, _I, _P, _P, _I, _P],
    "vj_quant_rows_fp8": [_I, _I, _P, _I, _L, _P, _L, _P, _P],
    "vj_layernorm_fwd_fp8": [_I, _I, _P, _I, _L, _P, _P, _F, _P, _L, _P, _P, _P, _P],
    "vj_video_transform": [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P],
    "vj_mask_count": [_I, _I, _I, _I, _I, _P, _I, _I, _I, _I, _P, _P],
    "vj_mask_emit": [_I, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P],
    "vj_gemm_f32": [_I, _I, _I, _P, _L, _P, _L, _I, _P, _P, _L, _P, _L, _P, _L, _P],
    "vj_attn_fwd_f32": [_I, _I, _I, _P, _L, _I, _I, _I, _P, _L, _P, _F, _I, _P, _P, _P],
    "vj_rope_f32": [_I, _I, _I, _P, _L, _I, _I, _P, _I, _I, _I, _P, _P, _I, _P],
    "vj_im2col_tubelet_f32": [_I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P],
    "vj_layernorm_bwd_blocks": [_I],
    "vj_layernorm_bwd": [_I, _I, _P, _L, _P, _L, _P, _P, _P, _P, _L, _P, _L, _P, _L, _P, _P, _P, _P, _P, _L, _P],
    "vj_gelu_eval": [_I, _P, _P, _P, _P],
    "vj_layernorm_bwd_bf16": [_I, _I, _P, _L, _P, _L, _P, _P, _P, _P, _L, _P, _L, _P, _P, _P, _P, _P, _L, _P],
    "vj_colsum_f32": [_I, _I, _P, _I, _L, _P, _I, _P, _L, _P],
    "vj_rope": [_I, _I, _I, _P, _L, _I, _I, _P, _I, _I, _I, _P, _P, _I, _I, _P],
    "vj_im2col_tubelet": [_I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P],
    "vj_gather_rows": [_I, _I, _P, _L, _P, _P, _L, _I, _P],
    "vj_fill_rows": [_I, _I, _P, _L, _P, _P, _P],
    "vj_add_rows": [_I, _I, _P, _L, _P, _L, _I, _P, _I, _P],
    "vj_pred_index": [_I, _I, _I, _P, _P, _I, _I, _I, _P, _P, _P, _P, _P],
    "vj_ids64to32": [_L, _P, _P, _P],
    "vj_jepa_loss": [_I, _I, _P, _I, _L, _P, _I, _L, _P, _P, _P, _F, _F, _F, _I, _P, _F, _P, _L, _P, _P, _P],
    "vj_check_finite": [_L, _P, _P, _P],
    "vj_adamw": [_L, _P, _P, _P, _P, _P, _F, _F, _F, _F, _F, _I, _F, _P, _P],
    "vj_ema": [_L, _P, _P, _F, _P, _P],
    "vj_adamw_ema": [_L, _P, _P, _P, _P, _P, _F, _F, _F, _F, _F, _I, _F, _P, _P, _P, _F, _P],
    "vj_cast_bf16": [_L, _P, _P, _P],
    "vj_proxy_copy": [_P, _P, _L, _I, _I, _P],
    "vj_set_reserved_cus": [_I],
    "vj_transpose_bf16": [_I, _I, _P, _L, _P, _L, _P],
    "vj_transpose_bf16_batch": [_I, _P, _L, _P],
    "vj_swiglu_fwd": [_I, _I, _P, _L, _P, _L, _P],
    "vj_swiglu_bwd": [_I, _I, _P, _L, _P, _L, _P, _L, _P],
    "vj_rowscale_add": [_I, _I, _P, _L, _P, _P, _L, _P, _L, _I, _P],
    "vj_rowscale_bf16": [_I, _I, _P, _L, _P, _P, _L, _P],
    "vj_dropout": [_I, _I, _P, _L, _I, _P, _L, _P, _L, _I, _P, _L, _F, _U, _P],
    "vj_xattn_ws_floats": [_I, _I, _I, _I, _I, ctypes.POINTER(_L)],
    "vj_xattn_fwd": [_I, _I, _I, _I, _I, _P, _L, _P, _L, _P, _L, _P, _F, _P, _L, _P],
    "vj_xattn_bwd": [_I, _I, _I, _I, _I, _P, _L, _P, _L, _P, _L, _P, _L, _P, _F, _P, _L, _P, _L, _P, _L, _P],
}

_lib = None


def load():
    """Load and type the library (raises if it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} not found: the HIP extension is not built (run `python -m vjepa2_amd.build` or "
            "__graft_entry__.build()). There is no CPU fallback."
        )
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if os.environ.get("VJ_LIB"):  # an older build selected for an A/B run: its own symbol set
                continue
            raise RuntimeError(f"{LIB_PATH} does not export {name}: stale build (rebuild the extension)")
        fn.argtypes = args
        fn.restype = ctypes.c_int
    if not os.environ.get("VJ_LIB"):  # A/B builds of older trees carry their own header
        import zlib

        hdr = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "vjepa_hip.h")
        crc_fn = getattr(lib, "vj_header_crc", None)
        if crc_fn is None:
            raise RuntimeError(f"{LIB_PATH} predates vj_header_crc: stale build (rebuild the extension)")
        with open(hdr, "rb") as f:
            want = zlib.crc32(f.read()) & 0xFFFFFFFF
        got = crc_fn() & 0xFFFFFFFF
        if got != want:
            raise RuntimeError(f"{LIB_PATH} was built from another include/vjepa_hip.h (crc {got:08x}, "
                               f"header {want:08x}): stale build (rebuild the extension)")
    _lib = lib
    return lib


def last_error():
    buf = ctypes.create_string_buffer(1024)
    load().vj_get_last_error(buf, 1024)
    return buf.value.decode(errors="replace")


def call(name, *args):
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed (code {rc}): {last_error()}")
    return rc


def int_array(vals):
    vals = list(vals)
    return (ctypes.c_int * max(1, len(vals)))(*vals)
