"""ctypes binding of libvcf_amd.so (include/vcf_amd.h).

There is deliberately no CPU fallback: if the HIP library is missing or fails
to load, every entry point raises.  The oracle under oracle/ is test
infrastructure and is never imported from here.
"""
from __future__ import annotations

import ctypes
import os
import threading

from . import _build

VCF_OK = 0
VCF_ERR_INVALID = -1
VCF_ERR_HIP = -2
VCF_ERR_UNSUPPORTED = -3
VCF_ERR_TIMEOUT = -4

VCF_DTYPE_F32 = 0
VCF_DTYPE_F64 = 1
VCF_DTYPE_I16 = 2
VCF_DTYPE_I32 = 3
VCF_DTYPE_U8 = 4
VCF_DTYPE_U16 = 5

VCF_DCT_NO_SUBBANDS = 1
VCF_DCT_PERCEPTUAL = 2


class VCFError(RuntimeError):
    """A libvcf_amd call failed (status < 0)."""

    def __init__(self, status: int, message: str):
        super().__init__(f"[vcf status {status}] {message}")
        self.status = status


class VCFInvalidArgument(VCFError, ValueError):
    """VCF_ERR_INVALID: the reference raises ValueError in the same cases."""


class VCFUnsupported(VCFError, NotImplementedError):
    pass


class VCFTimeout(VCFError, TimeoutError):
    """VCF_ERR_TIMEOUT: a cross-rank exchange did not finish in time (the
    RCCL communicator has been aborted)."""


_P = ctypes.c_void_p
_SZ = ctypes.c_size_t
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_U32 = ctypes.c_uint32
_PI32 = ctypes.POINTER(ctypes.c_int32)
_PI = ctypes.POINTER(ctypes.c_int)

# name -> argtypes (restype is int for all but vcf_last_error and the *_bound functions)
SIGNATURES = {
    "vcf_version": [_PI, _PI],
    "vcf_device_count": [_PI],
    "vcf_set_device": [ctypes.c_int],
    "vcf_get_device": [_PI],
    "vcf_device_sync": [],
    "vcf_malloc": [ctypes.POINTER(_P), _SZ],
    "vcf_free": [_P],
    "vcf_host_alloc": [ctypes.POINTER(_P), _SZ],
    "vcf_host_free": [_P],
    "vcf_memcpy_htod": [_P, _P, _SZ, _P],
    "vcf_memcpy_dtoh": [_P, _P, _SZ, _P],
    "vcf_memcpy_dtod": [_P, _P, _SZ, _P],
    "vcf_memset": [_P, ctypes.c_int, _SZ, _P],
    "vcf_stream_create": [ctypes.POINTER(_P)],
    "vcf_stream_destroy": [_P],
    "vcf_stream_sync": [_P],
    "vcf_event_create": [ctypes.POINTER(_P)],
    "vcf_event_destroy": [_P],
    "vcf_event_record": [_P, _P],
    "vcf_event_sync": [_P],
    "vcf_stream_wait_event": [_P, _P],
    "vcf_copy_pieces": [_P, _P, _I64, _P, _P],
    "vcf_event_elapsed_ms": [_P, _P, ctypes.POINTER(ctypes.c_float)],
    "vcf_dct_padded_shape": [_I32, _I32, _I32, _PI32, _PI32],
    "vcf_dct_dz_encode": [_P, _I64, _I32, _I32, _I32, _I32, _U32, _P, _P],
    "vcf_dct_dz_decode": [_P, _I64, _I32, _I32, _I32, _I32, _U32, _P, _P],
    "vcf_dct_block_size_supported": [_I32],
    "vcf_dct_perceptual_tables": [_I32, ctypes.c_void_p, ctypes.c_void_p],
    "vcf_dct_dz_encode_any": [_P, _I64, _I32, _I32, _I32, _I32, _U32, _P, _P],
    "vcf_dct_dz_decode_any": [_P, _I64, _I32, _I32, _I32, _I32, _U32, _P, _P],
    "vcf_dct_dz_encode_k32": [_P, _I64, _I32, _I32, _I32, _I32, _U32, _P, _P],
    "vcf_dct_dz_decode_k32": [_P, _I64, _I32, _I32, _I32, _I32, _U32, _P, _P],
    "vcf_dct_raw_encode": [_P, _I64, _I32, _I32, _I32, _U32, _P, _P],
    "vcf_dct_raw_decode": [_P, _I64, _I32, _I32, _I32, _U32, _P, _P],
    "vcf_ycrcb_from_rgb": [_P, _I64, _P, _P],
    "vcf_ycrcb_to_rgb": [_P, _I64, _P, _P],
    "vcf_ycrcb_dz_encode": [_P, _I64, _I32, _P, _P],
    "vcf_ycrcb_dz_decode": [_P, _I64, _I32, _P, _P],
    "vcf_ycocg_dz_encode": [_P, _I64, _I32, _P, _P],
    "vcf_ycocg_dz_decode": [_P, _I64, _I32, _P, _P],
    "vcf_ycocg_i16_from_rgb": [_P, _I64, _I32, _P, _P],
    "vcf_ycocg_i16_to_rgb": [_P, _I64, _I32, _P, _P],
    "vcf_dz_u8_encode": [_P, _I64, _I32, _P, _P],
    "vcf_dz_u8_decode": [_P, _I64, _I32, _P, _P],
    "vcf_lm_levels": [_I32, _I32, _I32],
    "vcf_lm_histogram": [_P, _I32, _I64, _I32, _I32, _I32, _P, _P],
    "vcf_lm_design": [_P, _I32, _I32, _I32, _P],
    "vcf_lm_encode": [_P, _I32, _I64, _I32, _P, _I32, _P, _I32, _P],
    "vcf_lm_decode": [_P, _I32, _I64, _I32, _P, _I32, _P, _I32, _P, _P],
    "vcf_wavelet_index": [ctypes.c_char_p, _PI32],
    "vcf_dwt_layout": [_I32, _I32, _I32, _PI32, _PI32, ctypes.POINTER(_I64), ctypes.POINTER(_I64)],
    "vcf_dwt_dz_encode": [_P, _I64, _I32, _I32, _I32, _I32, _I32, _P, _P, _P],
    "vcf_dwt_dz_decode": [_P, _I64, _I32, _I32, _I32, _I32, _I32, _P, _P, _P],
    "vcf_dwt_dz_encode_lift": [_P, _I64, _I32, _I32, _I32, _I32, _I32, _P, _P, _P],
    "vcf_dwt_dz_decode_lift": [_P, _I64, _I32, _I32, _I32, _I32, _I32, _P, _P, _P],
    "vcf_ipp_block_match": [_P, _P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P],
    "vcf_ipp_set_full_search_variant": [_I32],
    "vcf_ipp_motion_compensate": [_P, _P, _I32, _I32, _I32, _P, _P],
    "vcf_ipp_residual": [_P, _P, _I64, _P, _P],
    "vcf_ipp_reconstruct": [_P, _P, _I64, _P, _P],
    "vcf_ipp_rdo_modes": [_P, _P, _I32, _I32, _I32, _I32, ctypes.c_double, _P, _P, _P],
    "vcf_ipp_rdo_residual": [_P, _P, _P, _I32, _I32, _I32, _P, _P],
    "vcf_ipp_rdo_reconstruct": [_P, _P, _P, _I32, _I32, _I32, _P, _P],
    "vcf_cbaac_bound": [_I64],
    "vcf_cbaac_encode": [_P, _I64, _I32, _P, _I64, ctypes.POINTER(_I64), ctypes.POINTER(_I64)],
    "vcf_cbaac_decode": [_P, _I64, _I64, _I32, _P],
    "vcf_cbaac_model_trace": [_P, _I64, _I32, _P],
    "vcf_cbahc_bound": [_I64],
    "vcf_cbahc_encode": [_P, _I64, _I32, _P, _I64, ctypes.POINTER(_I64), ctypes.POINTER(_I64)],
    "vcf_cbahc_decode": [_P, _I64, _I64, _I32, _P],
    "vcf_png_info": [_P, _I64, _PI32, _PI32, _PI32],
    "vcf_png_decode_rgb": [_P, _I64, _P, _I64],
    "vcf_png_encode_rgb": [_P, _I32, _I32, _I32, _I32, _P, _I64, ctypes.POINTER(_I64)],
    "vcf_png_encode_bound": [_I32, _I32],
    "vcf_zlib_bound": [_I64],
    "vcf_zlib_workspace": [_I64],
    "vcf_zlib_set_workspace_budget": [_I64],
    "vcf_dwt_lift_set_fused": [_I32],
    "vcf_dwt_set_inverse_band21": [_I32],
    "vcf_dwt_lift_analyze_f64": [_P, _I32, _I32, _I32, _P, _P, _P, _P],
    "vcf_zlib_max_strip": [],
    "vcf_inflate_strips": [_P, _P, _P, _I64, _P, _P, _P, _P, _P],
    "vcf_zlib_strip_count": [_I64, _I32],
    "vcf_zlib_strips": [_P, _I64, _I64, _I32, _I32, _P, _I64, _P, _P, _P],
    "vcf_deadzone_quantize": [_P, _I32, _I64, _I32, _P, _P],
    "vcf_deadzone_dequantize": [_P, _I32, _I64, _I32, _P, _P],
    "vcf_cbaac_tiled_set_variant": [_I32],
    "vcf_cbaac_tiled_segments": [_I64, _I64],
    "vcf_cbaac_tiled_frames_workspace": [_I64, _I64, _I64],
    "vcf_cbaac_tiled_prior_frames": [_P, _I64, _I64, _I64, _P, _P, _P],
    "vcf_cbaac_tiled_encode_frames": [_P, _I64, _I64, _I64, _I32, _P, _I64, _P, _I64, _P, _P, _P],
    "vcf_cbaac_tiled_decode_frames": [_P, _P, _I64, _I64, _I32, _P, _I64, _P, _I64, _P],
    "vcf_cbaac_tiled_workspace": [_I64, _I64],
    "vcf_cbaac_tiled_bound": [_I64, _I64],
    "vcf_cbaac_tiled_encode": [_P, _I64, _I32, _I64, _P, _I64, _P, _P, _P],
    "vcf_cbaac_tiled_trace": [_P, _I64, _I32, _I64, _P, _P, _P, _P],
    "vcf_cbaac_tiled_decode": [_P, _P, _I64, _I32, _I64, _P, _P],
    "vcf_cbaac_tiled_prior": [_P, _I64, _P, _P, _P],
    "vcf_cbaac_tiled_prior_classes": [_P, _I64, _I64, _I64, _I64, _I32, _P, _P, _P],
    "vcf_cbaac_tiled_encode_classes": [_P, _I64, _I64, _I64, _I32, _P, _I32, _I64, _P, _I64, _P, _P, _P],
    "vcf_cbaac_tiled_decode_classes": [_P, _P, _I64, _I64, _I32, _P, _I32, _I64, _P, _I64, _P],
    "vcf_cbaac_tiled_encode_prior": [_P, _I64, _I32, _P, _I64, _P, _I64, _P, _P, _P],
    "vcf_cbaac_tiled_decode_prior": [_P, _P, _I64, _I32, _P, _I64, _P, _P],
    "vcf_cbaac_encode_prior": [_P, _I64, _I32, _P, _P, _I64, ctypes.POINTER(_I64), ctypes.POINTER(_I64)],
    "vcf_cbaac_decode_prior": [_P, _I64, _I64, _I32, _P, _P],
    "vcf_leb128_encode_rows": [_P, _I64, _I64, _P, _I64, _P],
    "vcf_prior_rows_sparse": [_P, _I64, _I32, _P, _I64, _P],
    "vcf_comm_unique_id": [_P, _SZ],
    "vcf_comm_init": [ctypes.POINTER(_P), _P, ctypes.c_int, ctypes.c_int],
    "vcf_comm_init_timeout": [ctypes.POINTER(_P), _P, ctypes.c_int, ctypes.c_int, _I64],
    "vcf_comm_wait": [_P, _P],
    "vcf_comm_destroy": [_P],
    "vcf_comm_rank": [_P, _PI, _PI],
    "vcf_comm_allgather_i64": [_P, _P, _I64, _P, _P],
    "vcf_comm_allreduce_f64": [_P, _P, _P, _I64, ctypes.c_int, _P],
    "vcf_comm_gatherv": [_P, _P, _I64, _P, _P, ctypes.c_int, _P],
}

# the experimental A/B library (include/vcf_amd_ab.h): kernel variants, loaded
# only by the A/B scripts and the cross-check tests
AB_SIGNATURES = {
    "vcf_dct_dz_encode_variant": [ctypes.c_int, _P, _I64, _I32, _I32, _I32, _I32, _U32, _P, _P],
    "vcf_dct_dz_decode_variant": [ctypes.c_int, _P, _I64, _I32, _I32, _I32, _I32, _U32, _P, _P],
    "vcf_dwt_dz_encode_variant": [_I32, _P, _I64, _I32, _I32, _I32, _I32, _I32, _P, _P, _P],
    "vcf_dwt_dz_decode_variant": [_I32, _P, _I64, _I32, _I32, _I32, _I32, _I32, _P, _P, _P],
    "vcf_inflate_strips_wincheck": [_P, _P, _P, _I64, _P, _P, _P, _P, _P, _P],
}

_lib = None
_ab = None
_lock = threading.Lock()


def lib_path() -> str:
    return os.environ.get("VCF_AMD_LIB", _build.LIB)


def lib():
    """Load (once) and return the ctypes handle.  Raises if it cannot."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            path = lib_path()
            if not os.path.exists(path):
                raise ImportError(
                    f"libvcf_amd.so not found at {path}: build it with "
                    "`python -m vcf_amd._build` (hipcc, gfx950). There is no CPU fallback.")
            L = ctypes.CDLL(path)
            for name, argtypes in SIGNATURES.items():
                f = getattr(L, name)
                f.argtypes = argtypes
                f.restype = ctypes.c_int
            L.vcf_last_error.argtypes = []
            L.vcf_last_error.restype = ctypes.c_char_p
            L.vcf_cbaac_bound.restype = ctypes.c_int64
            L.vcf_cbahc_bound.restype = ctypes.c_int64
            L.vcf_png_encode_bound.restype = ctypes.c_int64
            for name in ("vcf_cbaac_tiled_segments", "vcf_cbaac_tiled_workspace", "vcf_cbaac_tiled_bound",
                         "vcf_cbaac_tiled_frames_workspace", "vcf_zlib_bound", "vcf_zlib_workspace",
                         "vcf_zlib_strip_count"):
                getattr(L, name).restype = ctypes.c_int64
            _lib = L
    return _lib


def ab():
    """Load (once) and return the A/B library (libvcf_amd_ab.so)."""
    global _ab
    if _ab is not None:
        return _ab
    with _lock:
        if _ab is None:
            path = os.environ.get("VCF_AMD_AB_LIB", _build.AB_LIB)
            if not os.path.exists(path):
                raise ImportError(f"libvcf_amd_ab.so not found at {path}: `python -m vcf_amd._build` builds it")
            L = ctypes.CDLL(path)
            for name, argtypes in AB_SIGNATURES.items():
                f = getattr(L, name)
                f.argtypes = argtypes
                f.restype = ctypes.c_int
            L.vcf_last_error.argtypes = []
            L.vcf_last_error.restype = ctypes.c_char_p
            _ab = L
    return _ab


def check(status: int, handle=None) -> int:
    """Raise for a negative status; a non-negative one (VCF_OK, or a count such as
    vcf_lm_levels' N) is returned."""
    if status >= VCF_OK:
        return status
    msg = (handle or lib()).vcf_last_error().decode(errors="replace")
    if status == VCF_ERR_INVALID:
        raise VCFInvalidArgument(status, msg)
    if status == VCF_ERR_UNSUPPORTED:
        raise VCFUnsupported(status, msg)
    if status == VCF_ERR_TIMEOUT:
        raise VCFTimeout(status, msg)
    raise VCFError(status, msg)


def call(name: str, *args) -> int:
    return check(getattr(lib(), name)(*args))


def call_ab(name: str, *args) -> int:
    """An entry point of the A/B library (variants; not the product path)."""
    L = ab()
    return check(getattr(L, name)(*args), L)


# A/B scripts: variant 0 = the product entry point, others = the A/B library's
def dct_encode_v(variant, *args):
    return call("vcf_dct_dz_encode", *args) if variant == 0 else call_ab("vcf_dct_dz_encode_variant", variant, *args)


def dct_decode_v(variant, *args):
    return call("vcf_dct_dz_decode", *args) if variant == 0 else call_ab("vcf_dct_dz_decode_variant", variant, *args)


def dwt_encode_v(variant, *args):
    return call("vcf_dwt_dz_encode", *args) if variant == 0 else call_ab("vcf_dwt_dz_encode_variant", variant, *args)


def dwt_decode_v(variant, *args):
    return call("vcf_dwt_dz_decode", *args) if variant == 0 else call_ab("vcf_dwt_dz_decode_variant", variant, *args)
