"""ctypes binding of the C ABI in include/wvgpu.h (weaviate_amd/libwvgpu.so).

The library is built in-tree by ``__graft_entry__.build()`` (make -C
weaviate_amd/csrc).  There is no CPU fallback: if the shared object is
missing or cannot be loaded, importing the ops raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# WVG_LIB: an alternative in-tree build of the same library (A/B runs of a kernel change)
LIB_PATH = os.environ.get("WVG_LIB") or os.path.join(_HERE, "libwvgpu.so")

WVG_OK = 0
WVG_ERR_INVALID = -1
WVG_ERR_DIM_MISMATCH = -2
WVG_ERR_NOMEM = -3
WVG_ERR_DEVICE = -4
WVG_ERR_NOT_FOUND = -5
WVG_ERR_UNSUPPORTED = -6
WVG_ERR_CAPACITY = -7

KIND_F32, KIND_BQ, KIND_PQ = 0, 1, 2
METRIC_L2, METRIC_DOT, METRIC_COSINE, METRIC_MANHATTAN, METRIC_HAMMING = 0, 1, 2, 3, 4
ORDER_AVX256, ORDER_AVX512 = 0, 1  # reference SIMD kernel whose reduction order distances follow
ABI_VERSION = 3  # WVG_ABI_VERSION of include/wvgpu.h this binding follows
METRIC_BY_NAME = {"l2-squared": METRIC_L2, "dot": METRIC_DOT, "cosine": METRIC_COSINE,
                  "cosine-dot": METRIC_COSINE, "manhattan": METRIC_MANHATTAN, "hamming": METRIC_HAMMING}



class Options(ctypes.Structure):
    """struct wvg_options (include/wvgpu.h): context options fixed at wvg_open_ex."""
    _fields_ = [("size", c_uint32), ("mfma_min_queries", c_uint32), ("cache_reuse", ctypes.c_int32),
                ("merge_wait_us", c_uint32), ("batch_screen", ctypes.c_int32), ("coalesce", ctypes.c_int32),
                ("heap_replay", ctypes.c_int32)]


# name -> (restype, argtypes); every symbol declared in include/wvgpu.h.
_P = POINTER
SIGNATURES = {
    "wvg_abi_version": (c_int, []),
    "wvg_last_error": (c_char_p, []),
    "wvg_device_count": (c_int, [_P(c_int)]),
    "wvg_open": (c_int, [c_int, _P(c_void_p)]),
    "wvg_options_default": (None, [_P(Options)]),
    "wvg_open_ex": (c_int, [c_int, _P(Options), _P(c_void_p)]),
    "wvg_close": (c_int, [c_void_p]),
    "wvg_synchronize": (c_int, [c_void_p]),
    "wvg_host_alloc": (c_int, [c_void_p, c_uint64, POINTER(c_void_p)]),
    "wvg_host_free": (c_int, [c_void_p, c_void_p]),
    "wvg_device_alloc": (c_int, [c_void_p, c_uint64, c_int, POINTER(c_void_p)]),
    "wvg_device_free": (c_int, [c_void_p, c_void_p]),
    "wvg_stream_create": (c_int, [c_void_p, POINTER(c_void_p)]),
    "wvg_stream_destroy": (c_int, [c_void_p, c_void_p]),
    "wvg_stream_synchronize": (c_int, [c_void_p, c_void_p]),
    "wvg_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "wvg_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "wvg_set_distance_order": (c_int, [c_void_p, c_int]),
    "wvg_corpus_create": (c_int, [c_void_p, c_int, c_int, c_uint32, c_uint64, c_uint64, _P(c_void_p)]),
    "wvg_corpus_destroy": (c_int, [c_void_p]),
    "wvg_corpus_reserve": (c_int, [c_void_p, c_uint64]),
    "wvg_corpus_info": (c_int, [c_void_p, _P(c_uint64), _P(c_uint64), _P(c_uint64)]),
    "wvg_corpus_upsert": (c_int, [c_void_p, _P(c_uint64), _P(c_float), c_uint64, c_uint32]),
    "wvg_corpus_upsert_codes": (c_int, [c_void_p, _P(c_uint64), c_void_p, c_uint64]),
    "wvg_corpus_load_kv": (c_int, [c_void_p, _P(c_uint8), _P(c_uint8), c_uint64, c_uint64]),
    "wvg_corpus_distance_by_ids": (c_int, [c_void_p, _P(c_float), _P(c_uint64), c_uint64, _P(c_float), _P(c_uint8)]),
    "wvg_corpus_distance_by_ids_batch": (c_int, [c_void_p, _P(c_float), c_uint32, _P(c_uint64), _P(c_uint64),
                                                 _P(c_float), _P(c_uint8)]),
    "wvg_corpus_delete": (c_int, [c_void_p, _P(c_uint64), c_uint64]),
    "wvg_corpus_get": (c_int, [c_void_p, c_uint64, c_void_p]),
    "wvg_corpus_get_batch": (c_int, [c_void_p, _P(c_uint64), c_uint64, c_void_p, _P(c_uint8)]),
    "wvg_corpus_fill_synthetic": (c_int, [c_void_p, c_uint64, c_uint64, c_int]),
    "wvg_pq_set_codebook": (c_int, [c_void_p, _P(c_float), c_uint32, c_uint32]),
    "wvg_search": (c_int, [c_void_p, _P(c_float), c_uint32, c_uint32, _P(c_uint64), c_uint64,
                           _P(c_uint64), _P(c_float), _P(c_uint32)]),
    "wvg_search_bq_rescore": (c_int, [c_void_p, c_void_p, _P(c_float), c_uint32, c_uint32, c_uint32,
                                      _P(c_uint64), c_uint64, _P(c_uint64), _P(c_float), _P(c_uint32)]),
    "wvg_search_bq_candidates": (c_int, [c_void_p, _P(c_float), c_uint32, c_uint32, _P(c_uint64), c_uint64,
                                         _P(c_uint64), _P(c_float), _P(c_uint32)]),
    "wvg_search_by_distance": (c_int, [c_void_p, _P(c_float), c_float, ctypes.c_int64, _P(c_uint64), c_uint64,
                                       _P(c_uint64), _P(c_float), c_uint64, _P(c_uint64)]),
    "wvg_search_by_distance_window": (c_int, [c_void_p, _P(c_float), c_float, c_uint32, _P(c_uint64), c_uint64,
                                              _P(c_uint64), _P(c_float), c_uint64, _P(c_uint64)]),
    "wvg_search_workspace_size": (c_size_t, [c_void_p, c_uint32, c_uint32]),
    "wvg_search_device": (c_int, [c_void_p, c_void_p, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_size_t, c_void_p]),
    "wvg_search_device_pipelined": (c_int, [c_void_p, c_void_p, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_size_t, c_void_p]),
    "wvg_topk_merge_device": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_uint32, c_uint32, c_uint32,
                                      c_void_p, c_void_p, c_void_p, c_void_p]),
    "wvg_search_device_check": (c_int, [c_void_p, c_void_p, c_void_p]),
    "wvg_topk_packed_bytes": (c_size_t, [c_uint32, c_uint32]),
    "wvg_topk_merge_packed": (c_int, [c_void_p, c_void_p, c_uint32, c_uint32, c_uint32, c_uint32,
                                      c_void_p, c_void_p, c_void_p, c_void_p]),
    "wvg_rescore": (c_int, [c_void_p, c_int, _P(c_float), _P(c_float), _P(c_uint64), c_uint64, c_uint32, c_uint32,
                            _P(c_uint64), _P(c_float), _P(c_uint32)]),
    "wvg_pq_encode_corpus": (c_int, [c_void_p, c_void_p]),
    "wvg_multi_open": (c_int, [_P(c_int), c_int, _P(Options), _P(c_void_p)]),
    "wvg_multi_close": (c_int, [c_void_p]),
    "wvg_multi_info": (c_int, [c_void_p, _P(c_int), _P(c_int)]),
    "wvg_multi_ctx": (c_int, [c_void_p, c_int, _P(c_void_p)]),
    "wvg_multi_corpus_create": (c_int, [c_void_p, c_int, c_int, c_uint32, c_uint64, _P(c_void_p)]),
    "wvg_multi_corpus_destroy": (c_int, [c_void_p]),
    "wvg_multi_corpus_shard": (c_int, [c_void_p, c_int, _P(c_void_p), _P(c_uint64), _P(c_uint64)]),
    "wvg_multi_corpus_upsert": (c_int, [c_void_p, _P(c_uint64), _P(c_float), c_uint64, c_uint32]),
    "wvg_multi_corpus_delete": (c_int, [c_void_p, _P(c_uint64), c_uint64]),
    "wvg_multi_corpus_fill_synthetic": (c_int, [c_void_p, c_uint64, c_uint64, c_int]),
    "wvg_multi_corpus_set_codebook": (c_int, [c_void_p, _P(c_float), c_uint32, c_uint32]),
    "wvg_multi_search": (c_int, [c_void_p, _P(c_float), c_uint32, c_uint32, _P(c_uint64), c_uint64,
                                 _P(c_uint64), _P(c_float), _P(c_uint32)]),
    "wvg_synthetic_rows": (c_int, [c_void_p, c_uint64, _P(c_uint64), c_uint64, c_uint32, c_int, c_int, _P(c_float)]),
    "wvg_profile_start": (c_int, [c_void_p]),
    "wvg_profile_stop": (c_int, [c_void_p, _P(ctypes.c_double), _P(c_uint64)]),
    "wvg_measure_hbm_read": (c_int, [c_void_p, c_uint64, c_uint32, _P(ctypes.c_double)]),
    "wvg_distance_batch": (c_int, [c_void_p, c_int, _P(c_float), _P(c_float), c_uint64, c_uint32, _P(c_float)]),
    "wvg_normalize_batch": (c_int, [c_void_p, _P(c_float), c_uint64, c_uint32, _P(c_float)]),
    "wvg_bq_encode": (c_int, [c_void_p, _P(c_float), c_uint64, c_uint32, _P(c_uint64)]),
    "wvg_bq_distance_batch": (c_int, [c_void_p, _P(c_uint64), _P(c_uint64), c_uint64, c_uint32, _P(c_float)]),
    "wvg_pq_encode": (c_int, [c_void_p, _P(c_float), c_uint32, c_uint32, _P(c_float), c_uint64, c_uint32,
                              _P(c_uint8)]),
    "wvg_pq_lut": (c_int, [c_void_p, c_int, _P(c_float), c_uint32, c_uint32, c_uint32, _P(c_float), _P(c_float)]),
    "wvg_pq_fit": (c_int, [c_void_p, _P(c_float), c_uint64, c_uint32, c_uint32, c_uint32, c_uint64, c_uint64,
                           _P(c_float), _P(c_uint32)]),
    "wvg_pq_global_distances": (c_int, [c_void_p, c_int, _P(c_float), c_uint32, c_uint32, c_uint32, _P(c_float)]),
    "wvg_pq_sdc_batch": (c_int, [c_void_p, c_int, _P(c_float), c_uint32, c_uint32, _P(c_uint8), _P(c_uint8),
                                 c_uint64, _P(c_float)]),
    "wvg_pq_adc_batch": (c_int, [c_void_p, c_int, _P(c_float), c_uint32, c_uint32, _P(c_uint8), c_uint64,
                                 _P(c_float)]),
}


class WvgError(RuntimeError):
    """A negative status from the C ABI, carrying wvg_last_error()."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"wvg error {code}: {msg}")
        self.code = code
        self.msg = msg


_lib = None


def load() -> ctypes.CDLL:
    """Load libwvgpu.so (raises if it was not built: no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C weaviate_amd/csrc)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.wvg_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH}: ABI {lib.wvg_abi_version()}, this binding needs {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != WVG_OK:
        lib = load()
        raise WvgError(rc, lib.wvg_last_error().decode(errors="replace"))


def fptr(a):
    return a.ctypes.data_as(POINTER(c_float))


def u64ptr(a):
    return a.ctypes.data_as(POINTER(c_uint64))


def u32ptr(a):
    return a.ctypes.data_as(POINTER(c_uint32))


def u8ptr(a):
    return a.ctypes.data_as(POINTER(c_uint8))
