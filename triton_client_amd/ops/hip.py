"""ctypes binding of libtcamd_hip.so: HIP runtime glue and CDNA4 kernels.

Runtime: device memory, pinned host memory, IPC handles, copies, streams,
events, peer access.  Kernels (csrc/kernels/*.hip, gfx950):

* :func:`synth_fill`      K1 Philox synthetic data (random/zero/constant/normal)
* :func:`convert`         K4/K5 FP32 <-> BF16 (trunc|RNE) / FP16 / FP8 e4m3,e5m2
* :func:`layout_pack`     K6 fused gather + NCHW<->NHWC + convert + scale/bias
* :func:`batched_copy`    K7 one-launch gather/concat/scatter of byte ranges
* :func:`pack_bytes`      K2 BYTES serialisation (LDS block scan + scatter)
* :func:`index_bytes`     K3 BYTES index walk through an LDS window

Pointers are plain ints (device addresses).  ``stream`` is a hipStream_t as an
int (``torch.cuda.current_stream().cuda_stream`` works) or None for the
library's per-device copy stream / the null stream.
"""

import contextlib
import ctypes
import os
import sys

import numpy as np

from . import dtypes

# TCAMD_HIP_LIB: load another build of the library (A/B timing of two kernel
# builds in one tree, tools only)
_PATH = os.environ.get("TCAMD_HIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                        "libtcamd_hip.so")
IPC_HANDLE_SIZE = 64

MEMORY_UNREGISTERED = 0
MEMORY_HOST = 1
MEMORY_DEVICE = 2
MEMORY_MANAGED = 3


class HipError(RuntimeError):
    def __init__(self, code, what):
        self.code = code
        msg = _lib.tcamd_error_string(code).decode() if _lib is not None else str(code)
        super().__init__("%s failed: %s (hipError %d)" % (what, msg, code))


_lib = None

_SIGS = {
    "tcamd_error_string": ([ctypes.c_int], ctypes.c_char_p),
    "tcamd_ipc_handle_size": ([], ctypes.c_int),
    "tcamd_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "tcamd_set_device": ([ctypes.c_int], ctypes.c_int),
    "tcamd_get_device": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "tcamd_device_synchronize": ([ctypes.c_int], ctypes.c_int),
    "tcamd_device_uva": ([ctypes.c_int, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "tcamd_device_name": ([ctypes.c_int, ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
    "tcamd_malloc": ([ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "tcamd_free": ([ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
    "tcamd_host_alloc": ([ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "tcamd_host_free": ([ctypes.c_void_p], ctypes.c_int),
    "tcamd_host_register": ([ctypes.c_void_p, ctypes.c_size_t], ctypes.c_int),
    "tcamd_host_unregister": ([ctypes.c_void_p], ctypes.c_int),
    "tcamd_ipc_get_handle": ([ctypes.c_void_p, ctypes.c_char_p], ctypes.c_int),
    "tcamd_ipc_open": ([ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "tcamd_ipc_close": ([ctypes.c_void_p, ctypes.c_int], ctypes.c_int),
    "tcamd_pointer_info": (
        [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)],
        ctypes.c_int,
    ),
    "tcamd_memcpy": ([ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t], ctypes.c_int),
    "tcamd_memcpy_async": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p], ctypes.c_int),
    "tcamd_memset_async": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p], ctypes.c_int),
    "tcamd_memcpy_peer_async": (
        [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_enable_peer": ([ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "tcamd_stream_create": ([ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "tcamd_stream_destroy": ([ctypes.c_void_p], ctypes.c_int),
    "tcamd_stream_synchronize": ([ctypes.c_void_p], ctypes.c_int),
    "tcamd_event_create": ([ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "tcamd_event_destroy": ([ctypes.c_void_p], ctypes.c_int),
    "tcamd_event_record": ([ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "tcamd_event_synchronize": ([ctypes.c_void_p], ctypes.c_int),
    "tcamd_event_elapsed_ms": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
    "tcamd_stream_wait_event": ([ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "tcamd_last_error": ([], ctypes.c_int),
    # kernels
    "tcamd_synth_fill": (
        [
            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_double,
            ctypes.c_double, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    "tcamd_convert": (
        [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_layout_pack": (
        [
            ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
            ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    "tcamd_batched_copy": (
        [
            ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64),
            ctypes.c_int, ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    # fused DenseNet kernels (csrc/kernels/densenet.hip)
    "tcamd_dn_conv1x1": (
        [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    "tcamd_dn_conv1x1_ex": (
        [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
            ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    "tcamd_dn_conv1x1_v": (
        [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    "tcamd_dn_conv3x3_v": (
        [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
         ctypes.c_int, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_dn_conv3x3": (
        [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
         ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_dn_stem_pool": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
         ctypes.c_int, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_dn_stem_fused": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
         ctypes.c_int, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_dn_head_pool": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
         ctypes.c_void_p],
        ctypes.c_int,
    ),
    # fp32-parity (bf16x3 split-precision) DenseNet kernels (csrc/kernels/densenet_x3.hip)
    "tcamd_x3_conv1x1_ws_bytes": ([ctypes.c_int, ctypes.c_int, ctypes.c_int], ctypes.c_size_t),
    "tcamd_x3_conv1x1": (
        [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
            ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    "tcamd_x3_conv3x3": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_x3_dense_layer": (
        [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
            ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    "tcamd_x3s_dense_layer": (
        [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    "tcamd_x3s_steps_per_block": ([ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "tcamd_x3c_base": (
        [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
         ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_x3c_layer": (
        [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
         ctypes.c_int, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_x3_dense_fused": (
        [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    "tcamd_x3_dense_small": (
        [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    "tcamd_x3_small_tiles": ([ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "tcamd_x3_dense_fused_ws": (
        [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    "tcamd_x3_dense_fused3": (
        [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
    "tcamd_k3_set_check": ([ctypes.c_int], ctypes.c_int),
    "tcamd_knob_count": ([], ctypes.c_int),
    "tcamd_knob_info": (
        [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_longlong),
         ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_char_p)],
        ctypes.c_int,
    ),
    "tcamd_knob_set": ([ctypes.c_char_p, ctypes.c_longlong, ctypes.POINTER(ctypes.c_longlong)], ctypes.c_int),
    "tcamd_k17_gemm": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_k17_last_tm": ([], ctypes.c_int),
    "tcamd_k18_gemm": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
         ctypes.c_longlong, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_k18_cfg": (
        [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
         ctypes.POINTER(ctypes.c_int)],
        ctypes.c_int,
    ),
    "tcamd_k18_calls": ([], ctypes.c_longlong),
    "tcamd_qa_head": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
         ctypes.c_int, ctypes.c_int, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_add_layernorm_parts": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_add_layernorm_parts3": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
         ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_k17_calls": ([], ctypes.c_longlong),
    "tcamd_x3_cat": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
    "tcamd_x3_stem": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
         ctypes.c_int, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_x3_head_pool": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
         ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_x3_split": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_add_layernorm": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
         ctypes.c_int, ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_embed_layernorm": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
         ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_attention_bias": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
         ctypes.c_float, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_attention_f32": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
         ctypes.c_int, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_attention": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
         ctypes.c_void_p],
        ctypes.c_int,
    ),
    # native batch executor for pointer-table graph models (csrc/runtime/graph_exec.hip)
    "tcamd_pgx_create": (
        [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int32,
         ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, ctypes.c_int32],
        ctypes.c_void_p,
    ),
    "tcamd_pgx_set_instance": (
        [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64,
         ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.c_char_p, ctypes.c_int32],
        ctypes.c_int32,
    ),
    "tcamd_pgx_execute": (
        [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32], ctypes.c_int,
    ),
    "tcamd_pgx_stats": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int32),
    "tcamd_pgx_destroy": ([ctypes.c_void_p], None),
    "tcamd_pack_bytes_workspace": ([ctypes.c_uint64], ctypes.c_uint64),
    "tcamd_pack_bytes": (
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_index_bytes_last_path": ([ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "tcamd_pack_bytes_strided": (
        [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_void_p],
        ctypes.c_int,
    ),
    "tcamd_index_bytes": (
        [
            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p,
        ],
        ctypes.c_int,
    ),
}


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_PATH):
        raise ImportError(
            "libtcamd_hip.so is not built (expected at %s); run `python __graft_entry__.py build`" % _PATH
        )
    # One HIP runtime per process: torch bundles libamdhip64.so.7 with the same
    # SONAME, so whichever copy is loaded first is shared by both.
    lib = ctypes.CDLL(_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (argtypes, restype) in _SIGS.items():
        if os.environ.get("TCAMD_HIP_LIB") and not hasattr(lib, name):
            continue  # an older A/B build: entry points it predates stay unbound
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    _lib = lib
    return lib


def lib():
    return _load()


def _check(rc, what):
    if rc != 0:
        raise HipError(rc, what)


def _vp(x):
    return None if x is None or x == 0 else ctypes.c_void_p(int(x))


def loaded_path():
    return _PATH


# ---------------------------------------------------------------------------
# runtime
# ---------------------------------------------------------------------------
def device_count():
    n = ctypes.c_int(0)
    rc = _load().tcamd_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def set_device(dev):
    _check(_load().tcamd_set_device(dev), "hipSetDevice")


def get_device():
    d = ctypes.c_int(0)
    _check(_load().tcamd_get_device(ctypes.byref(d)), "hipGetDevice")
    return d.value


def synchronize(dev=0):
    _check(_load().tcamd_device_synchronize(dev), "hipDeviceSynchronize")


def device_uva(dev):
    v = ctypes.c_int(0)
    _check(_load().tcamd_device_uva(dev, ctypes.byref(v)), "hipGetDeviceProperties")
    return bool(v.value)


def device_arch(dev=0):
    buf = ctypes.create_string_buffer(128)
    _check(_load().tcamd_device_name(dev, buf, 128), "hipGetDeviceProperties")
    return buf.value.decode()


def malloc(dev, nbytes):
    p = ctypes.c_void_p()
    _check(_load().tcamd_malloc(dev, nbytes, ctypes.byref(p)), "hipMalloc(%d B)" % nbytes)
    return p.value


def free(dev, ptr):
    _check(_load().tcamd_free(dev, _vp(ptr)), "hipFree")


def host_alloc(nbytes):
    p = ctypes.c_void_p()
    _check(_load().tcamd_host_alloc(nbytes, ctypes.byref(p)), "hipHostMalloc")
    return p.value


def host_free(ptr):
    _check(_load().tcamd_host_free(_vp(ptr)), "hipHostFree")


def host_register(ptr, nbytes):
    _check(_load().tcamd_host_register(_vp(ptr), nbytes), "hipHostRegister")


def host_unregister(ptr):
    _check(_load().tcamd_host_unregister(_vp(ptr)), "hipHostUnregister")


def ipc_get_handle(ptr):
    buf = ctypes.create_string_buffer(IPC_HANDLE_SIZE)
    _check(_load().tcamd_ipc_get_handle(_vp(ptr), buf), "hipIpcGetMemHandle")
    return buf.raw


def ipc_open(handle, dev):
    if len(handle) != IPC_HANDLE_SIZE:
        raise ValueError("IPC handle must be %d bytes" % IPC_HANDLE_SIZE)
    p = ctypes.c_void_p()
    _check(_load().tcamd_ipc_open(bytes(handle), dev, ctypes.byref(p)), "hipIpcOpenMemHandle")
    return p.value


def ipc_close(ptr, dev):
    _check(_load().tcamd_ipc_close(_vp(ptr), dev), "hipIpcCloseMemHandle")


def pointer_info(ptr):
    mt = ctypes.c_int(0)
    dev = ctypes.c_int(-1)
    _check(_load().tcamd_pointer_info(_vp(ptr), ctypes.byref(mt), ctypes.byref(dev)), "hipPointerGetAttributes")
    return mt.value, dev.value


def _host_ptr(buf):
    if isinstance(buf, np.ndarray):
        if not buf.flags["C_CONTIGUOUS"]:
            raise ValueError("host buffer must be C-contiguous")
        return buf.ctypes.data
    if isinstance(buf, int):
        return buf
    return ctypes.addressof(ctypes.c_char.from_buffer(buf))


def memcpy(dst, src, nbytes, dev=0):
    """Synchronous copy (any direction, UVA) on the per-device copy stream."""
    if nbytes:
        _check(_load().tcamd_memcpy(dev, _vp(dst), _vp(src), nbytes), "hipMemcpy")


def memcpy_h2d(dst_ptr, host, nbytes, dev=0):
    memcpy(dst_ptr, _host_ptr(host), nbytes, dev)


def memcpy_d2h(host, src_ptr, nbytes, dev=0):
    memcpy(_host_ptr(host), src_ptr, nbytes, dev)


def memcpy_d2d(dst_ptr, src_ptr, nbytes, dev=0):
    memcpy(dst_ptr, src_ptr, nbytes, dev)


def memcpy_async(dst, src, nbytes, stream=None):
    if nbytes:
        _check(_load().tcamd_memcpy_async(_vp(dst), _vp(src), nbytes, _vp(stream)), "hipMemcpyAsync")


def memset_async(dst, value, nbytes, stream=None):
    _check(_load().tcamd_memset_async(_vp(dst), value, nbytes, _vp(stream)), "hipMemsetAsync")


def memcpy_peer_async(dst, dst_dev, src, src_dev, nbytes, stream=None):
    _check(
        _load().tcamd_memcpy_peer_async(_vp(dst), dst_dev, _vp(src), src_dev, nbytes, _vp(stream)),
        "hipMemcpyPeerAsync",
    )


def enable_peer(dev, peer):
    _check(_load().tcamd_enable_peer(dev, peer), "hipDeviceEnablePeerAccess(%d->%d)" % (dev, peer))


class Stream:
    """A non-blocking HIP stream owned by this library."""

    def __init__(self, dev=0):
        self.dev = dev
        s = ctypes.c_void_p()
        _check(_load().tcamd_stream_create(dev, ctypes.byref(s)), "hipStreamCreate")
        self.handle = s.value

    def synchronize(self):
        _check(_load().tcamd_stream_synchronize(_vp(self.handle)), "hipStreamSynchronize")

    def close(self):
        if self.handle:
            _load().tcamd_stream_destroy(_vp(self.handle))
            self.handle = None

    def __int__(self):
        return self.handle or 0


def stream_synchronize(stream):
    _check(_load().tcamd_stream_synchronize(_vp(stream)), "hipStreamSynchronize")


class Event:
    def __init__(self):
        e = ctypes.c_void_p()
        _check(_load().tcamd_event_create(ctypes.byref(e)), "hipEventCreate")
        self.handle = e.value

    def record(self, stream=None):
        _check(_load().tcamd_event_record(_vp(self.handle), _vp(stream)), "hipEventRecord")

    def synchronize(self):
        _check(_load().tcamd_event_synchronize(_vp(self.handle)), "hipEventSynchronize")

    def elapsed_ms(self, end):
        ms = ctypes.c_float(0)
        _check(_load().tcamd_event_elapsed_ms(_vp(self.handle), _vp(end.handle), ctypes.byref(ms)), "hipEventElapsedTime")
        return ms.value

    def close(self):
        if self.handle:
            _load().tcamd_event_destroy(_vp(self.handle))
            self.handle = None


# ---------------------------------------------------------------------------
# kernels
# ---------------------------------------------------------------------------
SYNTH_ZERO, SYNTH_CONST, SYNTH_UNIFORM, SYNTH_NORMAL = 0, 1, 2, 3


def synth_fill(ptr, n_elems, datatype, mode=SYNTH_UNIFORM, lo=0.0, hi=1.0, seed=0, stream_id=0, stream=None):
    """K1: fill ``n_elems`` of ``datatype`` at device ``ptr`` (16-B aligned).

    uniform: floats in [lo, hi), integers in [lo, hi]; normal: mean lo, std hi.
    Deterministic in (seed, stream_id, element offset).
    """
    _check(
        _load().tcamd_synth_fill(
            _vp(ptr), n_elems, dtypes.code(datatype), mode, float(lo), float(hi),
            seed & (2**64 - 1), stream_id & (2**64 - 1), _vp(stream),
        ),
        "synth_fill",
    )


def convert(src, src_dtype, dst, dst_dtype, n, rounding="trunc", stream=None):
    """K4/K5 elementwise conversion between FP32 and BF16/FP16/FP8."""
    r = 0 if rounding == "trunc" else 1
    _check(
        _load().tcamd_convert(_vp(src), dtypes.code(src_dtype), _vp(dst), dtypes.code(dst_dtype), n, r, _vp(stream)),
        "convert %s->%s" % (src_dtype, dst_dtype),
    )


LAYOUTS = {"NCHW": 0, "NHWC": 1}


def layout_pack(srcs, src_dtype, src_layout, dst, dst_dtype, dst_layout, C, H, W,
                scale=None, bias=None, rounding="rne", stream=None):
    """K6: gather len(srcs) images (each C*H*W) into ``dst`` with layout/dtype
    conversion and per-channel ``x*scale[c]+bias[c]``."""
    n = len(srcs)
    arr = (ctypes.c_void_p * max(n, 1))(*[int(p) for p in srcs])
    sc = (ctypes.c_float * C)(*scale) if scale is not None else None
    bi = (ctypes.c_float * C)(*bias) if bias is not None else None
    _check(
        _load().tcamd_layout_pack(
            arr, n, dtypes.code(src_dtype), LAYOUTS[src_layout], _vp(dst), dtypes.code(dst_dtype),
            LAYOUTS[dst_layout], C, H, W, sc, bi, 0 if rounding == "trunc" else 1, _vp(stream),
        ),
        "layout_pack",
    )


def batched_copy(srcs, dsts, sizes, stream=None):
    """K7: copy sizes[i] bytes srcs[i] -> dsts[i] for all i in one launch."""
    n = len(srcs)
    if n == 0:
        return
    s = (ctypes.c_void_p * n)(*[int(p) for p in srcs])
    d = (ctypes.c_void_p * n)(*[int(p) for p in dsts])
    b = (ctypes.c_uint64 * n)(*[int(x) for x in sizes])
    _check(_load().tcamd_batched_copy(s, d, b, n, _vp(stream)), "batched_copy")


def dn_conv1x1(x, ldx, M, K, in_scale, in_bias, w, N, out_bias, relu_out, y, ldy, pool=0, H=0, W=0, stream=None,
               variant=0, splits=0, ws=None, ws_bytes=0):
    """K8: y[m, :N] = epi(relu(x[m, :K]*s + b) @ w[N, K]^T); pool=1 fuses a 2x2 avg-pool (transition).
    variant: 0 = heuristic, else 10*TM + BK/32 (tile-size override for benchmarking).
    splits: split-K factor (0 = heuristic when a fp32 workspace ``ws`` of ``ws_bytes`` is given)."""
    _check(_load().tcamd_dn_conv1x1_ex(x, ldx, M, K, in_scale, in_bias, w, N, out_bias, int(relu_out), y, ldy,
                                       int(pool), H, W, int(variant), int(splits), ws, int(ws_bytes), _vp(stream)),
           "dn_conv1x1")


def dn_conv3x3(z, imgs, H, W, w, y, ldy, stream=None, variant=0):
    """K9: 3x3/pad-1 conv 128->32 over NHWC rows z; 32 channels per pixel written at y + pixel*ldy.
    variant: 0 = heuristic, else 10*TM + taps-per-load-group."""
    _check(_load().tcamd_dn_conv3x3_v(z, imgs, H, W, w, y, ldy, int(variant), _vp(stream)), "dn_conv3x3")


def dn_stem_pool(x, bias, y, imgs, H, W, C, ldy, stream=None):
    """K10a: y = relu(maxpool3x3/2(x) + bias) into rows of ldy elements."""
    _check(_load().tcamd_dn_stem_pool(x, bias, y, imgs, H, W, C, ldy, _vp(stream)), "dn_stem_pool")


def dn_stem_fused(srcs, x, w, bias, y, imgs, ldy, stream=None):
    """K10s: y = relu(maxpool3x3/2(conv7x7/2(img)) + bias) for 224x224x3 images -> 56x56x64.
    ``srcs``: device array of per-image fp32 NCHW pointers (or None with ``x`` = bf16 NHWC batch);
    ``w``: [64][7][8][4] bf16 packed weights."""
    _check(_load().tcamd_dn_stem_fused(_vp(srcs), _vp(x), w, bias, y, imgs, ldy, _vp(stream)), "dn_stem_fused")


def add_layernorm(x, y, gamma, beta, out, rows, H, eps, stream=None):
    """K11: out = LayerNorm(x + y) * gamma + beta over ``rows`` rows of H bf16 (H in 512/1024/2048/4096)."""
    _check(_load().tcamd_add_layernorm(x, y, gamma, beta, out, rows, H, float(eps), _vp(stream)), "add_layernorm")


ATTENTION_MAX_SEQ = 384


def embed_layernorm(ids, types, word, pos, type_, gamma, beta, out, rows, S, H, vocab, ntypes, eps, stream=None):
    """BERT embeddings in one launch: out [rows][H] bf16 = LayerNorm(word[ids] +
    pos[row % S] + type[types]) * gamma + beta; ids / types int64 [rows]."""
    _check(_load().tcamd_embed_layernorm(_vp(ids), _vp(types), word, pos, type_, gamma, beta, out, int(rows), int(S),
                                         int(H), int(vocab), int(ntypes), float(eps), _vp(stream)), "embed_layernorm")


def attention(qkv, mask, out, seqs, S, heads, scale, stream=None, bias=None):
    """K12: multi-head attention (head dim 64, non-causal) over the fused QKV
    projection's output ``qkv`` [seqs*S][3*heads*64] bf16 into ``out``
    [seqs*S][heads*64] bf16; ``mask`` int32 [seqs][S] key-padding mask (0 =
    padded key) or None.  S % 64 == 0 and S <= ATTENTION_MAX_SEQ.  ``bias``
    (bf16 [3*heads*64] or None): the projection's bias, when ``qkv`` was
    computed without it (q + b_q feeds the scores, b_v is added to the output;
    b_k shifts every score of a query equally and cancels in the softmax)."""
    _check(_load().tcamd_attention_bias(qkv, _vp(bias), _vp(mask), out, int(seqs), int(S), int(heads), float(scale),
                                        _vp(stream)), "attention")


def attention_f32(qkv, mask, out, seqs, S, heads, scale, stream=None, x3=False):
    """K12x: fp32-parity attention (bf16x3 products, fp32 online softmax) over
    the fp32 QKV projection ``qkv`` [seqs*S][3*heads*64] (bias included) into
    ``out`` [seqs*S][heads*64] fp32 -- or, with ``x3``, into the out
    projection's bf16x3 operand, bf16 [seqs*S][3*heads*64] = [hi | hi | lo];
    ``mask`` int32 [seqs][S] (0 = padded key, additive -10000 as the
    reference) or None.  S % 64 == 0."""
    _check(_load().tcamd_attention_f32(qkv, _vp(mask), out, int(seqs), int(S), int(heads), float(scale),
                                       1 if x3 else 0, _vp(stream)), "attention_f32")


def x3_conv1x1_ws_bytes(M, K, N=128):
    """Split-K workspace bytes K8x wants for an M x K -> N 1x1 conv (0: none)."""
    return int(_load().tcamd_x3_conv1x1_ws_bytes(int(M), int(K), int(N)))


def x3_conv1x1(x, ldx, M, K, in_scale, in_bias, w_hi, w_lo, out_bias=None, z_hi=None, z_lo=None, y=None, ldy=0,
               pool=0, H=0, W=0, ws=None, ws_bytes=0, stream=None, N=128):
    """K8x fp32-parity 1x1 conv (N out channels, a multiple of 128): z_hi/z_lo
    split bf16 planes with bias+ReLU (N = 128), or raw fp32 into ``y`` rows of ``ldy``."""
    _check(_load().tcamd_x3_conv1x1(x, ldx, M, K, int(N), in_scale, in_bias, w_hi, w_lo, _vp(out_bias), _vp(z_hi),
                                    _vp(z_lo), _vp(y), int(ldy), int(pool), int(H), int(W), _vp(ws),
                                    int(ws_bytes), _vp(stream)), "x3_conv1x1")


def x3_w3_fragments(w):
    """K9x weight layout: a [32][9*128] (out, tap-major K) tensor -> the MFMA
    fragment-major copy the kernel loads, [tap 9][kq 4][kc 2][h 2][col 32][8]
    (one wave's 16-B-per-lane fragment = 1 KB contiguous).  Apply it to the
    hi and lo planes alike."""
    return w.reshape(32, 9, 4, 2, 2, 8).permute(1, 2, 3, 4, 0, 5).contiguous().reshape(32, 9 * 128)


def x3_conv3x3(z_hi, z_lo, imgs, H, W, w_hi, w_lo, y, ldy, stream=None):
    """K9x fp32-parity 3x3 conv 128 -> 32 into fp32 rows of ``ldy``; ``w_hi`` /
    ``w_lo`` in the x3_w3_fragments layout."""
    _check(_load().tcamd_x3_conv3x3(z_hi, z_lo, imgs, H, W, w_hi, w_lo, y, ldy, _vp(stream)), "x3_conv3x3")


def x3_dense_layer(x, ldx, imgs, H, W, K, s1, t1, w1_hi, w1_lo, b1, z_hi, z_lo, w2_hi, w2_lo, y, ldy, ws=None,
                   ws_bytes=0, stream=None):
    """One fp32-parity dense layer: K8x BN1+ReLU+1x1 (K -> 128, BN2 folded, bias
    ``b1``) then K9x 3x3 (128 -> 32) into ``y`` rows of ``ldy`` (the layer's
    slice).  A split-K 1x1 hands its partials to the 3x3, which reduces them
    while staging its band (no reduce launch)."""
    _check(_load().tcamd_x3_dense_layer(x, int(ldx), int(imgs), int(H), int(W), int(K), s1, t1, w1_hi, w1_lo, b1,
                                        z_hi, z_lo, w2_hi, w2_lo, y, int(ldy), _vp(ws), int(ws_bytes), _vp(stream)),
           "x3_dense_layer")


def x3s_dense_layer(x, ldx, imgs, H, W, K, s1, t1, w1_hi, w1_lo, b1, zacc, zacc_next, w2_hi, w2_lo, y, ldy,
                    stream=None):
    """K13x small-M dense layer (csrc/kernels/densenet_x3s.hip): the 1x1 adds
    into ``zacc`` ([M][128] fp32, ZERO on entry) with float atomics over many
    workgroups, then the 3x3 reads it (bias ``b1`` + ReLU + split in registers)
    into ``y`` rows of ``ldy``, zeroing rows [0, M) of ``zacc_next`` (may be
    None) for the next layer.  ``w1_*`` in x3_w1_fragments, ``w2_*`` in
    x3_w3_fragments."""
    _check(_load().tcamd_x3s_dense_layer(x, int(ldx), int(imgs), int(H), int(W), int(K), s1, t1, w1_hi, w1_lo, b1,
                                         zacc, _vp(zacc_next), w2_hi, w2_lo, y, int(ldy), _vp(stream)),
           "x3s_dense_layer")


X3C_LAYER_WORDS = 9  # int64 words of one X3cLayer table entry


def x3c_layer_entry(w1_hi, w1_lo, s1, t1, b1, w2_hi, w2_lo, zacc, K):
    """One K13x chain table entry (9 int64: 8 device pointers + K); ``w1_*`` in
    x3_w1_fragments, ``w2_*`` in x3_w3_fragments, ``zacc`` [>= M][128] fp32."""
    return [int(w1_hi), int(w1_lo), int(s1), int(t1), int(b1), int(w2_hi), int(w2_lo), int(zacc), int(K)]


def x3c_base(layers, n, x, ldx, imgs, H, W, stream=None):
    """K13x chain, once per run of ``n`` small-M layers: every layer's 1x1 over
    the run's first K_f input channels (plain stores into its zacc) and every
    layer's y slice zeroed.  ``layers``: device table of chain entries."""
    _check(_load().tcamd_x3c_base(_vp(layers), int(n), _vp(x), int(ldx), int(imgs), int(H), int(W), _vp(stream)),
           "x3c_base")


def x3c_layer(layers, l, n, x, ldx, imgs, H, W, stream=None):
    """K13x chain, layer ``l`` of the run (one launch): its 3x3 (plus the
    previous layer's chunk of its 1x1, computed for the tile and halo) and the
    previous layer's chunk fanned out to every later layer's zacc."""
    _check(_load().tcamd_x3c_layer(_vp(layers), int(l), int(n), _vp(x), int(ldx), int(imgs), int(H), int(W),
                                   _vp(stream)), "x3c_layer")


def x3s_steps_per_block(M, K):
    """k16 steps per workgroup the K13x 1x1 plans for an M x K layer."""
    return int(_load().tcamd_x3s_steps_per_block(int(M), int(K)))


def x3_w1_fragments(w):
    """K11x 1x1 weight layout: [128][K] (out, in) -> the 32x32x16 MFMA
    fragment-major copy the fused layer reads from L2, [K/16][q 4][h 2][col 32][8]
    (lane (h, col) = w[32q + col][16ks + 8h .. +8]; one wave load = 1 KB)."""
    n, k = w.shape
    return w.reshape(4, 32, k // 16, 2, 8).permute(2, 0, 3, 1, 4).contiguous().reshape(n, k)


def x3_w3f_fragments(w):
    """K11x 3x3 weight layout: [32][9*128] (out, tap-major K) -> the 16x16x32
    MFMA fragment-major copy, [tap 9][kq 4][oh 2][h 4][col 16][8] (lane
    (h, col) = w[16oh + col][t][32kq + 8h .. +8])."""
    return w.reshape(2, 16, 9, 4, 4, 8).permute(2, 3, 0, 4, 1, 5).contiguous().reshape(32, 9 * 128)


def x3_dense_fused(x, ldx, imgs, H, W, K, s1, t1, w1_hi, w1_lo, b1, w2_hi, w2_lo, y, ldy, stream=None):
    """K11x: one fp32-parity dense layer in ONE kernel, the 128-channel
    bottleneck kept in LDS (never written to HBM).  ``w1_*`` in the
    x3_w1_fragments layout, ``w2_*`` in x3_w3f_fragments; 16 <= W <= 56, K a multiple
    of 32 in 64..224."""
    _check(_load().tcamd_x3_dense_fused(x, int(ldx), int(imgs), int(H), int(W), int(K), s1, t1, w1_hi, w1_lo, b1,
                                        w2_hi, w2_lo, y, int(ldy), _vp(stream)), "x3_dense_fused")


def x3_dense_small(x, ldx, imgs, H, W, K, s1, t1, w1f_hi, w1f_lo, b1, w2_hi, w2_lo, y, ldy, stream=None, tiles=0):
    """K14x: one fp32-parity dense layer of the 14x14 or 7x7 block in ONE
    kernel, ``tiles`` row tiles per image (each with the halo rows its 3x3
    needs, recomputed; 14x14: 2, 4 or 7, 7x7: 1, 2, 4 or 7; 0 = the fewest that give
    every CU a workgroup, :func:`x3_small_tiles`), z kept in a zero-padded LDS
    image of the tile.  ``w1f_*`` in x3_w1_fragments, ``w2_*`` in
    x3_w3f_fragments; K a multiple of 32 in 64..2048."""
    _check(_load().tcamd_x3_dense_small(x, int(ldx), int(imgs), int(H), int(W), int(K), s1, t1, w1f_hi, w1f_lo, b1,
                                        w2_hi, w2_lo, y, int(ldy), int(tiles), _vp(stream)), "x3_dense_small")


def x3_small_tiles(imgs, W):
    """The tiles per image K14x picks for ``imgs`` images of side ``W``."""
    return int(_load().tcamd_x3_small_tiles(int(imgs), int(W)))


def x3_dense_fused3(x, ldx, imgs, H, W, K, s1, t1, w1_hi, w1_lo, b1, w2_hi, w2_lo, y, ldy, stream=None):
    """K11x v3: v1's roles and fragment layouts (``w2_*`` in x3_w3f_fragments),
    with the next chunk's 1x1 K steps interleaved into each tile's 3x3."""
    _check(_load().tcamd_x3_dense_fused3(x, int(ldx), int(imgs), int(H), int(W), int(K), s1, t1, w1_hi, w1_lo, b1,
                                         w2_hi, w2_lo, y, int(ldy), _vp(stream)), "x3_dense_fused3")


def x3_dense_fused_ws(x, ldx, imgs, H, W, K, s1, t1, w1_hi, w1_lo, b1, w2_hi, w2_lo, y, ldy, stream=None):
    """K11w: v1's layer (same fragments, same products in the same order) on
    768 threads: producer waves convert X into LDS stages, consumer waves run
    the MFMAs (csrc/kernels/densenet_x3.hip)."""
    _check(_load().tcamd_x3_dense_fused_ws(x, int(ldx), int(imgs), int(H), int(W), int(K), s1, t1, w1_hi, w1_lo,
                                           b1, w2_hi, w2_lo, y, int(ldy), _vp(stream)), "x3_dense_fused_ws")


def x3_cat(x, out, rows, K, stream=None):
    """fp32-parity bert operand: x fp32 [rows][K] -> out bf16 [rows][3K] =
    [hi | hi | lo] (csrc/kernels/bert.hip), for one bf16 GEMM against
    [W_hi | W_lo | W_hi] that accumulates the three split products."""
    _check(_load().tcamd_x3_cat(x, out, int(rows), int(K), _vp(stream)), "x3_cat")


def x3_stem_fragments(w):
    """K10x weight layout: [64][224] (out, (kh, kw[8], ch[4])) -> the MFMA
    fragment-major copy the stem loads, [half 2][k-step 14][h 2][col 32][8]."""
    return w.reshape(2, 32, 14, 2, 8).permute(0, 2, 3, 1, 4).contiguous().reshape(64, 224)


def x3_stem(srcs, w_hi, w_lo, bias, y, imgs, ldy, stream=None):
    """K10x fp32 stem from a device table of fp32 NCHW image pointers;
    ``w_hi`` / ``w_lo`` in the x3_stem_fragments layout."""
    _check(_load().tcamd_x3_stem(srcs, w_hi, w_lo, bias, y, imgs, ldy, _vp(stream)), "x3_stem")


def x3_head_pool(x, scale, bias, out, imgs, HW, C, stream=None):
    """K10x head: out[i, c] = mean_p relu(x[i, p, c]*scale[c] + bias[c]), fp32."""
    _check(_load().tcamd_x3_head_pool(x, scale, bias, out, imgs, HW, C, _vp(stream)), "x3_head_pool")


def x3_split(w, hi, lo, n, stream=None):
    """fp32 -> (bf16 hi, bf16 lo) planes on the device: w ~= hi + lo to 2^-17."""
    _check(_load().tcamd_x3_split(w, hi, lo, int(n), _vp(stream)), "x3_split")


def dn_head_pool(x, scale, bias, out, imgs, HW, C, stream=None):
    """K10b: out[i, c] = mean_p relu(x[i, p, c]*scale[c] + bias[c])."""
    _check(_load().tcamd_dn_head_pool(x, scale, bias, out, imgs, HW, C, _vp(stream)), "dn_head_pool")


def pack_bytes_workspace(n):
    return int(_load().tcamd_pack_bytes_workspace(n))


def pack_bytes(data_ptr, lens_ptr, n, out_ptr, workspace_ptr, stream=None):
    """K2: device BYTES serialisation (see csrc/kernels/bytes.hip)."""
    _check(
        _load().tcamd_pack_bytes(_vp(data_ptr), _vp(lens_ptr), n, _vp(out_ptr), _vp(workspace_ptr), _vp(stream)),
        "pack_bytes",
    )


def pack_bytes_strided(data_ptr, stride, lens_ptr, n, out_ptr, workspace_ptr, stream=None):
    """K2 over a fixed-width payload (numpy 'S' array): element i's bytes at data + i * stride."""
    _check(
        _load().tcamd_pack_bytes_strided(_vp(data_ptr), int(stride), _vp(lens_ptr), n, _vp(out_ptr),
                                         _vp(workspace_ptr), _vp(stream)),
        "pack_bytes_strided",
    )


def index_bytes_last_path():
    """(path, window) of this thread's last index_bytes: 0 serial walk, 1 v3
    speculative block walk (64-B candidate window), 3 v3 with the 256-B
    window (an element of 60..252 B crossed a block), 2 general
    pointer-doubling fallback."""
    w = ctypes.c_uint64(0)
    p = _load().tcamd_index_bytes_last_path(ctypes.byref(w))
    return p, w.value


def k3_set_check(on):
    """K3 overrun check mode (process-wide): each index_bytes call allocates its
    workspace at exactly the size it needs with a 4 KiB canary behind it and
    fails if the canary changed.  Returns the previous setting."""
    return bool(_load().tcamd_k3_set_check(1 if on else 0))


K17_EPI = {"none": 0, "bias": 1, "bias_gelu": 2, "bias_gelu_erf": 3, "bias_gelu_erf_x3": 4}


def k17_gemm(a, b, bias, c, M, N, K, lda, ldb, ldc, epilogue="none", out_f32=False, stream=None):
    """K17 (csrc/kernels/gemm.hip): C[M, N] = A[M, K] . B[N, K]^T (+ bias) (GELU)
    with bf16 A and B (K contiguous, row strides lda / ldb), fp32 bias [N], C
    bf16 or fp32 (``out_f32``) with row stride ldc; fp32 accumulate.  N a
    multiple of 256, K of 32."""
    _check(_load().tcamd_k17_gemm(a, b, _vp(bias), c, int(M), int(N), int(K), int(lda), int(ldb), int(ldc),
                                  K17_EPI[epilogue], 1 if out_f32 else 0, _vp(stream)), "k17_gemm")


def k18_gemm(a, b, bias, c, M, N, K, lda, ldb, ldc, epilogue="none", out_f32=False, cfg=0, splits=1,
             split_stride=0, stream=None):
    """K18 (csrc/kernels/gemm_tiles.hip): the small / mid-M tiled GEMM.  As
    k17_gemm, with the tile configuration ``cfg`` (k18_cfg) and, for
    ``splits`` > 1, K split over workgroups: C is then fp32, no epilogue, and
    split z writes its partial product at C + z * split_stride (elements)."""
    _check(_load().tcamd_k18_gemm(a, b, _vp(bias), c, int(M), int(N), int(K), int(lda), int(ldb), int(ldc),
                                  K17_EPI[epilogue], 1 if out_f32 else 0, int(cfg), int(splits), int(split_stride),
                                  _vp(stream)), "k18_gemm")


def k18_cfg(cfg):
    """(tile rows, tile columns, threads, ring stages) of K18 configuration ``cfg``, or None past the table."""
    v = [ctypes.c_int(0) for _ in range(4)]
    if _load().tcamd_k18_cfg(int(cfg), *[ctypes.byref(x) for x in v]) != 0:
        return None
    return tuple(x.value for x in v)


def k18_calls():
    """K18 launches so far in this process."""
    return int(_load().tcamd_k18_calls())


def qa_head(x, w, b, start, end, rows, H, f32=False, stream=None):
    """BERT's span head: start[r] = x[r] . w[0] + b[0], end[r] = x[r] . w[1] +
    b[1] in fp32; x [rows][H] and w [2][H] bf16 (or fp32 with ``f32``), b fp32 [2]."""
    _check(_load().tcamd_qa_head(x, w, b, start, end, int(rows), int(H), 1 if f32 else 0, _vp(stream)), "qa_head")


def add_layernorm_parts(x, parts, nparts, pstride, bias, gamma, beta, out, rows, H, eps, f32=False, stream=None,
                        out3=None):
    """K11p: out = LayerNorm(x + bias + sum of ``nparts`` fp32 partial slabs
    (``parts`` + z * ``pstride`` elements, [rows][H] each)) * gamma + beta.
    bias fp32 [H] or None; x / gamma / beta / out bf16, or fp32 with ``f32``.
    ``out3`` (f32 only, or None): the output also as a bf16x3 GEMM operand,
    bf16 [rows][3H] = [hi | hi | lo] (x3_cat's layout)."""
    _check(_load().tcamd_add_layernorm_parts3(x, _vp(parts), int(nparts), int(pstride), _vp(bias), gamma, beta, out,
                                              _vp(out3), int(rows), int(H), float(eps), 1 if f32 else 0, _vp(stream)),
           "add_layernorm_parts")


def k17_last_tm():
    """Tile height (128 / 256) the last k17_gemm picked (TCAMD_K17_TM forces one)."""
    return int(_load().tcamd_k17_last_tm())


def k17_calls():
    """K17 launches so far in this process."""
    return int(_load().tcamd_k17_calls())


def knobs():
    """The native knob registry (csrc/runtime/knobs.hip): {name: {"default",
    "value", "doc"}} -- every tuning / diagnostic switch the kernels' host
    entry points read, seeded from the environment variable of that name."""
    lib_ = _load()
    out = {}
    for i in range(lib_.tcamd_knob_count()):
        name, doc = ctypes.c_char_p(), ctypes.c_char_p()
        d, v = ctypes.c_longlong(), ctypes.c_longlong()
        if lib_.tcamd_knob_info(i, ctypes.byref(name), ctypes.byref(d), ctypes.byref(v), ctypes.byref(doc)) == 0:
            out[name.value.decode()] = {"default": d.value, "value": v.value, "doc": doc.value.decode()}
    return out


def knob_set(name, value):
    """Sets a native knob for this process (read at each launch; a captured HIP
    graph keeps what it captured); returns the previous value."""
    prev = ctypes.c_longlong()
    if _load().tcamd_knob_set(name.encode(), int(value), ctypes.byref(prev)) != 0:
        raise KeyError("unknown native knob %r (known: %s)" % (name, ", ".join(sorted(knobs()))))
    return prev.value


@contextlib.contextmanager
def knob(**settings):
    """``with hip.knob(TCAMD_X3_WS=0): ...`` -- native knobs set for the block, restored after."""
    prev = {}
    try:
        for k, v in settings.items():
            prev[k] = knob_set(k, v)
        yield
    finally:
        for k, v in prev.items():
            knob_set(k, v)


def index_bytes(buf_ptr, nbytes, n_expected, offs_ptr, lens_ptr, status_ptr, stream=None):
    """K3: device BYTES index (offsets/lengths of each element).  Synchronises
    ``stream`` (it reads its own status to size the scan window)."""
    _check(
        _load().tcamd_index_bytes(
            _vp(buf_ptr), nbytes, n_expected, _vp(offs_ptr), _vp(lens_ptr), _vp(status_ptr), _vp(stream)
        ),
        "index_bytes",
    )


class PtrGraphExecutor:
    """Native per-batch dispatch for a pointer-table graph model
    (csrc/runtime/graph_exec.hip): the server's C++ batcher calls
    ``fn_address`` with ``handle`` directly, so no Python runs per batch.

    ``bind(i, stream, graph_execs, tbl_dev, stage_dev, out_dev, pad_ptrs)``
    hands instance ``i`` its HIP stream, one graph exec per bucket, the
    engine's device row-pointer table, a device staging area for host rows,
    the graph's output buffer and per-row padding pointers."""

    STAT_KEYS = ("batches", "prep_ns", "enqueue_ns", "wait_ns", "post_ns", "total_ns", "rows")

    def __init__(self, device, instances, in_row_bytes, out_row_bytes, buckets):
        lib = _load()
        self.buckets = [int(b) for b in buckets]
        self.max_rows = max(self.buckets)
        err = ctypes.create_string_buffer(512)
        arr = (ctypes.c_int32 * len(self.buckets))(*self.buckets)
        h = lib.tcamd_pgx_create(int(device), int(instances), int(in_row_bytes), int(out_row_bytes),
                                 len(self.buckets), arr, err, 512)
        if not h:
            raise RuntimeError(err.value.decode(errors="replace"))
        self.handle = h

    def bind(self, i, stream, graph_execs, tbl_dev, stage_dev, out_dev, pad_ptrs):
        if len(graph_execs) != len(self.buckets) or len(pad_ptrs) < self.max_rows:
            raise ValueError("one graph exec per bucket and max_rows padding pointers are required")
        err = ctypes.create_string_buffer(512)
        ge = (ctypes.c_uint64 * len(graph_execs))(*[int(g) for g in graph_execs])
        pad = (ctypes.c_uint64 * self.max_rows)(*[int(p) for p in pad_ptrs[:self.max_rows]])
        rc = _load().tcamd_pgx_set_instance(self.handle, int(i), _vp(stream), ge, int(tbl_dev), int(stage_dev),
                                            int(out_dev), pad, err, 512)
        if rc != 0:
            raise RuntimeError(err.value.decode(errors="replace"))

    @property
    def fn_address(self):
        return ctypes.cast(_load().tcamd_pgx_execute, ctypes.c_void_p).value

    def execute(self, instance, batch_ptr):
        """Run one tcserve_batch (a ctypes pointer/address) on ``instance``."""
        err = ctypes.create_string_buffer(1024)
        rc = _load().tcamd_pgx_execute(self.handle, int(instance), batch_ptr, err, 1024)
        if rc != 0:
            raise RuntimeError(err.value.decode(errors="replace"))

    def stats(self):
        out = (ctypes.c_uint64 * len(self.STAT_KEYS))()
        _load().tcamd_pgx_stats(self.handle, out)
        return dict(zip(self.STAT_KEYS, [int(v) for v in out]))

    def close(self):
        if self.handle:
            _load().tcamd_pgx_destroy(self.handle)
            self.handle = None


def available():
    """True if the library loads and at least one GPU is visible."""
    try:
        _load()
    except Exception:
        return False
    return device_count() > 0


# eager load so a missing .so fails at import time (loudly) on GPU boxes
if os.environ.get("TCAMD_LAZY_HIP", "0") != "1":
    try:
        _load()
    except OSError as e:  # pragma: no cover
        print("warning: libtcamd_hip.so failed to load: %s" % e, file=sys.stderr)
        raise
