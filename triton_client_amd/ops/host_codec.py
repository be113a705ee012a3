"""ctypes binding of libtcamd_host.so (BYTES pack / scan on the host)."""
import ctypes
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libtcamd_host.so")


class HostCodec:
    def __init__(self, lib):
        self._lib = lib
        lib.tcamd_host_pack_bytes.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        lib.tcamd_host_pack_bytes.restype = ctypes.c_int
        lib.tcamd_host_count_bytes.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        lib.tcamd_host_count_bytes.restype = ctypes.c_int64
        lib.tcamd_host_scan_bytes.argtypes = [
            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
        ]
        lib.tcamd_host_scan_bytes.restype = ctypes.c_int64
        lib.tcamd_host_scan_bytes_prefix.argtypes = [
            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
        ]
        lib.tcamd_host_scan_bytes_prefix.restype = ctypes.c_int64

    def pack_bytes(self, elems, lens):
        payload = b"".join(elems)
        lens = np.ascontiguousarray(lens, dtype="<u4")
        out = ctypes.create_string_buffer(len(payload) + 4 * len(elems))
        self._lib.tcamd_host_pack_bytes(payload, lens.ctypes.data, len(elems), out)
        return out.raw

    def scan_bytes(self, buf):
        arr = np.frombuffer(buf, dtype=np.uint8)
        ptr = arr.ctypes.data
        n = self._lib.tcamd_host_count_bytes(ptr, arr.size)
        if n < 0:
            raise ValueError("malformed BYTES tensor: element overruns buffer")
        offs = np.empty(n, dtype=np.uint64)
        lens = np.empty(n, dtype=np.uint32)
        self._lib.tcamd_host_scan_bytes(ptr, arr.size, offs.ctypes.data, lens.ctypes.data, n)
        return offs, lens


    def scan_prefix(self, arr, offs, lens, cap):
        """Index up to ``cap`` complete elements of the uint8 array ``arr`` (a
        prefix of a BYTES stream) into ``offs`` / ``lens``; returns (count,
        bytes consumed)."""
        consumed = ctypes.c_uint64(0)
        n = self._lib.tcamd_host_scan_bytes_prefix(arr.ctypes.data, arr.size, offs.ctypes.data, lens.ctypes.data,
                                                   cap, ctypes.byref(consumed))
        return int(n), int(consumed.value)


_INSTANCE = None


def load():
    global _INSTANCE
    if _INSTANCE is None:
        _INSTANCE = HostCodec(ctypes.CDLL(_PATH))
    return _INSTANCE
