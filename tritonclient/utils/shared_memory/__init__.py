"""System (POSIX) shared-memory regions for zero-copy host tensors.

Same public API as reference ``tritonclient/utils/shared_memory/__init__.py``
(create/set/get_contents_as_numpy/mapped_shared_memory_regions/destroy,
``SharedMemoryException`` codes -2..-6, :93-340), backed by the native
``libcshm.so`` built from ``csrc/cshm/cshm.cc``.
"""

import ctypes
import os
import struct
from ctypes import POINTER, byref, c_char_p, c_int, c_uint64, c_void_p

import numpy as np

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcshm.so")


class _utf8:
    @classmethod
    def from_param(cls, value):
        if value is None:
            return None
        if isinstance(value, bytes):
            return value
        return value.encode("utf8")


class SharedMemoryException(Exception):
    """Exception indicating non-Success status (``err`` may be a code or str)."""

    err_code_map = {
        -2: "unable to get shared memory descriptor",
        -3: "unable to initialize the size",
        -4: "unable to read/mmap the shared memory region",
        -5: "unable to unlink the shared memory region",
        -6: "unable to munmap the shared memory region",
        -7: "requested range is outside the shared memory region",
        -8: "invalid shared memory handle",
    }

    def __init__(self, err):
        self._msg = None
        if isinstance(err, str):
            self._msg = err
        else:
            code = err.value if hasattr(err, "value") else int(err)
            self._msg = self.err_code_map.get(code)
        super().__init__(self._msg)

    def __str__(self):
        return super().__str__() if self._msg is None else self._msg


_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise SharedMemoryException(
                "libcshm.so not built; run `python __graft_entry__.py build` "
                "(or `make -C csrc`)"
            )
        lib = ctypes.CDLL(_LIB_PATH)
        lib.SharedMemoryRegionCreate.restype = c_int
        lib.SharedMemoryRegionCreate.argtypes = [_utf8, _utf8, c_uint64, POINTER(c_void_p)]
        lib.SharedMemoryRegionSet.restype = c_int
        lib.SharedMemoryRegionSet.argtypes = [c_void_p, c_uint64, c_uint64, c_void_p]
        lib.GetSharedMemoryHandleInfo.restype = c_int
        lib.GetSharedMemoryHandleInfo.argtypes = [
            c_void_p,
            POINTER(c_char_p),
            POINTER(c_char_p),
            POINTER(c_int),
            POINTER(c_uint64),
            POINTER(c_uint64),
        ]
        lib.SharedMemoryRegionDestroy.restype = c_int
        lib.SharedMemoryRegionDestroy.argtypes = [c_void_p]
        lib.SharedMemoryRegionOpen.restype = c_int
        lib.SharedMemoryRegionOpen.argtypes = [_utf8, c_uint64, c_uint64, POINTER(c_void_p)]
        lib.SharedMemoryRegionClose.restype = c_int
        lib.SharedMemoryRegionClose.argtypes = [c_void_p]
        _lib = lib
    return _lib


mapped_shm_regions = []


def _check(rc):
    if rc != 0:
        raise SharedMemoryException(c_int(rc))


def _raise_error(msg):
    raise SharedMemoryException(msg)


def _info(shm_handle):
    addr = c_char_p()
    key = c_char_p()
    fd = c_int()
    off = c_uint64()
    size = c_uint64()
    _check(
        _load().GetSharedMemoryHandleInfo(
            shm_handle, byref(addr), byref(key), byref(fd), byref(off), byref(size)
        )
    )
    base = ctypes.cast(addr, c_void_p).value or 0
    return base, key.value.decode("utf-8"), off.value, size.value


def create_shared_memory_region(triton_shm_name, shm_key, byte_size):
    """Create (or open) the POSIX region ``shm_key`` of ``byte_size`` bytes.

    Returns an opaque handle (``c_void_p``).
    """
    handle = c_void_p()
    _check(_load().SharedMemoryRegionCreate(triton_shm_name, shm_key, byte_size, byref(handle)))
    mapped_shm_regions.append(shm_key)
    return handle


def set_shared_memory_region(shm_handle, input_values, offset=0, serialize_bytes=False):
    """Copy a list of numpy arrays back-to-back into the region from ``offset``.

    Reference semantics: object arrays are the output of
    ``serialize_byte_tensor`` and are copied as-is, ``np.bytes_`` arrays are
    copied raw.  ``serialize_bytes=True`` (same option as the HIP module)
    treats object / ``np.bytes_`` arrays as UNserialised BYTES tensors and
    writes their ``<u32 len>||bytes`` form."""
    if not isinstance(input_values, (list, tuple)):
        _raise_error("input_values must be specified as a list/tuple of numpy arrays")
    for v in input_values:
        if not isinstance(v, np.ndarray):
            _raise_error("each element of input_values must be a numpy array")
    lib = _load()
    cur = offset
    for v in input_values:
        if serialize_bytes and (v.dtype == np.object_ or v.dtype.type == np.bytes_):
            from tritonclient.utils import serialize_byte_tensor

            v = serialize_byte_tensor(v) if v.size else np.empty(0, np.uint8)
            if v.dtype != np.object_:
                continue
        if v.dtype == np.object_:
            # A serialised BYTES tensor (0-d object array wrapping bytes) or a
            # flat object array of bytes produced by serialize_byte_tensor.
            raw = v.item() if v.ndim == 0 or v.size == 1 else b"".join(v.ravel().tolist())
            buf = ctypes.create_string_buffer(raw, len(raw))
            _check(lib.SharedMemoryRegionSet(shm_handle, cur, len(raw), ctypes.cast(buf, c_void_p)))
            cur += len(raw)
        else:
            c = np.ascontiguousarray(v)
            _check(lib.SharedMemoryRegionSet(shm_handle, cur, c.nbytes, c.ctypes.data_as(c_void_p)))
            cur += c.nbytes


def get_contents_as_numpy(shm_handle, datatype, shape, offset=0):
    """Zero-copy numpy view (or BYTES decode) of region contents."""
    base, _, region_off, size = _info(shm_handle)
    start = region_off + offset
    dt = np.dtype(datatype)
    n = int(np.prod(shape)) if len(shape) else 1
    if dt != np.object_ and dt.type != np.bytes_:
        need = n * dt.itemsize
        if size < start + need:
            _raise_error(
                "The size of the shared memory region is insufficient to provide "
                "numpy array with requested size"
            )
        if need == 0:
            return np.empty(shape, dtype=dt)
        buf = (ctypes.c_byte * (start + need)).from_address(base)
        return np.frombuffer(buf, dtype=dt, count=n, offset=start).reshape(shape)
    buf = (ctypes.c_byte * size).from_address(base)
    mv = memoryview(buf).cast("B")
    strs = []
    pos = start
    for _ in range(n):
        if pos + 4 > size:
            _raise_error("BYTES element runs past the end of the shared memory region")
        (ln,) = struct.unpack_from("<I", mv, pos)
        pos += 4
        if pos + ln > size:
            _raise_error("BYTES element runs past the end of the shared memory region")
        strs.append(bytes(mv[pos : pos + ln]))
        pos += ln
    out = np.empty(n, dtype=np.object_)
    out[:] = strs
    return out.reshape(shape)


def mapped_shared_memory_regions():
    """Keys of regions created by this process and not yet destroyed."""
    return mapped_shm_regions


def destroy_shared_memory_region(shm_handle):
    """Unmap + unlink the region."""
    _, key, _, _ = _info(shm_handle)
    if key in mapped_shm_regions:
        mapped_shm_regions.remove(key)
    _check(_load().SharedMemoryRegionDestroy(shm_handle))


# --- server-side helpers (not part of the reference client API) ----------
class MappedRegion:
    """An existing region mapped by key (what a server does on register)."""

    def __init__(self, key, offset, byte_size):
        self.key = key
        self.offset = offset
        self.byte_size = byte_size
        self._h = c_void_p()
        _check(_load().SharedMemoryRegionOpen(key, offset, byte_size, byref(self._h)))
        self.base, _, _, self.mapped_size = _info(self._h)

    def view(self, offset=0, nbytes=None):
        """Writable uint8 numpy view of [offset, offset+nbytes) of the region."""
        if nbytes is None:
            nbytes = self.byte_size - offset
        if offset < 0 or offset + nbytes > self.byte_size:
            raise SharedMemoryException(c_int(-7))
        start = self.offset + offset
        buf = (ctypes.c_ubyte * nbytes).from_address(self.base + start)
        return np.frombuffer(buf, dtype=np.uint8)

    def address(self, offset=0):
        return self.base + self.offset + offset

    def close(self):
        if self._h:
            _check(_load().SharedMemoryRegionClose(self._h))
            self._h = c_void_p()
