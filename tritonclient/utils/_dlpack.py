"""Minimal DLPack (v0.8 ABI) producer/consumer over ctypes.

Capability parity with reference ``tritonclient/utils/_dlpack.py:37-272``; the
design differs: device tensors are tagged ``kDLROCM`` (the reference defines
``kDLROCM=10`` but hard-codes ``kDLCUDA`` in ``_shared_memory_tensor.py:58-62``),
FP8 maps onto DLPack 1.x float8 codes, and exported managed tensors are one
malloc'ed block freed by libc ``free`` (no Python callback on the consumer's
release path, so views may safely outlive interpreter teardown).
"""

import ctypes

from . import _dtype_info

# ---- DLPack enums ---------------------------------------------------------
kDLCPU = 1
kDLCUDA = 2
kDLCUDAHost = 3
kDLROCM = 10
kDLROCMHost = 11

kDLInt = 0
kDLUInt = 1
kDLFloat = 2
kDLBfloat = 4
kDLBool = 6
kDLFloat8_e4m3fn = 10
kDLFloat8_e5m2 = 12


class DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32)]


class DLDataType(ctypes.Structure):
    _fields_ = [
        ("type_code", ctypes.c_uint8),
        ("bits", ctypes.c_uint8),
        ("lanes", ctypes.c_uint16),
    ]


class DLTensor(ctypes.Structure):
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("device", DLDevice),
        ("ndim", ctypes.c_int32),
        ("dtype", DLDataType),
        ("shape", ctypes.POINTER(ctypes.c_int64)),
        ("strides", ctypes.POINTER(ctypes.c_int64)),
        ("byte_offset", ctypes.c_uint64),
    ]


class DLManagedTensor(ctypes.Structure):
    pass


_DELETER_T = ctypes.CFUNCTYPE(None, ctypes.POINTER(DLManagedTensor))
DLManagedTensor._fields_ = [
    ("dl_tensor", DLTensor),
    ("manager_ctx", ctypes.c_void_p),
    ("deleter", _DELETER_T),
]

_DLTENSOR_NAME = b"dltensor"
_USED_DLTENSOR_NAME = b"used_dltensor"

_api = ctypes.pythonapi
_api.PyCapsule_New.restype = ctypes.py_object
_api.PyCapsule_New.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
_api.PyCapsule_IsValid.restype = ctypes.c_int
_api.PyCapsule_IsValid.argtypes = [ctypes.py_object, ctypes.c_char_p]
_api.PyCapsule_GetPointer.restype = ctypes.c_void_p
_api.PyCapsule_GetPointer.argtypes = [ctypes.py_object, ctypes.c_char_p]
_api.PyCapsule_SetName.restype = ctypes.c_int
_api.PyCapsule_SetName.argtypes = [ctypes.py_object, ctypes.c_char_p]

# Exported managed tensors live in ONE libc-malloc'ed block:
#   [DLManagedTensor][shape int64 x ndim][strides int64 x ndim]
# and their deleter is libc ``free`` itself (``void(void*)`` is ABI-identical
# to ``void(DLManagedTensor*)``).  No Python callback is ever invoked by the
# consumer, so a tensor may outlive the interpreter's ctypes machinery (torch
# frees DLPack-imported tensors at shutdown).  An exported capsule that is
# never consumed leaks its (tiny) block; the underlying region is owned by
# the shared-memory handle, not by the view.
_libc = ctypes.CDLL(None)
_libc.malloc.restype = ctypes.c_void_p
_libc.malloc.argtypes = [ctypes.c_size_t]
_FREE_ADDR = ctypes.cast(_libc.free, ctypes.c_void_p).value


def triton_to_dlpack_dtype(dtype):
    """Triton datatype string -> DLDataType (raises on BYTES/unknown)."""
    info = _dtype_info.DLPACK_CODES.get(dtype)
    if info is None:
        raise ValueError("datatype %s has no DLPack equivalent" % dtype)
    code, bits = info
    return DLDataType(type_code=code, bits=bits, lanes=1)


def dlpack_to_triton_dtype(dl_dtype):
    """DLDataType -> Triton datatype string (None if unsupported)."""
    if dl_dtype.lanes != 1:
        return None
    return _dtype_info.DLPACK_REVERSE.get((dl_dtype.type_code, dl_dtype.bits))


def make_capsule(data_ptr, device_type, device_id, datatype, shape, byte_offset=0, owner=None):
    """Create a ``dltensor`` PyCapsule viewing ``data_ptr`` (row-major).

    ``owner`` is accepted for API symmetry; the caller keeps the region alive.
    """
    ndim = len(shape)
    head = ctypes.sizeof(DLManagedTensor)
    block = _libc.malloc(head + 16 * max(ndim, 1))
    if not block:
        raise MemoryError("DLPack: malloc failed")
    ctypes.memset(block, 0, head + 16 * max(ndim, 1))
    mt = DLManagedTensor.from_address(block)
    shape_p = block + head
    strides_p = shape_p + 8 * max(ndim, 1)
    shp = (ctypes.c_int64 * max(ndim, 1)).from_address(shape_p)
    std = (ctypes.c_int64 * max(ndim, 1)).from_address(strides_p)
    acc = 1
    for i in range(ndim - 1, -1, -1):
        shp[i] = int(shape[i])
        std[i] = acc
        acc *= int(shape[i])
    mt.dl_tensor.data = data_ptr
    mt.dl_tensor.device = DLDevice(device_type, device_id)
    mt.dl_tensor.ndim = ndim
    mt.dl_tensor.dtype = triton_to_dlpack_dtype(datatype)
    mt.dl_tensor.shape = ctypes.cast(shape_p, ctypes.POINTER(ctypes.c_int64))
    mt.dl_tensor.strides = ctypes.cast(strides_p, ctypes.POINTER(ctypes.c_int64))
    mt.dl_tensor.byte_offset = byte_offset
    mt.manager_ctx = None
    ctypes.cast(block + head - ctypes.sizeof(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p))[0] = _FREE_ADDR
    return _api.PyCapsule_New(block, _DLTENSOR_NAME, None)


class ConsumedTensor:
    """View of a consumed DLPack capsule; call :meth:`release` when done."""

    def __init__(self, capsule):
        if not _api.PyCapsule_IsValid(capsule, _DLTENSOR_NAME):
            raise ValueError("object is not an unconsumed 'dltensor' capsule")
        addr = _api.PyCapsule_GetPointer(capsule, _DLTENSOR_NAME)
        self._mt = DLManagedTensor.from_address(addr)
        _api.PyCapsule_SetName(capsule, _USED_DLTENSOR_NAME)
        t = self._mt.dl_tensor
        self.data_ptr = (t.data or 0) + t.byte_offset
        self.device_type = t.device.device_type
        self.device_id = t.device.device_id
        self.shape = [t.shape[i] for i in range(t.ndim)]
        self.strides = [t.strides[i] for i in range(t.ndim)] if t.strides else None
        self.datatype = dlpack_to_triton_dtype(t.dtype)
        self.itemsize = (t.dtype.bits * t.dtype.lanes + 7) // 8
        self._released = False

    def is_contiguous(self):
        if self.strides is None:
            return True
        acc = 1
        for d, s in zip(reversed(self.shape), reversed(self.strides)):
            if d != 1 and s != acc:
                return False
            acc *= d
        return True

    def byte_size(self):
        n = 1
        for d in self.shape:
            n *= d
        return n * self.itemsize

    def is_device(self):
        return self.device_type in (kDLROCM, kDLCUDA)

    def release(self):
        if not self._released:
            self._released = True
            if self._mt.deleter:
                self._mt.deleter(ctypes.pointer(self._mt))

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


def consume(obj, stream=None):
    """Consume ``obj`` (``__dlpack__`` provider or raw capsule)."""
    if hasattr(obj, "__dlpack__"):
        dev = get_dlpack_device(obj)
        on_device = dev is not None and dev[0] in (kDLROCM, kDLCUDA)
        try:
            # producers reject a stream argument for host tensors
            capsule = obj.__dlpack__(stream=stream) if (stream is not None and on_device) else obj.__dlpack__()
        except TypeError:
            capsule = obj.__dlpack__()
    else:
        capsule = obj
    return ConsumedTensor(capsule)


def get_dlpack_device(obj):
    if hasattr(obj, "__dlpack_device__"):
        return obj.__dlpack_device__()
    return None
