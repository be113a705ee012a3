"""DLPack view of a shared-memory region (reference utils/_shared_memory_tensor.py:34-87).

Device regions report ``kDLROCM`` (the reference hard-codes kDLCUDA), so
``torch.from_dlpack`` on ROCm builds maps them onto ``cuda:<id>`` tensors with
no copy.
"""


class SharedMemoryTensor:
    """A DLPack-exportable view of ``byte_size`` bytes at ``shm_addr+offset``.

    ``device_id == -1`` means host (system) shared memory.  The view is
    invalidated when the underlying region is destroyed.
    """

    def __init__(self, dtype, shape, shm_addr, offset, byte_size, device_id, owner=None):
        from . import _dlpack

        self._dtype = dtype
        self._shape = list(shape)
        self._shm_addr = shm_addr
        self._offset = offset
        self._byte_size = byte_size
        self._device_id = device_id
        self._owner = owner
        if device_id != -1:
            self._dl_device = (_dlpack.kDLROCM, device_id)
        else:
            self._dl_device = (_dlpack.kDLCPU, 0)

    def __dlpack__(self, stream=None):
        from . import _dlpack

        # Producer-side work on the region is synchronous (set_* calls sync
        # their stream), so there is nothing to order against ``stream``.
        return _dlpack.make_capsule(
            self._shm_addr,
            self._dl_device[0],
            self._dl_device[1],
            self._dtype,
            self._shape,
            byte_offset=self._offset,
            owner=self,
        )

    def __dlpack_device__(self):
        return self._dl_device
