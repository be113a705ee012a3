"""Wire bytes of a DLPack tensor for ``InferInput.set_data_from_dlpack``.

MI355X extension (the reference's InferInput only takes numpy,
``tritonclient/http/_infer_input.py:106-214``): a GPU-resident tensor — a
torch ROCm tensor, a HIP-shm ``SharedMemoryTensor``, anything exporting
``__dlpack__`` — becomes the binary tensor payload of a request without a
numpy round trip on the host:

* same element type as the wire datatype: one D2H copy;
* an FP32 tensor for a BF16 / FP16 / FP8 input: converted on the GPU first
  (K4/K5, ``csrc/kernels/convert.hip``; BF16 by truncation, byte-identical to
  ``serialize_bf16_tensor``), so only the narrow bytes cross PCIe;
* host (CPU) DLPack tensors go through ``np.from_dlpack`` and the numpy path.
"""

import numpy as np

from . import _dlpack, raise_error

_NARROW = ("BF16", "FP16", "FP8_E4M3", "FP8_E5M2")


def wire_bytes(tensor, datatype, shape):
    """Serialised bytes of ``tensor`` for an input of ``datatype`` / ``shape``."""
    dev = _dlpack.get_dlpack_device(tensor)
    if dev is None or dev[0] not in (_dlpack.kDLROCM, _dlpack.kDLCUDA):
        from tritonclient.http._infer_input import _check_dtype_shape, _raw_bytes

        arr = np.from_dlpack(tensor)
        _check_dtype_shape(datatype, shape, arr)
        return _raw_bytes(datatype, arr)
    if datatype == "BYTES":
        raise_error("BYTES inputs cannot be taken from a device tensor")
    from triton_client_amd.ops import dtypes, hip

    from . import _hip_device

    ctx = _hip_device.context(dev[1])
    with ctx.lock:
        t = _dlpack.consume(tensor, stream=ctx.stream.handle)
        try:
            if not t.is_contiguous():
                raise_error("DLPack tensor is not contiguous (only C-order tensors are supported)")
            if [int(d) for d in t.shape] != [int(d) for d in shape]:
                raise_error("got unexpected tensor shape %s, expected %s" % (list(t.shape), list(shape)))
            n = 1
            for d in t.shape:
                n *= int(d)
            out = np.empty(n * dtypes.SIZES.get(datatype, t.itemsize), dtype=np.uint8)
            if t.datatype == datatype:
                if out.size:
                    hip.memcpy_async(out.ctypes.data, t.data_ptr, out.size, ctx.stream.handle)
            elif datatype in _NARROW and t.datatype == "FP32":
                if n:
                    src = t.data_ptr
                    if src % 16:
                        tmp = ctx.scratch(4 * n + out.size + 256)
                        hip.memcpy_async(tmp, src, 4 * n, ctx.stream.handle)
                        src = tmp
                        dst = tmp + ((4 * n + 255) & ~255)
                    else:
                        dst = ctx.scratch(out.size + 16)
                    hip.convert(src, "FP32", dst, datatype, n, "trunc", ctx.stream.handle)
                    hip.memcpy_async(out.ctypes.data, dst, out.size, ctx.stream.handle)
            else:
                raise_error("got unexpected datatype %s from the DLPack tensor, expected %s" % (t.datatype, datatype))
            ctx.stream.synchronize()
        finally:
            t.release()
    return out.tobytes()
