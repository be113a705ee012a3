"""Device (HIP) shared-memory regions for zero-copy GPU tensors on MI355X.

Same public API as the reference's ``tritonclient.utils.cuda_shared_memory``
(``__init__.py:107-429``) — ``create_shared_memory_region``,
``get_raw_handle``, ``set_shared_memory_region``, ``get_contents_as_numpy``,
``set_shared_memory_region_from_dlpack``, ``as_shared_memory_tensor``,
``allocated_shared_memory_regions``, ``destroy_shared_memory_region`` — built on
``hipMalloc`` + ``hipIpcGetMemHandle`` through the in-tree ``libtcamd_hip.so``
instead of cuda-python.  The 64-byte hipIpcMemHandle_t travels in the same
``raw_handle`` field the server's ``cudasharedmemory`` routes expect.

Differences by design:

* views report ``kDLROCM`` (reference hard-codes kDLCUDA);
* ``get_contents_as_numpy`` copies only the requested bytes (the reference
  copies the whole region every call, ``__init__.py:266-276``);
* several device-resident DLPack inputs are concatenated with ONE K7
  ``batched_copy`` launch instead of k memcpys;
* extras: ``offset`` arguments, ``fill_synthetic_data`` (K1 on device), and
  ``set_shared_memory_region_from_fp32(..., "BF16"|"FP16"|"FP8_*")`` which
  converts on the GPU (K4/K5) while writing the region.
"""

import base64

import numpy as np

from .. import _dlpack
from .._shared_memory_tensor import SharedMemoryTensor


class CudaSharedMemoryException(Exception):
    """Exception indicating non-Success status."""

    def __init__(self, msg):
        super().__init__(msg)
        self._msg = msg

    def __str__(self):
        return super().__str__() if self._msg is None else self._msg


HipSharedMemoryException = CudaSharedMemoryException


def _hip():
    try:
        from triton_client_amd.ops import hip
    except ImportError as e:
        raise CudaSharedMemoryException("HIP runtime library unavailable: %s" % e) from e
    return hip


class HipSharedMemoryRegion:
    """One hipMalloc'ed region exportable through an IPC handle."""

    def __init__(self, triton_shm_name, ipc_handle, base_addr, byte_size, device_id):
        self._triton_shm_name = triton_shm_name
        self._hip_shm_handle = ipc_handle
        self._base_addr = base_addr
        self._byte_size = byte_size
        self._device_id = device_id
        self._freed = False

    # reference attribute name, kept for code that pokes at it
    @property
    def _cuda_shm_handle(self):
        return self._hip_shm_handle

    def _free(self):
        if not self._freed and self._base_addr:
            self._freed = True
            try:
                _hip().free(self._device_id, self._base_addr)
            except Exception:
                pass

    def __del__(self):
        self._free()


allocated_shm_regions = []


def _check_handle(h):
    if not isinstance(h, HipSharedMemoryRegion) or h._freed:
        raise CudaSharedMemoryException("invalid or destroyed HIP shared memory handle")


def create_shared_memory_region(triton_shm_name, byte_size, device_id):
    """Allocate ``byte_size`` bytes on ``device_id`` and make them IPC-exportable."""
    hip = _hip()
    try:
        # every MI355X is UVA: hipDeviceProp_t.unifiedAddressing is not a
        # reliable probe on ROCm, so no capability check here
        ptr = hip.malloc(device_id, byte_size)
        handle = hip.ipc_get_handle(ptr)
    except CudaSharedMemoryException:
        raise
    except Exception as ex:
        raise CudaSharedMemoryException("unable to create cuda shared memory handle") from ex
    region = HipSharedMemoryRegion(triton_shm_name, handle, ptr, byte_size, device_id)
    allocated_shm_regions.append(triton_shm_name)
    return region


def get_raw_handle(cuda_shm_handle):
    """Base64 of the 64-byte IPC handle (what register_cuda_shared_memory takes)."""
    _check_handle(cuda_shm_handle)
    return base64.b64encode(cuda_shm_handle._hip_shm_handle)


def _as_bytes(v):
    v = np.ascontiguousarray(v)
    if v.dtype == np.object_ or v.dtype.type == np.bytes_:
        # a tensor already serialised with serialize_byte_tensor (0-d / 1 element)
        raw = v.item() if v.size == 1 else b"".join(v.ravel().tolist())
        return np.frombuffer(raw, dtype=np.uint8)
    return v.reshape(-1).view(np.uint8)


def _is_unserialized_bytes(v):
    """An object/bytes tensor of several elements that is NOT the output of
    serialize_byte_tensor (which is a single bytes blob)."""
    return (v.dtype == np.object_ or v.dtype.type == np.bytes_) and v.size > 1


def _pack_bytes_on_device(hip, handle, dst, elems):
    """K2: serialise a BYTES tensor straight into device memory.  The payload
    bytes and u32 lengths go H2D once; the <u32 len>||bytes stream is built by
    the pack kernel inside the region (no host-side serialisation pass)."""
    n = len(elems)
    lens = np.fromiter((len(e) for e in elems), dtype="<u4", count=n)
    payload = np.frombuffer(b"".join(elems), dtype=np.uint8)
    dev = handle._device_id
    nbytes = int(lens.sum()) + 4 * n
    ws_n = hip.pack_bytes_workspace(n)
    scratch = hip.malloc(dev, max(16, payload.size) + 4 * n + ws_n + 32)
    try:
        d_payload = scratch
        d_lens = (scratch + max(16, payload.size) + 15) & ~15
        d_ws = (d_lens + 4 * n + 15) & ~15
        if payload.size:
            hip.memcpy_h2d(d_payload, payload, payload.size, dev)
        hip.memcpy_h2d(d_lens, lens, 4 * n, dev)
        s = hip.Stream(dev)
        try:
            hip.pack_bytes(d_payload, d_lens, n, dst, d_ws, s.handle)
            s.synchronize()
        finally:
            s.close()
    finally:
        hip.free(dev, scratch)
    return nbytes


def set_shared_memory_region(cuda_shm_handle, input_values, offset=0):
    """Copy numpy arrays back-to-back into the region starting at ``offset``.

    BYTES arrays already serialised with ``serialize_byte_tensor`` are copied
    as-is (reference behaviour, tc/utils/cuda_shared_memory/__init__.py:199-231).
    An UNserialised BYTES tensor (object/bytes array of several elements) is
    serialised on the device by K2 directly into the region.
    """
    _check_handle(cuda_shm_handle)
    if not isinstance(input_values, (list, tuple)):
        raise CudaSharedMemoryException("input_values must be specified as a numpy array")
    for v in input_values:
        if not isinstance(v, np.ndarray):
            raise CudaSharedMemoryException("input_values must be specified as a list/tuple of numpy arrays")
    hip = _hip()
    from tritonclient.utils import _element_bytes

    plan = []  # (kind, payload, nbytes)
    for v in input_values:
        if _is_unserialized_bytes(v):
            elems = _element_bytes(np.ascontiguousarray(v))
            plan.append(("k2", elems, sum(len(e) for e in elems) + 4 * len(elems)))
        else:
            b = _as_bytes(v)
            plan.append(("copy", b, b.size))
    total = offset + sum(nb for _, _, nb in plan)
    if total > cuda_shm_handle._byte_size:
        raise CudaSharedMemoryException(
            "unable to set values in cuda shared memory: %d bytes exceed the region size %d"
            % (total, cuda_shm_handle._byte_size)
        )
    try:
        cur = cuda_shm_handle._base_addr + offset
        for kind, b, nb in plan:
            if kind == "k2":
                _pack_bytes_on_device(hip, cuda_shm_handle, cur, b)
            elif nb:
                hip.memcpy_h2d(cur, b, nb, cuda_shm_handle._device_id)
            cur += nb
    except Exception as ex:
        raise CudaSharedMemoryException("unable to set values in cuda shared memory") from ex


def get_contents_as_numpy(cuda_shm_handle, datatype, shape, offset=0):
    """Copy region contents back to the host as a numpy array."""
    _check_handle(cuda_shm_handle)
    hip = _hip()
    dt = np.dtype(datatype)
    n = int(np.prod(shape)) if len(shape) else 1
    size = cuda_shm_handle._byte_size
    if dt != np.object_ and dt.type != np.bytes_:
        need = n * dt.itemsize
        if size < offset + need:
            raise CudaSharedMemoryException(
                "The size of the shared memory region is insufficient to provide numpy array with requested size"
            )
        out = np.empty(shape, dtype=dt)
        if need:
            try:
                hip.memcpy_d2h(out, cuda_shm_handle._base_addr + offset, need, cuda_shm_handle._device_id)
            except Exception as ex:
                raise CudaSharedMemoryException("failed to read cuda shared memory results") from ex
        return out
    # BYTES: K3 indexes the <u32 len>||bytes chain on the device (parallel
    # block walk for large tensors), then only the bytes the elements span
    # come back to the host and are sliced without a host-side walk
    dev = cuda_shm_handle._device_id
    nbytes = size - offset
    out = np.empty(n, dtype=np.object_)
    if n == 0:
        return out.reshape(shape)
    scratch = hip.malloc(dev, 12 * n + 32)
    try:
        d_offs, d_lens = scratch, scratch + 8 * n
        d_status = (d_lens + 4 * n + 15) & ~15
        s = hip.Stream(dev)
        try:
            hip.index_bytes(cuda_shm_handle._base_addr + offset, nbytes, n, d_offs, d_lens, d_status, s.handle)
            s.synchronize()
        finally:
            s.close()
        status = np.empty(4, dtype=np.int32)
        hip.memcpy_d2h(status, d_status, 16, dev)
        if status[0] != 0:
            raise CudaSharedMemoryException(
                "BYTES element runs past the end of the region" if status[0] < 0 else
                "the region holds %d BYTES elements, %d requested" % (int(status[2:4].view(np.uint64)[0]), n))
        offs = np.empty(n, dtype=np.uint64)
        lens = np.empty(n, dtype=np.uint32)
        hip.memcpy_d2h(offs, d_offs, 8 * n, dev)
        hip.memcpy_d2h(lens, d_lens, 4 * n, dev)
    except CudaSharedMemoryException:
        raise
    except Exception as ex:
        raise CudaSharedMemoryException("failed to read cuda shared memory results") from ex
    finally:
        hip.free(dev, scratch)
    end = int(offs[-1]) + int(lens[-1])
    host = np.empty(end, dtype=np.uint8)
    try:
        hip.memcpy_d2h(host, cuda_shm_handle._base_addr + offset, end, dev)
    except Exception as ex:
        raise CudaSharedMemoryException("failed to read cuda shared memory results") from ex
    mv = memoryview(host)
    out[:] = [bytes(mv[o:o + ln]) for o, ln in zip(offs.tolist(), lens.tolist())]
    return out.reshape(shape)


def set_shared_memory_region_from_dlpack(cuda_shm_handle, input_values, offset=0):
    """Copy DLPack tensors (host or ROCm device) back-to-back into the region.

    Device inputs are gathered with a single K7 ``batched_copy`` launch.
    """
    _check_handle(cuda_shm_handle)
    hip = _hip()
    stream = hip.Stream(cuda_shm_handle._device_id)
    try:
        consumed = []
        for v in input_values:
            dev = _dlpack.get_dlpack_device(v)
            if dev is not None and dev[0] not in (_dlpack.kDLCPU, _dlpack.kDLROCM, _dlpack.kDLCUDA,
                                                  _dlpack.kDLROCMHost, _dlpack.kDLCUDAHost):
                raise CudaSharedMemoryException("DLPack device type {} is not supported".format(dev[0]))
            t = _dlpack.consume(v, stream=stream.handle)
            if not t.is_contiguous():
                t.release()
                raise CudaSharedMemoryException(
                    "DLPack tensor is not contiguous. Only contiguous DLPack tensors that are stored "
                    "in C-Order are supported."
                )
            consumed.append(t)
        total = offset + sum(t.byte_size() for t in consumed)
        if total > cuda_shm_handle._byte_size:
            raise CudaSharedMemoryException("inputs exceed the shared memory region size")
        srcs, dsts, sizes = [], [], []
        cur = cuda_shm_handle._base_addr + offset
        for t in consumed:
            nbytes = t.byte_size()
            if t.is_device():
                srcs.append(t.data_ptr)
                dsts.append(cur)
                sizes.append(nbytes)
            else:
                hip.memcpy_async(cur, t.data_ptr, nbytes, stream.handle)
            cur += nbytes
        if srcs:
            hip.batched_copy(srcs, dsts, sizes, stream.handle)
        stream.synchronize()
        for t in consumed:
            t.release()
    except CudaSharedMemoryException:
        raise
    except Exception as ex:
        raise CudaSharedMemoryException("unable to set values in cuda shared memory") from ex
    finally:
        stream.close()


def as_shared_memory_tensor(cuda_shm_handle, datatype, shape, offset=0):
    """A DLPack (kDLROCM) view of the region, e.g. for ``torch.from_dlpack``."""
    _check_handle(cuda_shm_handle)
    return SharedMemoryTensor(
        datatype,
        shape,
        cuda_shm_handle._base_addr,
        offset,
        cuda_shm_handle._byte_size,
        cuda_shm_handle._device_id,
    )


def allocated_shared_memory_regions():
    """Names of regions created by this process and not yet destroyed."""
    return allocated_shm_regions


def destroy_shared_memory_region(cuda_shm_handle):
    """Free the region (outstanding server registrations become invalid)."""
    _check_handle(cuda_shm_handle)
    if cuda_shm_handle._triton_shm_name in allocated_shm_regions:
        allocated_shm_regions.remove(cuda_shm_handle._triton_shm_name)
    cuda_shm_handle._free()


# ---------------------------------------------------------------------------
# MI355X extras (device-side data preparation)
# ---------------------------------------------------------------------------
def fill_synthetic_data(cuda_shm_handle, datatype, n_elems, mode="random", lo=0.0, hi=1.0,
                        seed=0, stream_id=0, offset=0):
    """Fill the region on the GPU with K1 (Philox) data: mode random|zero|constant|normal."""
    _check_handle(cuda_shm_handle)
    hip = _hip()
    from triton_client_amd.ops import dtypes

    if offset + n_elems * dtypes.SIZES[datatype] > cuda_shm_handle._byte_size:
        raise CudaSharedMemoryException("synthetic data exceeds the region size")
    m = {"zero": hip.SYNTH_ZERO, "constant": hip.SYNTH_CONST, "random": hip.SYNTH_UNIFORM,
         "normal": hip.SYNTH_NORMAL}[mode]
    s = hip.Stream(cuda_shm_handle._device_id)
    try:
        hip.synth_fill(cuda_shm_handle._base_addr + offset, n_elems, datatype, m, lo, hi, seed,
                       stream_id, s.handle)
        s.synchronize()
    finally:
        s.close()


def set_shared_memory_region_from_fp32(cuda_shm_handle, array, datatype, offset=0, rounding="trunc"):
    """Upload an fp32 array and convert it on the GPU into ``datatype``
    (BF16 truncation by default = the wire format of serialize_bf16_tensor)."""
    _check_handle(cuda_shm_handle)
    hip = _hip()
    from triton_client_amd.ops import dtypes

    a = np.ascontiguousarray(array, dtype=np.float32)
    n = a.size
    out_bytes = n * dtypes.SIZES[datatype]
    if offset + out_bytes > cuda_shm_handle._byte_size:
        raise CudaSharedMemoryException("converted data exceeds the region size")
    dev = cuda_shm_handle._device_id
    tmp = hip.malloc(dev, max(a.nbytes, 16))
    s = hip.Stream(dev)
    try:
        hip.memcpy_h2d(tmp, a, a.nbytes, dev)
        dst = cuda_shm_handle._base_addr + offset
        if dst % 16:
            raise CudaSharedMemoryException("offset must be 16-byte aligned for device conversion")
        hip.convert(tmp, "FP32", dst, datatype, n, rounding, s.handle)
        s.synchronize()
    finally:
        s.close()
        hip.free(dev, tmp)
