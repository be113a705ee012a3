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
* one cached HIP stream and a grow-only device scratch per device
  (``tritonclient/utils/_hip_device.py``) instead of a stream per call;
* extras, all opt-in and on the GPU:
  - ``offset`` arguments;
  - ``set_shared_memory_region(..., serialize_bytes=True)``: BYTES tensors
    serialised by K2 inside the region (fixed-width ``np.bytes_`` arrays with
    no host join at all);
  - ``set_shared_memory_region(..., datatype="BF16"|"FP16"|"FP8_E4M3"|"FP8_E5M2")``:
    float arrays converted by K4/K5 on the way in (BF16 by truncation, the
    wire format of ``serialize_bf16_tensor``);
  - ``get_contents_as_numpy(..., datatype=...)``: a BF16/FP16/FP8 region read
    back as float32, widened on the device;
  - ``fill_synthetic_data`` (K1 Philox).

BYTES semantics are the reference's (``__init__.py:199-231``): an object array
is the output of ``serialize_byte_tensor`` (its bytes are copied as-is; a
multi-element object array is concatenated, like the system-shm module) and an
``np.bytes_`` array is copied raw (``size * itemsize`` bytes).
"""

import base64
import os

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
    """Raw bytes of one input per the reference semantics (no serialisation)."""
    v = np.ascontiguousarray(v)
    if v.dtype == np.object_:
        # the output of serialize_byte_tensor: 0-d / 1-element wrapper of bytes
        raw = v.item() if v.size == 1 else b"".join(v.ravel().tolist())
        return np.frombuffer(raw, dtype=np.uint8)
    return v.reshape(-1).view(np.uint8)  # np.bytes_ too: size * itemsize raw bytes


# bytes_path="auto" for BYTES tensors (measured with tools/bytes_crossover.py
# on MI355X, mean string length 20: profiles/r4_bytes_crossover.md):
# * set: up to _BYTES_HOST_MAX elements the C++ host codec packs the stream
#   and one H2D copies it; above it K2 packs on the device.  The host wins up
#   to 4096 elements (413 vs 442 us), K2 from 16384 on (1.67 vs 1.78 ms) and by
#   ~12% at 1e6.
# * get: the host walk over a prefix copied D2H won at every size measured
#   (16 .. 1e6 elements: the K3 path needs the same D2H of the span plus three
#   stream syncs and the offsets / lengths copies), so "auto" always walks on
#   the host unless _BYTES_GET_DEVICE_MIN is set; "device" still runs K3.
# TCAMD_BYTES_HOST_MAX / TCAMD_BYTES_GET_DEVICE_MIN override (0 = always K2 /
# K3 above 0 elements).
_BYTES_HOST_MAX = int(os.environ.get("TCAMD_BYTES_HOST_MAX", "8192"))
_BYTES_GET_DEVICE_MIN = (int(os.environ["TCAMD_BYTES_GET_DEVICE_MIN"])
                         if os.environ.get("TCAMD_BYTES_GET_DEVICE_MIN") else None)


def _bytes_on_host(n, path, get=False):
    if path not in ("auto", "host", "device"):
        raise CudaSharedMemoryException("bytes_path must be auto, host or device")
    if path != "auto":
        return path == "host"
    if get:
        return _BYTES_GET_DEVICE_MIN is None or n < _BYTES_GET_DEVICE_MIN
    return n <= _BYTES_HOST_MAX


def _index_bytes_host(hip, src, nbytes, n, dev):
    """Host walk of the ``<u32 len>||bytes`` chain at device ``src`` (the
    reference's path, tc/utils/cuda_shared_memory/__init__.py:242-325, but on
    a prefix copied D2H in growing chunks, indexed by the C++ host codec).
    Returns (host bytes, offsets, lengths)."""
    from triton_client_amd.ops import host_codec

    codec = host_codec.load()
    offs = np.empty(n, dtype=np.uint64)
    lens = np.empty(n, dtype=np.uint32)
    span = min(nbytes, max(1 << 14, 32 * n))
    host = np.empty(span, dtype=np.uint8)
    have = got = pos = 0
    while True:
        if have < span:
            hip.memcpy_d2h(host[have:span], src + have, span - have, dev)
            have = span
        k, used = codec.scan_prefix(host[pos:span], offs[got:], lens[got:], n - got)
        if k:
            offs[got:got + k] += pos
        got += k
        pos += used
        if got == n:
            return host, offs, lens
        if span == nbytes:
            if pos == nbytes:
                raise CudaSharedMemoryException("the region holds %d BYTES elements, %d requested" % (got, n))
            raise CudaSharedMemoryException("BYTES element runs past the end of the region")
        want = 2 * span
        if pos + 4 <= span:  # the next element's length is known: fetch at least through it
            want = max(want, pos + 4 + int(host[pos:pos + 4].view("<u4")[0]))
        span = min(nbytes, want)
        grown = np.empty(span, dtype=np.uint8)
        grown[:have] = host[:have]
        host = grown


_NARROW = {"BF16": None, "FP16": np.float16, "FP8_E4M3": None, "FP8_E5M2": None}


def _ctx(handle):
    from .. import _hip_device

    return _hip_device.context(handle._device_id)


def _pack_bytes_on_device(hip, ctx, dst, v):
    """K2: serialise a BYTES tensor straight into device memory at ``dst``.
    ``np.bytes_`` arrays upload their fixed-width buffer as-is (element i at
    i * itemsize, lengths with trailing NULs stripped as numpy does); object
    arrays upload one joined payload.  Returns the serialised size."""
    v = np.ascontiguousarray(v)
    n = int(v.size)
    if n == 0:
        return 0
    if v.dtype.type == np.bytes_:
        flat = v.reshape(-1)
        lens = np.char.str_len(flat).astype("<u4")
        payload = flat.view(np.uint8)
        stride = v.dtype.itemsize
    else:
        from tritonclient.utils import _element_bytes

        elems = _element_bytes(v)
        lens = np.fromiter((len(e) for e in elems), dtype="<u4", count=n)
        payload = np.frombuffer(b"".join(elems), dtype=np.uint8)
        stride = 0
    nbytes = int(lens.sum(dtype=np.uint64)) + 4 * n
    ws_n = hip.pack_bytes_workspace(n)
    pay_n = (max(16, payload.size) + 255) & ~255
    len_n = (4 * n + 255) & ~255
    base = ctx.scratch(pay_n + len_n + ws_n)
    d_payload, d_lens, d_ws = base, base + pay_n, base + pay_n + len_n
    if payload.size:
        hip.memcpy_async(d_payload, payload.ctypes.data, payload.size, ctx.stream.handle)
    hip.memcpy_async(d_lens, lens.ctypes.data, 4 * n, ctx.stream.handle)
    if stride:
        hip.pack_bytes_strided(d_payload, stride, d_lens, n, dst, d_ws, ctx.stream.handle)
    else:
        hip.pack_bytes(d_payload, d_lens, n, dst, d_ws, ctx.stream.handle)
    ctx.stream.synchronize()  # the host arrays above must outlive the async copies
    return nbytes


def _convert_into(hip, ctx, dst, arr, datatype):
    """K4/K5: float array -> ``datatype`` at device ``dst`` (any alignment)."""
    from triton_client_amd.ops import dtypes

    a = np.ascontiguousarray(arr, dtype=np.float32)
    n = a.size
    out_bytes = n * dtypes.SIZES[datatype]
    if n == 0:
        return 0
    src_n = (a.nbytes + 255) & ~255
    tmp = ctx.scratch(src_n + (out_bytes + 255 & ~255))
    hip.memcpy_async(tmp, a.ctypes.data, a.nbytes, ctx.stream.handle)
    if dst % 16 == 0:
        hip.convert(tmp, "FP32", dst, datatype, n, "trunc", ctx.stream.handle)
    else:  # the kernel wants 16-B aligned operands: convert in scratch, then copy
        hip.convert(tmp, "FP32", tmp + src_n, datatype, n, "trunc", ctx.stream.handle)
        hip.memcpy_async(dst, tmp + src_n, out_bytes, ctx.stream.handle)
    ctx.stream.synchronize()
    return out_bytes


def set_shared_memory_region(cuda_shm_handle, input_values, offset=0, serialize_bytes=False, datatype=None,
                             bytes_path="auto"):
    """Copy numpy arrays back-to-back into the region starting at ``offset``.

    Reference behaviour (tc/utils/cuda_shared_memory/__init__.py:173-239):
    arrays are copied as raw bytes; BYTES object arrays are expected to be the
    output of ``serialize_byte_tensor``.  Opt-in device work (MI355X):

    * ``serialize_bytes=True``: object / ``np.bytes_`` arrays are UNserialised
      BYTES tensors; K2 writes the ``<u32 len>||bytes`` stream into the region
      (up to ``_BYTES_HOST_MAX`` elements, ``bytes_path="auto"``, the host
      codec packs them and one H2D copies the stream);
    * ``datatype`` in BF16 / FP16 / FP8_E4M3 / FP8_E5M2: float arrays are
      converted on the GPU (K4/K5; BF16 truncates like serialize_bf16_tensor).
    """
    _check_handle(cuda_shm_handle)
    if not isinstance(input_values, (list, tuple)):
        raise CudaSharedMemoryException("input_values must be specified as a numpy array")
    for v in input_values:
        if not isinstance(v, np.ndarray):
            raise CudaSharedMemoryException("input_values must be specified as a list/tuple of numpy arrays")
    if datatype is not None and datatype not in _NARROW:
        raise CudaSharedMemoryException("datatype must be one of %s" % (sorted(_NARROW),))
    hip = _hip()
    from triton_client_amd.ops import dtypes

    _bytes_on_host(0, bytes_path)  # validates the argument
    plan = []  # (kind, value, nbytes)
    for v in input_values:
        is_bytes = v.dtype == np.object_ or v.dtype.type == np.bytes_
        if is_bytes and serialize_bytes:
            if v.dtype.type == np.bytes_:
                nb = int(np.char.str_len(v.reshape(-1)).sum(dtype=np.uint64)) + 4 * v.size
            else:
                from tritonclient.utils import _element_bytes

                nb = sum(len(e) for e in _element_bytes(np.ascontiguousarray(v))) + 4 * v.size
            plan.append(("k2", v, nb))
        elif datatype is not None and v.dtype.kind == "f" and v.dtype != _NARROW[datatype]:
            plan.append(("cvt", v, v.size * dtypes.SIZES[datatype]))  # float -> narrow on the GPU
        else:
            b = _as_bytes(v)
            plan.append(("copy", b, b.size))
    total = offset + sum(nb for _, _, nb in plan)
    if total > cuda_shm_handle._byte_size:
        raise CudaSharedMemoryException(
            "unable to set values in cuda shared memory: %d bytes exceed the region size %d"
            % (total, cuda_shm_handle._byte_size)
        )
    ctx = _ctx(cuda_shm_handle)
    try:
        with ctx.lock:
            cur = cuda_shm_handle._base_addr + offset
            for kind, b, nb in plan:
                if kind == "k2" and _bytes_on_host(b.size, bytes_path):
                    from tritonclient.utils import _element_bytes
                    from triton_client_amd.ops import host_codec

                    el = _element_bytes(np.ascontiguousarray(b))
                    packed = np.frombuffer(host_codec.load().pack_bytes(el, [len(e) for e in el]), dtype=np.uint8)
                    hip.memcpy_async(cur, packed.ctypes.data, packed.size, ctx.stream.handle)
                    ctx.stream.synchronize()  # `packed` must outlive the copy
                elif kind == "k2":
                    _pack_bytes_on_device(hip, ctx, cur, b)
                elif kind == "cvt":
                    _convert_into(hip, ctx, cur, b, datatype)
                elif nb:
                    hip.memcpy_async(cur, b.ctypes.data, nb, ctx.stream.handle)
                cur += nb
            ctx.stream.synchronize()
    except Exception as ex:
        raise CudaSharedMemoryException("unable to set values in cuda shared memory") from ex


def get_contents_as_numpy(cuda_shm_handle, datatype, shape, offset=0, region_datatype=None, bytes_path="auto"):
    """Copy region contents back to the host as a numpy array.

    Only the requested bytes are copied (the reference copies the whole
    region every call, tc/utils/cuda_shared_memory/__init__.py:266-276).
    BYTES: the ``<u32 len>||bytes`` chain is walked on the host over a prefix
    copied in growing chunks (``bytes_path="auto"`` / ``"host"``; measured
    faster than the device index at every size), or indexed by K3 on the
    device (``"device"``), after which only the bytes the elements span come
    back.
    ``region_datatype`` (BF16 / FP16 /
    FP8_E4M3 / FP8_E5M2) with a float32 ``datatype``: the region holds that
    narrow type and is widened to float32 on the GPU before the copy.
    """
    _check_handle(cuda_shm_handle)
    hip = _hip()
    dt = np.dtype(datatype)
    n = int(np.prod(shape)) if len(shape) else 1
    size = cuda_shm_handle._byte_size
    dev = cuda_shm_handle._device_id
    src = cuda_shm_handle._base_addr + offset
    if region_datatype is not None and region_datatype != "FP32":
        from triton_client_amd.ops import dtypes

        if region_datatype not in _NARROW or dt != np.float32:
            raise CudaSharedMemoryException("region_datatype %r needs datatype float32" % (region_datatype,))
        need = n * dtypes.SIZES[region_datatype]
        if size < offset + need:
            raise CudaSharedMemoryException(
                "The size of the shared memory region is insufficient to provide numpy array with requested size"
            )
        out = np.empty(shape, dtype=np.float32)
        if n:
            ctx = _ctx(cuda_shm_handle)
            try:
                with ctx.lock:
                    in_n = (need + 255) & ~255
                    tmp = ctx.scratch(in_n + 4 * n)
                    s = ctx.stream.handle
                    if src % 16:
                        hip.memcpy_async(tmp, src, need, s)
                        src = tmp
                    hip.convert(src, region_datatype, tmp + in_n, "FP32", n, "trunc", s)
                    hip.memcpy_async(out.ctypes.data, tmp + in_n, 4 * n, s)
                    ctx.stream.synchronize()
            except Exception as ex:
                raise CudaSharedMemoryException("failed to read cuda shared memory results") from ex
        return out
    if dt != np.object_ and dt.type != np.bytes_:
        need = n * dt.itemsize
        if size < offset + need:
            raise CudaSharedMemoryException(
                "The size of the shared memory region is insufficient to provide numpy array with requested size"
            )
        out = np.empty(shape, dtype=dt)
        if need:
            try:
                hip.memcpy_d2h(out, src, need, dev)
            except Exception as ex:
                raise CudaSharedMemoryException("failed to read cuda shared memory results") from ex
        return out
    nbytes = size - offset
    out = np.empty(n, dtype=np.object_)
    if n == 0:
        return out.reshape(shape)
    if _bytes_on_host(n, bytes_path, get=True):
        try:
            host, offs, lens = _index_bytes_host(hip, src, nbytes, n, dev)
        except CudaSharedMemoryException:
            raise
        except Exception as ex:
            raise CudaSharedMemoryException("failed to read cuda shared memory results") from ex
        mv = memoryview(host)
        out[:] = [bytes(mv[o:o + ln]) for o, ln in zip(offs.tolist(), lens.tolist())]
        return out.reshape(shape)
    ctx = _ctx(cuda_shm_handle)
    try:
        with ctx.lock:
            base = ctx.scratch(12 * n + 64)
            d_offs, d_lens = base, base + 8 * n
            d_status = (d_lens + 4 * n + 15) & ~15
            # K3 sizes its scan window from n (a small tensor in a large
            # region is not walked to the region's end) and synchronises
            hip.index_bytes(src, nbytes, n, d_offs, d_lens, d_status, ctx.stream.handle)
            status = np.empty(4, dtype=np.int32)
            hip.memcpy_async(status.ctypes.data, d_status, 16, ctx.stream.handle)
            ctx.stream.synchronize()
            if status[0] != 0:
                raise CudaSharedMemoryException(
                    "BYTES element runs past the end of the region" if status[0] < 0 else
                    "the region holds %d BYTES elements, %d requested" % (int(status[2:4].view(np.uint64)[0]), n))
            offs = np.empty(n, dtype=np.uint64)
            lens = np.empty(n, dtype=np.uint32)
            hip.memcpy_async(offs.ctypes.data, d_offs, 8 * n, ctx.stream.handle)
            hip.memcpy_async(lens.ctypes.data, d_lens, 4 * n, ctx.stream.handle)
            ctx.stream.synchronize()
    except CudaSharedMemoryException:
        raise
    except Exception as ex:
        raise CudaSharedMemoryException("failed to read cuda shared memory results") from ex
    end = int(offs[-1]) + int(lens[-1])
    host = np.empty(end, dtype=np.uint8)
    try:
        hip.memcpy_d2h(host, src, end, dev)
    except Exception as ex:
        raise CudaSharedMemoryException("failed to read cuda shared memory results") from ex
    # the span K3 indexed is on the host now: re-walking it with the host
    # codec costs a pass at memory speed and catches an index that does not
    # match the chain (then the host walk's result is returned)
    from triton_client_amd.ops import host_codec

    ho = np.empty(n, dtype=np.uint64)
    hl = np.empty(n, dtype=np.uint32)
    k, _ = host_codec.load().scan_prefix(host, ho, hl, n)
    if k != n or not (np.array_equal(ho, offs) and np.array_equal(hl, lens)):
        import warnings

        warnings.warn("hip_shared_memory: the device BYTES index disagreed with the host walk; using the host walk")
        host, offs, lens = _index_bytes_host(hip, src, nbytes, n, dev)
    mv = memoryview(host)
    out[:] = [bytes(mv[o:o + ln]) for o, ln in zip(offs.tolist(), lens.tolist())]
    return out.reshape(shape)


def set_shared_memory_region_from_dlpack(cuda_shm_handle, input_values, offset=0):
    """Copy DLPack tensors (host or ROCm device) back-to-back into the region.

    Device inputs are gathered with a single K7 ``batched_copy`` launch.
    """
    _check_handle(cuda_shm_handle)
    hip = _hip()
    ctx = _ctx(cuda_shm_handle)
    stream = ctx.stream
    ctx.lock.acquire()
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
        ctx.lock.release()


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
    ctx = _ctx(cuda_shm_handle)
    with ctx.lock:
        hip.synth_fill(cuda_shm_handle._base_addr + offset, n_elems, datatype, m, lo, hi, seed,
                       stream_id, ctx.stream.handle)
        ctx.stream.synchronize()


def set_shared_memory_region_from_fp32(cuda_shm_handle, array, datatype, offset=0, rounding="trunc"):
    """Upload an fp32 array and convert it on the GPU into ``datatype``
    (BF16 truncation by default = the wire format of serialize_bf16_tensor;
    ``rounding="rne"`` rounds to nearest even)."""
    _check_handle(cuda_shm_handle)
    hip = _hip()
    from triton_client_amd.ops import dtypes

    a = np.ascontiguousarray(array, dtype=np.float32)
    n = a.size
    out_bytes = n * dtypes.SIZES[datatype]
    if offset + out_bytes > cuda_shm_handle._byte_size:
        raise CudaSharedMemoryException("converted data exceeds the region size")
    dst = cuda_shm_handle._base_addr + offset
    if dst % 16:
        raise CudaSharedMemoryException("offset must be 16-byte aligned for device conversion")
    ctx = _ctx(cuda_shm_handle)
    with ctx.lock:
        tmp = ctx.scratch(max(a.nbytes, 16))
        hip.memcpy_async(tmp, a.ctypes.data, a.nbytes, ctx.stream.handle)
        hip.convert(tmp, "FP32", dst, datatype, n, rounding, ctx.stream.handle)
        ctx.stream.synchronize()
