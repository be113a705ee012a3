"""Datatype maps and tensor (de)serialisers shared by every client.

API-compatible with reference ``tritonclient/utils/__init__.py:36-348``.  The
wire formats are byte-identical to the reference:

* BYTES: each element is ``<u32 little-endian length> || bytes``, row-major.
* BF16: the high 16 bits of the IEEE fp32 value (i.e. *truncation*, matching
  ``struct.pack("<f")[2:4]`` at reference ``utils/__init__.py:314``).

Unlike the reference (per-element ``np.nditer`` loops) the fixed-width codecs
here are vectorised numpy, and large BYTES tensors go through the native
``libtcamd_host`` walker when it is built.  Device-resident tensors use the
HIP kernels in :mod:`triton_client_amd.ops` instead.

FP8 (OCP ``e4m3fn`` / ``e5m2``, native on CDNA4) is **not** a KServe/Triton
datatype; it is offered as an opt-in extension (``"FP8_E4M3"`` /
``"FP8_E5M2"``) and never emitted unless a caller names it explicitly.
"""

import struct

import numpy as np

from ._shared_memory_tensor import SharedMemoryTensor  # noqa: F401


def raise_error(msg):
    """Raise :class:`InferenceServerException` with ``msg``."""
    raise InferenceServerException(msg=msg) from None


class InferenceServerException(Exception):
    """Exception indicating non-Success status.

    Parameters
    ----------
    msg : str
        A brief description of error
    status : str
        The error code
    debug_details : str
        The additional details on the error
    """

    def __init__(self, msg, status=None, debug_details=None):
        super().__init__(msg)
        self._msg = msg
        self._status = status
        self._debug_details = debug_details

    def __str__(self):
        msg = super().__str__() if self._msg is None else self._msg
        if self._status is not None:
            msg = "[" + self._status + "] " + msg
        return msg

    def message(self):
        """The message associated with this exception, or None."""
        return self._msg

    def status(self):
        """The status (error code) of the exception."""
        return self._status

    def debug_details(self):
        """Additional details for debugging, or None."""
        return self._debug_details


_NP_TO_TRITON = {
    np.dtype(np.bool_): "BOOL",
    np.dtype(np.int8): "INT8",
    np.dtype(np.int16): "INT16",
    np.dtype(np.int32): "INT32",
    np.dtype(np.int64): "INT64",
    np.dtype(np.uint8): "UINT8",
    np.dtype(np.uint16): "UINT16",
    np.dtype(np.uint32): "UINT32",
    np.dtype(np.uint64): "UINT64",
    np.dtype(np.float16): "FP16",
    np.dtype(np.float32): "FP32",
    np.dtype(np.float64): "FP64",
    np.dtype(np.object_): "BYTES",
}

_TRITON_TO_NP = {
    "BOOL": bool,
    "INT8": np.int8,
    "INT16": np.int16,
    "INT32": np.int32,
    "INT64": np.int64,
    "UINT8": np.uint8,
    "UINT16": np.uint16,
    "UINT32": np.uint32,
    "UINT64": np.uint64,
    "FP16": np.float16,
    "FP32": np.float32,
    "BF16": np.float32,  # numpy has no bfloat16; fp32 is the host holder
    "FP64": np.float64,
    "BYTES": np.object_,
}

# Opt-in FP8 extension (not part of the KServe-v2 datatype set).
FP8_DATATYPES = ("FP8_E4M3", "FP8_E5M2")

# Bytes per element for fixed-size datatypes (BYTES is variable).
_DTYPE_SIZE = {
    "BOOL": 1,
    "INT8": 1,
    "UINT8": 1,
    "INT16": 2,
    "UINT16": 2,
    "FP16": 2,
    "BF16": 2,
    "INT32": 4,
    "UINT32": 4,
    "FP32": 4,
    "INT64": 8,
    "UINT64": 8,
    "FP64": 8,
    "FP8_E4M3": 1,
    "FP8_E5M2": 1,
}


def np_to_triton_dtype(np_dtype):
    """Map a numpy dtype to its Triton datatype string (None if unsupported)."""
    try:
        dt = np.dtype(np_dtype)
    except TypeError:
        return None
    if dt.type == np.bytes_:
        return "BYTES"
    return _NP_TO_TRITON.get(dt)


def triton_to_np_dtype(dtype):
    """Map a Triton datatype string to a numpy dtype (None if unsupported)."""
    return _TRITON_TO_NP.get(dtype)


def triton_dtype_byte_size(dtype):
    """Bytes per element of a fixed-size datatype, None for BYTES/unknown."""
    return _DTYPE_SIZE.get(dtype)


def serialized_byte_size(tensor_value):
    """Total payload bytes (excluding length prefixes) of a BYTES tensor."""
    if tensor_value.dtype != np.object_:
        raise_error("The tensor_value dtype must be np.object_")
    if tensor_value.size == 0:
        return 0
    return sum(len(x) for x in tensor_value.ravel(order="C").tolist())


def _element_bytes(input_tensor):
    """Row-major list of the raw bytes of each BYTES element."""
    items = input_tensor.ravel(order="C").tolist()
    if input_tensor.dtype == np.object_:
        return [
            x if type(x) == bytes else str(x).encode("utf-8")  # noqa: E721
            for x in items
        ]
    return items  # np.bytes_ elements already come back as bytes


def serialize_byte_tensor(input_tensor):
    """Serialise a BYTES tensor into ``<u32 len>||bytes`` elements.

    Returns a 0-d ``np.object_`` array wrapping the serialised ``bytes`` (use
    ``.item()``), or an empty object array for an empty tensor — the same
    contract as reference ``utils/__init__.py:193-246``.
    """
    if input_tensor.size == 0:
        return np.empty([0], dtype=np.object_)
    if (input_tensor.dtype != np.object_) and (input_tensor.dtype.type != np.bytes_):
        raise_error("cannot serialize bytes tensor: invalid datatype")
    elems = _element_bytes(input_tensor)
    lens = np.fromiter((len(e) for e in elems), dtype="<u4", count=len(elems))
    native = _native()
    if native is not None and len(elems) >= 4096:
        flattened = native.pack_bytes(elems, lens)
    else:
        pack = struct.Struct("<I").pack
        flattened = b"".join([b for e in elems for b in (pack(len(e)), e)])
    return np.asarray(flattened, dtype=np.object_)


def deserialize_bytes_tensor(encoded_tensor):
    """Parse ``<u32 len>||bytes`` elements into a 1-D ``np.object_`` array."""
    native = _native()
    buf = memoryview(encoded_tensor).cast("B") if not isinstance(encoded_tensor, bytes) else encoded_tensor
    if native is not None and len(buf) >= 65536:
        offsets, lengths = native.scan_bytes(buf)
        mv = memoryview(buf)
        return np.array(
            [bytes(mv[o : o + n]) for o, n in zip(offsets.tolist(), lengths.tolist())],
            dtype=np.object_,
        )
    strs = []
    offset = 0
    total = len(buf)
    unpack = struct.Struct("<I").unpack_from
    while offset < total:
        (n,) = unpack(buf, offset)
        offset += 4
        if offset + n > total:
            raise_error("malformed BYTES tensor: element overruns buffer")
        strs.append(bytes(buf[offset : offset + n]))
        offset += n
    out = np.empty(len(strs), dtype=np.object_)
    out[:] = strs
    return out


def serialize_bf16_tensor(input_tensor):
    """fp32 -> bf16 by truncation; returns a 0-d object array of bytes."""
    if input_tensor.size == 0:
        return np.empty([0], dtype=np.object_)
    if input_tensor.dtype != np.float32:
        raise_error("cannot serialize bf16 tensor: invalid datatype")
    bits = np.ascontiguousarray(input_tensor).view(np.uint32).ravel()
    hi = (bits >> np.uint32(16)).astype("<u2")
    return np.asarray(hi.tobytes(), dtype=np.object_)


def deserialize_bf16_tensor(encoded_tensor):
    """bf16 bytes -> 1-D fp32 array (exact widening)."""
    hi = np.frombuffer(encoded_tensor, dtype="<u2")
    return (hi.astype(np.uint32) << np.uint32(16)).view(np.float32)


# ---------------------------------------------------------------------------
# FP8 (OCP e4m3fn / e5m2) host reference codecs — extension, opt-in.
# The device path is triton_client_amd.ops.cvt_fp8 (v_cvt_pk_fp8_f32 on gfx950);
# these numpy versions are its numerics reference.
# ---------------------------------------------------------------------------
_FP8_SPEC = {
    # name: (exp bits, mantissa bits, bias, max finite, has_inf)
    "FP8_E4M3": (4, 3, 7, 448.0, False),
    "FP8_E5M2": (5, 2, 15, 57344.0, True),
}


def _fp8_table(fmt):
    ebits, mbits, bias, _, has_inf = _FP8_SPEC[fmt]
    codes = np.arange(256, dtype=np.uint32)
    sign = np.where(codes & 0x80, -1.0, 1.0)
    e = (codes >> mbits) & ((1 << ebits) - 1)
    m = codes & ((1 << mbits) - 1)
    sub = e == 0
    val = np.where(
        sub,
        m / float(1 << mbits) * 2.0 ** (1 - bias),
        (1.0 + m / float(1 << mbits)) * 2.0 ** (e.astype(np.float64) - bias),
    )
    val = sign * val
    emax = (1 << ebits) - 1
    if has_inf:
        val = np.where((e == emax) & (m == 0), sign * np.inf, val)
        val = np.where((e == emax) & (m != 0), np.nan, val)
    else:  # e4m3fn: only S.1111.111 is NaN
        val = np.where((e == emax) & (m == (1 << mbits) - 1), np.nan, val)
    return val.astype(np.float32)


_FP8_TABLES = {}


def deserialize_fp8_tensor(encoded_tensor, fmt="FP8_E4M3"):
    """FP8 bytes -> fp32 (extension)."""
    if fmt not in _FP8_TABLES:
        _FP8_TABLES[fmt] = _fp8_table(fmt)
    codes = np.frombuffer(encoded_tensor, dtype=np.uint8)
    return _FP8_TABLES[fmt][codes]


def serialize_fp8_tensor(input_tensor, fmt="FP8_E4M3"):
    """fp32 -> FP8 with round-to-nearest-even and saturation (extension).

    Matches the saturating ``v_cvt_pk_fp8_f32`` conversion used on device: out-of-
    range finite values clamp to +/-max; NaN maps to NaN.
    """
    if fmt not in _FP8_TABLES:
        _FP8_TABLES[fmt] = _fp8_table(fmt)
    table = _FP8_TABLES[fmt]
    x = np.ascontiguousarray(input_tensor, dtype=np.float32).ravel()
    _, _, _, fmax, _ = _FP8_SPEC[fmt]
    # positive finite code values in ascending order
    pos_codes = np.array(
        [c for c in range(128) if np.isfinite(table[c])], dtype=np.uint8
    )
    pos_vals = table[pos_codes].astype(np.float64)
    ax = np.minimum(np.abs(x.astype(np.float64)), fmax)
    idx = np.searchsorted(pos_vals, ax)  # first >= ax
    idx = np.clip(idx, 1, len(pos_vals) - 1)
    lo = pos_vals[idx - 1]
    hi = pos_vals[idx]
    pick_hi = (ax - lo > hi - ax) | ((ax - lo == hi - ax) & (pos_codes[idx] % 2 == 0))
    code = np.where(pick_hi, pos_codes[idx], pos_codes[idx - 1])
    code = np.where(ax <= pos_vals[0], pos_codes[0], code).astype(np.uint8)
    code = np.where(np.signbit(x), code | 0x80, code).astype(np.uint8)
    nan_code = 0x7F
    code = np.where(np.isnan(x), nan_code, code).astype(np.uint8)
    return np.asarray(code.tobytes(), dtype=np.object_)


_NATIVE = [False, None]


def _native():
    """Optional native host codec (libtcamd_host.so); None when not built."""
    if not _NATIVE[0]:
        _NATIVE[0] = True
        try:
            from triton_client_amd.ops import host_codec

            _NATIVE[1] = host_codec.load()
        except Exception:
            _NATIVE[1] = None
    return _NATIVE[1]
