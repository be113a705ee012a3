"""Server-side request/response value types.

The server is the in-repo KServe-v2 test + bench server that SURVEY.md §4
requires (the reference has none: its tests need a live Triton).  These types
are transport-neutral: the HTTP and gRPC front ends decode into them and encode
out of them, so the scheduler and backends never see wire formats.
"""

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np

from tritonclient.utils import triton_dtype_byte_size, triton_to_np_dtype


class ServerError(Exception):
    """An error carried back to the client (HTTP status / gRPC code)."""

    def __init__(self, msg, http_status=400, grpc_code="INVALID_ARGUMENT"):
        super().__init__(msg)
        self.msg = msg
        self.http_status = http_status
        self.grpc_code = grpc_code


def not_found(msg):
    return ServerError(msg, 404, "NOT_FOUND")


def unavailable(msg):
    return ServerError(msg, 503, "UNAVAILABLE")


def internal(msg):
    return ServerError(msg, 500, "INTERNAL")


@dataclass
class DeviceView:
    """A byte range of device memory (imported HIP IPC region)."""

    ptr: int
    nbytes: int
    device_id: int


@dataclass
class InputTensor:
    name: str
    datatype: str
    shape: List[int]
    # Host payload: np.ndarray (typed, BYTES as object array) — or a
    # DeviceView when the input lives in a registered device shm region.
    data: Any = None

    def numpy(self):
        if isinstance(self.data, DeviceView):
            from triton_client_amd.ops import hip

            raw = np.empty(self.data.nbytes, dtype=np.uint8)
            hip.memcpy_d2h(raw, self.data.ptr, self.data.nbytes)
            return decode_raw(raw, self.datatype, self.shape)
        return self.data

    @property
    def on_device(self):
        return isinstance(self.data, DeviceView)


@dataclass
class RequestedOutput:
    name: str
    binary: bool = True
    class_count: int = 0
    # (region name, byte_size, offset) when delivered through shared memory
    shm: Optional[tuple] = None


@dataclass
class InferRequest:
    model_name: str
    model_version: str = ""
    id: str = ""
    parameters: Dict[str, Any] = field(default_factory=dict)
    inputs: List[InputTensor] = field(default_factory=list)
    outputs: List[RequestedOutput] = field(default_factory=list)
    binary_data_output: bool = False
    # timestamps (ns) for statistics
    t_receive: int = 0

    def input(self, name):
        for t in self.inputs:
            if t.name == name:
                return t
        return None

    @property
    def sequence_id(self):
        return self.parameters.get("sequence_id", 0)

    @property
    def sequence_start(self):
        return bool(self.parameters.get("sequence_start", False))

    @property
    def sequence_end(self):
        return bool(self.parameters.get("sequence_end", False))


@dataclass
class OutputTensor:
    name: str
    datatype: str
    shape: List[int]
    # np.ndarray (host), or None when the data was written to shared memory
    data: Any = None
    shm: Optional[tuple] = None  # (region, byte_size, offset) if delivered via shm


@dataclass
class InferResponse:
    model_name: str
    model_version: str
    id: str = ""
    outputs: List[OutputTensor] = field(default_factory=list)
    parameters: Dict[str, Any] = field(default_factory=dict)
    error: Optional[str] = None
    final: bool = True


def decode_raw(raw, datatype, shape):
    """uint8 buffer -> numpy array of ``datatype`` / ``shape``."""
    from tritonclient.utils import (
        deserialize_bf16_tensor,
        deserialize_bytes_tensor,
        deserialize_fp8_tensor,
    )

    buf = raw if isinstance(raw, (bytes, bytearray, memoryview)) else raw.tobytes() if raw.dtype == np.object_ else raw
    if datatype == "BYTES":
        arr = deserialize_bytes_tensor(bytes(buf) if not isinstance(buf, bytes) else buf)
    elif datatype == "BF16":
        arr = deserialize_bf16_tensor(buf)
    elif datatype in ("FP8_E4M3", "FP8_E5M2"):
        arr = deserialize_fp8_tensor(buf, datatype)
    else:
        dt = triton_to_np_dtype(datatype)
        if dt is None:
            raise ServerError("unsupported datatype " + datatype)
        need = int(np.prod(shape)) * np.dtype(dt).itemsize if len(shape) else np.dtype(dt).itemsize
        if len(buf) != need:
            raise ServerError(
                "unexpected byte size %d for input of shape %s datatype %s (expected %d)"
                % (len(buf), list(shape), datatype, need)
            )
        arr = np.frombuffer(buf, dtype=dt)
    n = int(np.prod(shape)) if len(shape) else 1
    if arr.size != n:
        raise ServerError(
            "unexpected element count %d for shape %s" % (arr.size, list(shape))
        )
    return arr.reshape(shape)


def expected_byte_size(datatype, shape):
    sz = triton_dtype_byte_size(datatype)
    if sz is None:
        return None
    return int(np.prod(shape)) * sz if len(shape) else sz
