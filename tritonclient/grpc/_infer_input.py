"""gRPC input-tensor descriptor.

Behaviour contract: reference ``tritonclient/grpc/_infer_input.py:36-219``
(constructor, accessors, ``set_data_from_numpy`` validation and BYTES / BF16
serialisation, ``set_shared_memory``).  The descriptor keeps typed fields —
name, datatype, shape, the serialised raw bytes or the shared-memory
placement — and the request builder renders them into the request's
``inputs`` entry (``_render``); the raw bytes go to ``raw_input_contents``
without passing through an intermediate protobuf.  Validation and
serialisation are shared with the HTTP descriptor
(``tritonclient/http/_infer_input.py``).
"""
from tritonclient.http._infer_input import _check_dtype_shape, _raw_bytes


class InferInput:
    """Describes one input tensor of an inference request.

    Parameters
    ----------
    name : str
        Input tensor name.
    shape : list of int
        Input shape.
    datatype : str
        KServe datatype string (``"FP32"``, ``"BYTES"``, ...).
    """

    __slots__ = ("_name", "_shape", "_datatype", "_raw", "_shm")

    def __init__(self, name, shape, datatype):
        self._name = name
        self._shape = [int(d) for d in shape]
        self._datatype = datatype
        self._raw = None  # serialised tensor bytes (raw_input_contents)
        self._shm = None  # (region, byte_size, offset)

    def name(self):
        """Input name."""
        return self._name

    def datatype(self):
        """Input datatype."""
        return self._datatype

    def shape(self):
        """Input shape."""
        return list(self._shape)

    def set_shape(self, shape):
        """Set the input shape; returns self."""
        self._shape = [int(d) for d in shape]
        return self

    def set_data_from_numpy(self, input_tensor):
        """Serialise ``input_tensor`` as this input's ``raw_input_contents``
        (BYTES length-prefixed, BF16 truncated); clears any shared-memory
        placement.  Returns self."""
        _check_dtype_shape(self._datatype, self._shape, input_tensor)
        self._shm = None
        self._raw = _raw_bytes(self._datatype, input_tensor)
        return self

    def set_data_from_dlpack(self, tensor):
        """Attach a DLPack tensor (e.g. a torch ROCm tensor) as raw content.

        MI355X extension: a device tensor is copied D2H once; an FP32 device
        tensor for a BF16 / FP16 / FP8 input is narrowed on the GPU first
        (K4/K5; BF16 truncation = ``serialize_bf16_tensor``).  Returns self."""
        from tritonclient.utils._device_tensor import wire_bytes

        self._raw = wire_bytes(tensor, self._datatype, self._shape)
        self._shm = None
        return self

    def set_shared_memory(self, region_name, byte_size, offset=0):
        """Read this input from shared-memory ``region_name`` (``byte_size``
        bytes at ``offset``) instead of the request body.  Returns self."""
        self._raw = None
        self._shm = (region_name, int(byte_size), int(offset))
        return self

    def _render(self, tensor):
        """Fill an ``InferInputTensor`` message (``request.inputs.add()``)."""
        tensor.name = self._name
        tensor.datatype = self._datatype
        tensor.shape.extend(self._shape)
        if self._shm is not None:
            region, size, offset = self._shm
            params = tensor.parameters
            params["shared_memory_region"].string_param = region
            params["shared_memory_byte_size"].int64_param = size
            if offset != 0:
                params["shared_memory_offset"].int64_param = offset
        return tensor

    def _get_tensor(self):
        """A standalone ``InferInputTensor`` for this input."""
        from tritonclient.grpc import service_pb2

        return self._render(service_pb2.ModelInferRequest.InferInputTensor())

    def _get_content(self):
        """Serialised bytes for ``raw_input_contents`` (None with shared memory)."""
        return self._raw
