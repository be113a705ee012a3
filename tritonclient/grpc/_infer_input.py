"""gRPC input-tensor descriptor (reference tritonclient/grpc/_infer_input.py:36-219)."""
from tritonclient.grpc import service_pb2
from tritonclient.http._infer_input import _check_dtype_shape, _raw_bytes


class InferInput:
    """Describes one input tensor (holds an ``InferInputTensor`` proto)."""

    def __init__(self, name, shape, datatype):
        self._input = service_pb2.ModelInferRequest().InferInputTensor()
        self._input.name = name
        self._input.ClearField("shape")
        self._input.shape.extend(shape)
        self._input.datatype = datatype
        self._raw_content = None

    def name(self):
        """Input name."""
        return self._input.name

    def datatype(self):
        """Input datatype."""
        return self._input.datatype

    def shape(self):
        """Input shape."""
        return list(self._input.shape)

    def set_shape(self, shape):
        """Set the input shape; returns self."""
        self._input.ClearField("shape")
        self._input.shape.extend(shape)
        return self

    def set_data_from_numpy(self, input_tensor):
        """Attach ``input_tensor`` as ``raw_input_contents``; returns self."""
        _check_dtype_shape(self._input.datatype, list(self._input.shape), input_tensor)
        self._input.parameters.pop("shared_memory_region", None)
        self._input.parameters.pop("shared_memory_byte_size", None)
        self._input.parameters.pop("shared_memory_offset", None)
        self._raw_content = _raw_bytes(self._input.datatype, input_tensor)
        return self

    def set_shared_memory(self, region_name, byte_size, offset=0):
        """Read this input from shared-memory ``region_name``; returns self."""
        self._input.ClearField("contents")
        self._raw_content = None
        self._input.parameters["shared_memory_region"].string_param = region_name
        self._input.parameters["shared_memory_byte_size"].int64_param = byte_size
        if offset != 0:
            self._input.parameters["shared_memory_offset"].int64_param = offset
        return self

    def _get_tensor(self):
        return self._input

    def _get_content(self):
        return self._raw_content
