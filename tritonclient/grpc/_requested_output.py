"""gRPC requested-output descriptor.

Behaviour contract: reference ``tritonclient/grpc/_requested_output.py:33-108``
(constructor, ``set_shared_memory``/``unset_shared_memory`` semantics and the
``InferRequestedOutputTensor.parameters`` keys on the wire).  Like the HTTP
twin (``tritonclient/http/_requested_output.py``) the descriptor keeps typed
fields; the request builder renders them straight into the request's
``outputs`` entry (``_render``), so no protobuf object lives in the
descriptor and nothing has to be popped back out of a parameter map.
"""
from tritonclient.utils import raise_error


class InferRequestedOutput:
    """Describes one requested output tensor.

    Parameters
    ----------
    name : str
        Output tensor name.
    class_count : int
        If non-zero, request the top-``class_count`` classification results.
    """

    __slots__ = ("_name", "_class_count", "_shm")

    def __init__(self, name, class_count=0):
        self._name = name
        self._class_count = int(class_count)
        self._shm = None  # (region, byte_size, offset) while delivering into shm

    def name(self):
        """Output name."""
        return self._name

    def set_shared_memory(self, region_name, byte_size, offset=0):
        """Deliver this output into ``region_name`` (``byte_size`` bytes at ``offset``)."""
        if self._class_count != 0:
            raise_error("shared memory can't be set on classification output")
        self._shm = (region_name, int(byte_size), int(offset))

    def unset_shared_memory(self):
        """Undo :meth:`set_shared_memory`; the output comes back in the response again."""
        self._shm = None

    def _render(self, tensor):
        """Fill an ``InferRequestedOutputTensor`` message (``request.outputs.add()``)."""
        tensor.name = self._name
        params = tensor.parameters
        if self._class_count != 0:
            params["classification"].int64_param = self._class_count
        if self._shm is not None:
            region, size, offset = self._shm
            params["shared_memory_region"].string_param = region
            params["shared_memory_byte_size"].int64_param = size
            if offset != 0:
                params["shared_memory_offset"].int64_param = offset
        return tensor

    def _get_tensor(self):
        """A standalone ``InferRequestedOutputTensor`` for this output."""
        from tritonclient.grpc import service_pb2

        return self._render(service_pb2.ModelInferRequest.InferRequestedOutputTensor())
