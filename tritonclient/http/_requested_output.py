"""Requested-output descriptor for the KServe-v2 JSON request header.

Behaviour contract: reference ``tritonclient/http/_requested_output.py:31-117``
(same constructor, ``set_shared_memory``/``unset_shared_memory`` semantics and
the same ``outputs[i].parameters`` keys on the wire).  Here the descriptor
keeps typed fields and renders the JSON parameters only when the request is
built, so there is no mutable dict to keep consistent between calls.
"""
from tritonclient.utils import raise_error


class InferRequestedOutput:
    """Describes one requested output tensor.

    Parameters
    ----------
    name : str
        Output tensor name.
    binary_data : bool
        Return the data in the binary section of the body (default) instead
        of as a JSON ``data`` list.  Forced off while shared memory is set.
    class_count : int
        If non-zero, request the top-``class_count`` classification results.
    """

    __slots__ = ("_name", "_binary", "_class_count", "_shm")

    def __init__(self, name, binary_data=True, class_count=0):
        self._name = name
        self._binary = binary_data
        self._class_count = class_count
        self._shm = None  # (region, byte_size, offset) while delivering into shm

    def name(self):
        """Output name."""
        return self._name

    def set_shared_memory(self, region_name, byte_size, offset=0):
        """Deliver this output into ``region_name`` (``byte_size`` bytes at ``offset``)."""
        if self._class_count != 0:
            raise_error("shared memory can't be set on classification output")
        self._shm = (region_name, byte_size, offset)

    def unset_shared_memory(self):
        """Undo :meth:`set_shared_memory`; the output comes back in the response again."""
        self._shm = None

    def _get_tensor(self):
        params = {}
        if self._class_count != 0:
            params["classification"] = self._class_count
        if self._shm is None:
            params["binary_data"] = self._binary
        else:
            region, size, offset = self._shm
            params["binary_data"] = False
            params["shared_memory_region"] = region
            params["shared_memory_byte_size"] = size
            if offset != 0:
                params["shared_memory_offset"] = offset
        return {"name": self._name, "parameters": params}
