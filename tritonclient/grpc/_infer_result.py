"""gRPC inference result (reference tritonclient/grpc/_infer_result.py:34-158).

Fixes the reference bug where ``get_output(name, as_json=True)`` returned None
(its MessageToJson result was discarded, ``_infer_result.py:99-131``).
"""
import json

import numpy as np
from google.protobuf.json_format import MessageToJson

from tritonclient.utils import (
    deserialize_bf16_tensor,
    deserialize_bytes_tensor,
    deserialize_fp8_tensor,
    triton_to_np_dtype,
)

_TYPED = {
    "BOOL": "bool_contents",
    "INT8": "int_contents",
    "INT16": "int_contents",
    "INT32": "int_contents",
    "INT64": "int64_contents",
    "UINT8": "uint_contents",
    "UINT16": "uint_contents",
    "UINT32": "uint_contents",
    "UINT64": "uint64_contents",
    "FP32": "fp32_contents",
    "FP64": "fp64_contents",
    "BYTES": "bytes_contents",
}


class InferResult:
    """Wraps a ``ModelInferResponse``."""

    def __init__(self, result):
        self._result = result

    def as_numpy(self, name):
        """Output ``name`` as numpy (None if absent)."""
        index = 0
        for output in self._result.outputs:
            if output.name == name:
                shape = list(output.shape)
                datatype = output.datatype
                if index < len(self._result.raw_output_contents):
                    raw = self._result.raw_output_contents[index]
                    if datatype == "BYTES":
                        arr = deserialize_bytes_tensor(raw)
                    elif datatype == "BF16":
                        arr = deserialize_bf16_tensor(raw)
                    elif datatype in ("FP8_E4M3", "FP8_E5M2"):
                        arr = deserialize_fp8_tensor(raw, datatype)
                    else:
                        arr = np.frombuffer(raw, dtype=triton_to_np_dtype(datatype))
                else:
                    field = _TYPED.get(datatype)
                    values = getattr(output.contents, field) if field else []
                    if len(values):
                        if datatype == "BYTES":
                            arr = np.empty(len(values), dtype=np.object_)
                            arr[:] = list(values)
                        else:
                            arr = np.array(values, dtype=triton_to_np_dtype(datatype))
                    elif "shared_memory_region" in output.parameters:
                        return None  # delivered through shared memory
                    else:
                        arr = np.empty(0)
                return arr.reshape(shape)
            index += 1
        return None

    def get_output(self, name, as_json=False):
        """The ``InferOutputTensor`` (or its JSON dict) for ``name``."""
        for output in self._result.outputs:
            if output.name == name:
                if as_json:
                    return json.loads(MessageToJson(output, preserving_proto_field_name=True))
                return output
        return None

    def get_response(self, as_json=False):
        """The full ``ModelInferResponse`` (or its JSON dict)."""
        if as_json:
            return json.loads(MessageToJson(self._result, preserving_proto_field_name=True))
        return self._result
