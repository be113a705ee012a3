"""HTTP inference result (reference tritonclient/http/_infer_result.py:41-242)."""
import gzip
import json
import zlib

import numpy as np

from tritonclient.utils import (
    deserialize_bf16_tensor,
    deserialize_bytes_tensor,
    deserialize_fp8_tensor,
    raise_error,
    triton_to_np_dtype,
)


class _BodyReader:
    """Adapter giving a bytes-like body the ``get``/``read`` response interface."""

    def __init__(self, body, header_length=None, content_encoding=None):
        self._body = body
        self._pos = 0
        self._hdrs = {
            "inference-header-content-length": header_length,
            "content-encoding": content_encoding,
        }

    def get(self, key):
        return self._hdrs.get(key.lower())

    def read(self, length=-1):
        if length is None or length < 0:
            out = self._body[self._pos :]
            self._pos = len(self._body)
            return out
        start = self._pos
        self._pos += length
        return self._body[start : self._pos]


class InferResult:
    """Holds one inference response.

    ``response`` is any object with ``get(header)`` and ``read(length=-1)``.
    """

    def __init__(self, response, verbose):
        header_length = response.get("Inference-Header-Content-Length")
        content_encoding = response.get("Content-Encoding")
        if content_encoding is not None:
            if content_encoding == "gzip":
                response = _BodyReader(gzip.decompress(bytes(response.read())))
            elif content_encoding == "deflate":
                response = _BodyReader(zlib.decompress(bytes(response.read())))
        self._output_name_to_buffer_map = {}
        self._buffer = b""
        if header_length is None:
            content = response.read()
            if verbose:
                print(content)
            try:
                self._result = json.loads(bytes(content))
            except UnicodeDecodeError as e:
                raise_error(
                    "Failed to encode using UTF-8. Please use binary_data=True, if"
                    f" you want to pass a byte array. UnicodeError: {e}"
                )
        else:
            header_length = int(header_length)
            content = response.read(header_length)
            if verbose:
                print(content)
            self._result = json.loads(bytes(content))
            self._buffer = response.read()
            index = 0
            for output in self._result.get("outputs", []):
                params = output.get("parameters")
                if params is not None:
                    size = params.get("binary_data_size")
                    if size is not None:
                        self._output_name_to_buffer_map[output["name"]] = index
                        index += size

    @classmethod
    def from_response_body(cls, response_body, verbose=False, header_length=None, content_encoding=None):
        """Build an InferResult from a raw response body."""
        return cls(_BodyReader(response_body, header_length, content_encoding), verbose)

    def as_numpy(self, name):
        """Output ``name`` as a numpy array (None if absent)."""
        for output in self._result.get("outputs") or []:
            if output["name"] != name:
                continue
            datatype = output["datatype"]
            params = output.get("parameters")
            size = params.get("binary_data_size") if params is not None else None
            if size is not None:
                if size == 0:
                    arr = np.empty(0, dtype=triton_to_np_dtype(datatype) or np.uint8)
                else:
                    start = self._output_name_to_buffer_map[name]
                    chunk = self._buffer[start : start + size]
                    if datatype == "BYTES":
                        arr = deserialize_bytes_tensor(chunk)
                    elif datatype == "BF16":
                        arr = deserialize_bf16_tensor(chunk)
                    elif datatype in ("FP8_E4M3", "FP8_E5M2"):
                        arr = deserialize_fp8_tensor(chunk, datatype)
                    else:
                        arr = np.frombuffer(chunk, dtype=triton_to_np_dtype(datatype))
            elif "data" in output:
                arr = np.array(output["data"], dtype=triton_to_np_dtype(datatype))
            else:
                return None  # delivered through shared memory: no payload in the body
            return arr.reshape(output["shape"])
        return None

    def get_output(self, name):
        """The JSON dict of output ``name`` (None if absent)."""
        for output in self._result.get("outputs") or []:
            if output["name"] == name:
                return output
        return None

    def get_response(self):
        """The full response JSON dict."""
        return self._result
