"""HTTP input-tensor descriptor (reference tritonclient/http/_infer_input.py:38-272)."""
import numpy as np

from tritonclient.utils import (
    np_to_triton_dtype,
    raise_error,
    serialize_bf16_tensor,
    serialize_byte_tensor,
    serialize_fp8_tensor,
    triton_to_np_dtype,
)


def _check_dtype_shape(datatype, shape, input_tensor):
    if not isinstance(input_tensor, (np.ndarray,)):
        raise_error("input_tensor must be a numpy array")
    if datatype in ("BF16", "FP8_E4M3", "FP8_E5M2"):
        # numpy has no bf16/fp8: the host holder is float32
        if input_tensor.dtype != np.float32:
            raise_error(
                "got unexpected datatype {} from numpy array, expected {} for {} type".format(
                    input_tensor.dtype, np.dtype(np.float32), datatype
                )
            )
    else:
        dtype = np_to_triton_dtype(input_tensor.dtype)
        if datatype != dtype:
            raise_error(
                "got unexpected datatype {} from numpy array, expected {}".format(dtype, datatype)
            )
    valid = len(shape) == len(input_tensor.shape) and all(
        int(a) == int(b) for a, b in zip(shape, input_tensor.shape)
    )
    if not valid:
        raise_error(
            "got unexpected numpy array shape [{}], expected [{}]".format(
                str(input_tensor.shape)[1:-1], str(list(shape))[1:-1]
            )
        )


def _raw_bytes(datatype, input_tensor):
    if datatype == "BYTES":
        s = serialize_byte_tensor(input_tensor)
        return s.item() if s.size > 0 else b""
    if datatype == "BF16":
        s = serialize_bf16_tensor(input_tensor)
        return s.item() if s.size > 0 else b""
    if datatype in ("FP8_E4M3", "FP8_E5M2"):
        s = serialize_fp8_tensor(input_tensor, datatype)
        return s.item() if s.size > 0 else b""
    return input_tensor.tobytes()


class InferInput:
    """Describes one input tensor of an inference request.

    Parameters
    ----------
    name : str
        Input name.
    shape : list
        Input shape.
    datatype : str
        Triton datatype string (e.g. ``"FP32"``).
    """

    def __init__(self, name, shape, datatype):
        self._name = name
        self._shape = list(shape)
        self._datatype = datatype
        self._parameters = {}
        self._data = None
        self._raw_data = None

    def name(self):
        """Input name."""
        return self._name

    def datatype(self):
        """Input datatype."""
        return self._datatype

    def shape(self):
        """Input shape."""
        return self._shape

    def set_shape(self, shape):
        """Set the input shape; returns self."""
        self._shape = list(shape)
        return self

    def set_data_from_numpy(self, input_tensor, binary_data=True):
        """Attach ``input_tensor``; binary (default) or JSON ``data``."""
        _check_dtype_shape(self._datatype, self._shape, input_tensor)
        self._parameters.pop("shared_memory_region", None)
        self._parameters.pop("shared_memory_byte_size", None)
        self._parameters.pop("shared_memory_offset", None)
        if not binary_data:
            self._parameters.pop("binary_data_size", None)
            self._raw_data = None
            if self._datatype == "BF16":
                raise_error(
                    "BF16 inputs must be sent as binary data over HTTP. Please set binary_data=True"
                )
            if self._datatype in ("FP8_E4M3", "FP8_E5M2"):
                raise_error("FP8 inputs must be sent as binary data over HTTP.")
            if self._datatype == "BYTES":
                self._data = []
                obj = None
                try:
                    for obj in input_tensor.ravel(order="C").tolist():
                        if isinstance(obj, bytes):
                            self._data.append(str(obj, encoding="utf-8"))
                        else:
                            self._data.append(str(obj))
                except UnicodeDecodeError:
                    raise_error(
                        f'Failed to encode "{obj}" using UTF-8. Please use binary_data=True, if'
                        " you want to pass a byte array."
                    )
            else:
                self._data = input_tensor.ravel(order="C").tolist()
        else:
            self._data = None
            self._raw_data = _raw_bytes(self._datatype, input_tensor)
            self._parameters["binary_data_size"] = len(self._raw_data)
        return self

    def set_data_from_dlpack(self, tensor):
        """Attach a DLPack tensor (e.g. a torch ROCm tensor) as binary data.

        MI355X extension: a device tensor is copied D2H once; an FP32 device
        tensor for a BF16 / FP16 / FP8 input is narrowed on the GPU first
        (K4/K5; BF16 truncation = ``serialize_bf16_tensor``).  Returns self."""
        from tritonclient.utils._device_tensor import wire_bytes

        raw = wire_bytes(tensor, self._datatype, self._shape)
        self._parameters.pop("shared_memory_region", None)
        self._parameters.pop("shared_memory_byte_size", None)
        self._parameters.pop("shared_memory_offset", None)
        self._data = None
        self._raw_data = raw
        self._parameters["binary_data_size"] = len(raw)
        return self

    def set_shared_memory(self, region_name, byte_size, offset=0):
        """Read this input from shared-memory ``region_name`` at ``offset``."""
        self._data = None
        self._raw_data = None
        self._parameters.pop("binary_data_size", None)
        self._parameters["shared_memory_region"] = region_name
        self._parameters["shared_memory_byte_size"] = byte_size
        if offset != 0:
            self._parameters["shared_memory_offset"] = offset
        return self

    def _get_binary_data(self):
        return self._raw_data

    def _get_tensor(self):
        tensor = {"name": self._name, "shape": self._shape, "datatype": self._datatype}
        if self._parameters:
            tensor["parameters"] = self._parameters
        if self._parameters.get("shared_memory_region") is None and self._raw_data is None:
            if self._data is not None:
                tensor["data"] = self._data
        return tensor
