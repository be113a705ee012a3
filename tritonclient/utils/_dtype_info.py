"""Datatype tables shared by the DLPack layer and the native ops."""

from . import _dlpack_codes as _c

# triton dtype -> (DLPack type code, bits)
DLPACK_CODES = {
    "BOOL": (_c.kDLBool, 8),
    "INT8": (_c.kDLInt, 8),
    "INT16": (_c.kDLInt, 16),
    "INT32": (_c.kDLInt, 32),
    "INT64": (_c.kDLInt, 64),
    "UINT8": (_c.kDLUInt, 8),
    "UINT16": (_c.kDLUInt, 16),
    "UINT32": (_c.kDLUInt, 32),
    "UINT64": (_c.kDLUInt, 64),
    "FP16": (_c.kDLFloat, 16),
    "FP32": (_c.kDLFloat, 32),
    "FP64": (_c.kDLFloat, 64),
    "BF16": (_c.kDLBfloat, 16),
    "FP8_E4M3": (_c.kDLFloat8_e4m3fn, 8),
    "FP8_E5M2": (_c.kDLFloat8_e5m2, 8),
}

DLPACK_REVERSE = {v: k for k, v in DLPACK_CODES.items()}
# Producers that encode bool as 1-bit (the reference does, _dlpack.py:170-216)
DLPACK_REVERSE[(_c.kDLBool, 1)] = "BOOL"
DLPACK_REVERSE[(_c.kDLUInt, 1)] = "BOOL"
