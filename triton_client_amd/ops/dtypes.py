"""Datatype codes shared with csrc/kernels/common.h."""

CODES = {
    "BOOL": 0,
    "INT8": 1,
    "INT16": 2,
    "INT32": 3,
    "INT64": 4,
    "UINT8": 5,
    "UINT16": 6,
    "UINT32": 7,
    "UINT64": 8,
    "FP16": 9,
    "FP32": 10,
    "FP64": 11,
    "BF16": 12,
    "FP8_E4M3": 13,
    "FP8_E5M2": 14,
}

SIZES = {
    "BOOL": 1, "INT8": 1, "UINT8": 1, "FP8_E4M3": 1, "FP8_E5M2": 1,
    "INT16": 2, "UINT16": 2, "FP16": 2, "BF16": 2,
    "INT32": 4, "UINT32": 4, "FP32": 4,
    "INT64": 8, "UINT64": 8, "FP64": 8,
}


def code(dt):
    try:
        return CODES[dt]
    except KeyError:
        raise ValueError("unsupported datatype for device kernels: %s" % dt) from None
