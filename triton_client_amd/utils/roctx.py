"""roctx ranges from Python (the server's model execution, the multi-GPU
fan-out), visible in ``rocprofv3 --marker-trace`` next to the kernels.

Same switch as the C++ side (csrc/cpp/src/trace.h): a no-op unless
``TC_ROCTX=1`` and a roctx library is loadable, so production paths pay one
attribute check.
"""

import contextlib
import ctypes
import os

_LIBS = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so")
_lib = None
_tried = False


def _load():
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    if os.environ.get("TC_ROCTX") != "1":
        return None
    for name in _LIBS:
        for path in (name, os.path.join("/opt/rocm/lib", name)):
            try:
                lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            except OSError:
                continue
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.argtypes = []
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            lib.roctxMarkA.restype = None
            _lib = lib
            return _lib
    return None


def enabled():
    return _load() is not None


def mark(msg):
    lib = _load()
    if lib is not None:
        lib.roctxMarkA(msg.encode())


@contextlib.contextmanager
def range(msg):  # noqa: A001 - mirrors roctxRange naming
    lib = _load()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(msg.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()
