"""ctypes binding of the native perf engine (csrc/cpp/perf, libperfanalyzer.so).

``PerfSession(args)`` takes perf_analyzer command-line flags (see
``csrc/cpp/perf/options.cc``) and sets up the protocol client, model metadata,
request tensors and shared-memory regions.  ``run_fixed(concurrency, n)``
keeps ``concurrency`` requests in flight until exactly ``n`` have completed
and returns their latencies; the call drops the GIL (ctypes), so the request
path is entirely C++.
"""

import ctypes
import os

import numpy as np

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB_PATH = os.path.join(_REPO, "csrc", "cpp", "build", "lib", "libperfanalyzer.so")
BIN_PATH = os.path.join(_REPO, "csrc", "cpp", "build", "bin", "perf_analyzer")
_lib = None


def available():
    return os.path.exists(LIB_PATH)


def _load():
    global _lib
    if _lib is None:
        if not available():
            raise RuntimeError("native perf engine not built (%s); run `make -C csrc/cpp`" % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        lib.tcperf_session_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.c_char_p,
                                              ctypes.c_int]
        lib.tcperf_session_create.restype = ctypes.c_void_p
        lib.tcperf_run_fixed.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64,
                                         ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double),
                                         ctypes.c_char_p, ctypes.c_int]
        lib.tcperf_run_fixed.restype = ctypes.c_int
        lib.tcperf_run_fixed_timed.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64,
                                               ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                               ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, ctypes.c_int]
        lib.tcperf_run_fixed_timed.restype = ctypes.c_int
        lib.tcperf_server_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_char_p,
                                            ctypes.c_int]
        lib.tcperf_server_stats.restype = ctypes.c_int
        lib.tcperf_profile.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.POINTER(ctypes.c_double),
                                       ctypes.c_char_p, ctypes.c_int]
        lib.tcperf_profile.restype = ctypes.c_int
        lib.tcperf_loop_start.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        lib.tcperf_loop_start.restype = ctypes.c_int
        lib.tcperf_loop_count.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
        lib.tcperf_loop_count.restype = ctypes.c_uint64
        lib.tcperf_loop_wait.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_double, ctypes.c_char_p,
                                         ctypes.c_int]
        lib.tcperf_loop_wait.restype = ctypes.c_int
        lib.tcperf_loop_records.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                            ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                            ctypes.POINTER(ctypes.c_uint8)]
        lib.tcperf_loop_records.restype = ctypes.c_uint64
        lib.tcperf_loop_stop.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
        lib.tcperf_loop_stop.restype = ctypes.c_int
        lib.tcperf_describe.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
        lib.tcperf_describe.restype = ctypes.c_int
        lib.tcperf_session_destroy.argtypes = [ctypes.c_void_p]
        lib.tcperf_session_destroy.restype = None
        _lib = lib
    return _lib


STAT_KEYS = ("inference_count", "execution_count", "success_count", "success_ns", "queue_ns",
             "compute_input_ns", "compute_infer_ns", "compute_output_ns")
POINT_KEYS = ("load", "stable", "request_count", "window_s", "throughput", "avg_us", "p50_us", "p90_us",
              "p95_us", "p99_us", "client_send_us", "client_recv_us")


class PerfError(RuntimeError):
    pass


class PerfSession:
    def __init__(self, args):
        lib = _load()
        argv = [str(a).encode() for a in args]
        arr = (ctypes.c_char_p * len(argv))(*argv)
        err = ctypes.create_string_buffer(1024)
        self._h = lib.tcperf_session_create(len(argv), arr, err, 1024)
        if not self._h:
            raise PerfError(err.value.decode(errors="replace"))

    def run_fixed(self, concurrency, total):
        """Exactly ``total`` requests with ``concurrency`` in flight; returns (latencies_ns, elapsed_s)."""
        lat = np.zeros(int(total), dtype=np.uint64)
        el = ctypes.c_double(0.0)
        err = ctypes.create_string_buffer(1024)
        rc = _load().tcperf_run_fixed(self._h, int(concurrency), int(total),
                                      lat.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), ctypes.byref(el), err,
                                      1024)
        if rc != 0:
            raise PerfError(err.value.decode(errors="replace"))
        return lat, el.value

    def run_timed(self, concurrency, total):
        """As :meth:`run_fixed`, plus each request's completion time (ns since
        the run started); both arrays in completion order."""
        lat = np.zeros(int(total), dtype=np.uint64)
        end = np.zeros(int(total), dtype=np.uint64)
        el = ctypes.c_double(0.0)
        err = ctypes.create_string_buffer(1024)
        p64 = ctypes.POINTER(ctypes.c_uint64)
        rc = _load().tcperf_run_fixed_timed(self._h, int(concurrency), int(total), lat.ctypes.data_as(p64),
                                            end.ctypes.data_as(p64), ctypes.byref(el), err, 1024)
        if rc != 0:
            raise PerfError(err.value.decode(errors="replace"))
        return lat, end, el.value

    # ---- continuous closed loop (steady-state windows, no restart) ----
    def loop_start(self, concurrency):
        """Keep ``concurrency`` requests in flight until loop_stop."""
        err = ctypes.create_string_buffer(1024)
        if _load().tcperf_loop_start(self._h, int(concurrency), err, 1024) != 0:
            raise PerfError(err.value.decode(errors="replace"))

    def loop_count(self):
        """(completions so far = a record index, engine clock ns)."""
        now = ctypes.c_uint64(0)
        n = _load().tcperf_loop_count(self._h, ctypes.byref(now))
        return int(n), int(now.value)

    def loop_wait(self, target, timeout_s=600.0, heartbeat_s=30.0, log=None):
        """Block (GIL released) until ``target`` records exist; every
        ``heartbeat_s`` without reaching it, ``log`` (if given) gets the
        progress, so a long window never looks like a hung run."""
        import time

        t0 = time.time()
        while True:
            step = min(heartbeat_s, max(0.0, timeout_s - (time.time() - t0)))
            err = ctypes.create_string_buffer(1024)
            if _load().tcperf_loop_wait(self._h, int(target), float(step), err, 1024) == 0:
                return
            msg = err.value.decode(errors="replace")
            if "timed out" not in msg or time.time() - t0 >= timeout_s:
                raise PerfError(msg)
            if log is not None:
                log("loop: %d of %d requests after %.0f s" % (self.loop_count()[0], int(target), time.time() - t0))

    def loop_records(self, start, n):
        """Records [start, start + n): (start_ns, end_ns, ok) on the engine clock."""
        st = np.zeros(int(n), dtype=np.uint64)
        en = np.zeros(int(n), dtype=np.uint64)
        ok = np.zeros(int(n), dtype=np.uint8)
        p64 = ctypes.POINTER(ctypes.c_uint64)
        m = _load().tcperf_loop_records(self._h, int(start), int(n), st.ctypes.data_as(p64), en.ctypes.data_as(p64),
                                        ok.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
        return st[:m], en[:m], ok[:m]

    def loop_stop(self):
        err = ctypes.create_string_buffer(1024)
        if _load().tcperf_loop_stop(self._h, err, 1024) != 0:
            raise PerfError(err.value.decode(errors="replace"))

    def server_stats(self):
        out = (ctypes.c_uint64 * 8)()
        err = ctypes.create_string_buffer(1024)
        if _load().tcperf_server_stats(self._h, out, err, 1024) != 0:
            raise PerfError(err.value.decode(errors="replace"))
        return dict(zip(STAT_KEYS, list(out)))

    def profile(self, load):
        """One perf_analyzer measurement point (windows until stable)."""
        out = (ctypes.c_double * 12)()
        err = ctypes.create_string_buffer(1024)
        if _load().tcperf_profile(self._h, float(load), out, err, 1024) != 0:
            raise PerfError(err.value.decode(errors="replace"))
        return dict(zip(POINT_KEYS, list(out)))

    def describe(self):
        buf = ctypes.create_string_buffer(1024)
        _load().tcperf_describe(self._h, buf, 1024)
        return buf.value.decode(errors="replace")

    def close(self):
        if self._h:
            _load().tcperf_session_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
