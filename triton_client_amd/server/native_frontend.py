"""ctypes side of tcserve, the native gRPC front end (csrc/cpp/server).

``NativeFrontend(server, host, port, upstream_port)`` starts the C++ HTTP/2
server on the public gRPC port.  It proxies every RPC to the Python
grpc.aio server (listening on ``upstream_port`` on loopback) except
``ModelInfer`` for models that expose ``execute_native`` (fixed-size tensors,
dynamic batching): those are parsed, batched and answered in C++, and the
batch is handed to the model in one Python call.

The Python shared-memory registries stay the source of truth (they open the
regions); registrations are mirrored into the native table through
``InferenceServer.shm_listeners`` so the fast path can resolve region names
without Python.  Statistics of natively served requests are merged into
``InferenceServer.statistics()`` through ``InferenceServer.native_stats``.
"""

import ctypes
import os
import threading

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# TCSERVE_LIB: an alternative build (the sanitizer presets, tools/sanitize_tcserve.py)
LIB_PATH = os.environ.get("TCSERVE_LIB") or os.path.join(_REPO, "csrc", "cpp", "build", "lib", "libtcserve.so")


class TcRef(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("device", ctypes.c_int32), ("ptr", ctypes.c_uint64),
                ("bytes", ctypes.c_uint64)]


class TcBatch(ctypes.Structure):
    _fields_ = [("n_requests", ctypes.c_int32), ("total_rows", ctypes.c_int32),
                ("rows", ctypes.POINTER(ctypes.c_int32)), ("n_inputs", ctypes.c_int32),
                ("inputs", ctypes.POINTER(TcRef)), ("n_outputs", ctypes.c_int32),
                ("outputs", ctypes.POINTER(TcRef)), ("timing_ns", ctypes.POINTER(ctypes.c_uint64))]


EXEC_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(TcBatch), ctypes.c_void_p,
                           ctypes.c_int32)

_lib = None


def available():
    return os.path.exists(LIB_PATH)


def _load():
    global _lib
    if _lib is None:
        lib = ctypes.CDLL(LIB_PATH)
        cp = ctypes.c_char_p
        lib.tcserve_create.argtypes = [cp, ctypes.c_int32, cp, ctypes.c_int32, ctypes.c_int32, cp, ctypes.c_int32]
        lib.tcserve_create.restype = ctypes.c_void_p
        lib.tcserve_port.argtypes = [ctypes.c_void_p]
        lib.tcserve_port.restype = ctypes.c_int32
        lib.tcserve_add_model.argtypes = [
            ctypes.c_void_p, cp, cp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
            ctypes.c_int32, ctypes.POINTER(cp), ctypes.POINTER(cp), ctypes.POINTER(ctypes.c_int32),
            ctypes.POINTER(ctypes.c_int64),
            ctypes.c_int32, ctypes.POINTER(cp), ctypes.POINTER(cp), ctypes.POINTER(ctypes.c_int32),
            ctypes.POINTER(ctypes.c_int64),
            EXEC_FN, ctypes.c_void_p, cp, ctypes.c_int32]
        lib.tcserve_add_model.restype = ctypes.c_int32
        lib.tcserve_set_idle_dispatch.argtypes = [ctypes.c_void_p, cp, ctypes.c_int32]
        lib.tcserve_set_idle_dispatch.restype = ctypes.c_int32
        lib.tcserve_set_preferred.argtypes = [ctypes.c_void_p, cp, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]
        lib.tcserve_set_preferred.restype = ctypes.c_int32
        lib.tcserve_remove_model.argtypes = [ctypes.c_void_p, cp]
        lib.tcserve_remove_model.restype = ctypes.c_int32
        lib.tcserve_shm_add.argtypes = [ctypes.c_void_p, cp, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint64,
                                        ctypes.c_int32]
        lib.tcserve_shm_add.restype = ctypes.c_int32
        lib.tcserve_shm_remove.argtypes = [ctypes.c_void_p, ctypes.c_int32, cp]
        lib.tcserve_shm_remove.restype = ctypes.c_int32
        lib.tcserve_shm_busy.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64]
        lib.tcserve_shm_busy.restype = ctypes.c_int32
        lib.tcserve_model_stats.argtypes = [ctypes.c_void_p, cp, ctypes.POINTER(ctypes.c_uint64)]
        lib.tcserve_model_stats.restype = ctypes.c_int32
        lib.tcserve_batch_stats.argtypes = [ctypes.c_void_p, cp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32]
        lib.tcserve_batch_stats.restype = ctypes.c_int32
        lib.tcserve_counters.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
        lib.tcserve_counters.restype = ctypes.c_int32
        lib.tcserve_listen_http.argtypes = [ctypes.c_void_p, cp, ctypes.c_int32, cp, ctypes.c_int32, ctypes.c_char_p,
                                            ctypes.c_int32]
        lib.tcserve_listen_http.restype = ctypes.c_int32
        lib.tcserve_destroy.argtypes = [ctypes.c_void_p]
        lib.tcserve_destroy.restype = None
        _lib = lib
    return _lib


def _strs(xs):
    return (ctypes.c_char_p * max(1, len(xs)))(*[x.encode() for x in xs])


class NativeFrontend:
    def __init__(self, server, host, port, upstream_port, io_threads=None):
        if io_threads is None:
            # one epoll loop per connection group; in-band tensors cost ~1 core
            # per 2 GB/s, so scale with the CPUs this process may use (2..8)
            io_threads = int(os.environ.get("TCSERVE_IO_THREADS", "0")) or max(
                2, min(8, len(os.sched_getaffinity(0)) // 4))
        lib = _load()
        err = ctypes.create_string_buffer(512)
        h = lib.tcserve_create(host.encode(), int(port), b"127.0.0.1", int(upstream_port), int(io_threads), err, 512)
        if not h:
            raise RuntimeError("tcserve: %s" % err.value.decode(errors="replace"))
        self._h = h
        self.server = server
        self._cbs = {}
        self._lock = threading.Lock()
        self._versions = {}
        server.shm_listeners.append(self._on_shm)
        server.model_listeners.append(self._on_model)
        server.native_stats = self.model_stats
        # mirror regions registered before the front end started
        for name, e in list(server.sys_shm.regions.items()):
            self._on_shm("system", "add", name, e[0].address(0), e[3], 0)
        for name, e in list(server.dev_shm.regions.items()):
            self._on_shm("device", "add", name, e[0], e[2], e[1])

    @property
    def port(self):
        return _load().tcserve_port(self._h)

    def listen_http(self, host, port, upstream_port):
        """Serve KServe REST on host:port: native infer fast path, everything
        else relayed to the aiohttp server on 127.0.0.1:upstream_port."""
        err = ctypes.create_string_buffer(512)
        p = _load().tcserve_listen_http(self._h, host.encode(), int(port), b"127.0.0.1", int(upstream_port), err, 512)
        if p < 0:
            raise RuntimeError("tcserve: %s" % err.value.decode(errors="replace"))
        return p

    # -- shared memory mirror ------------------------------------------------------
    def _on_shm(self, kind, op, name, ptr=0, nbytes=0, device=0):
        """Mirror a registration.  On remove, returns a predicate that is True
        while queued/executing native requests still point into the region
        (the registry defers the unmap / IPC close until it is False)."""
        k = 0 if kind == "system" else 1
        if op == "add":
            _load().tcserve_shm_add(self._h, name.encode(), k, int(ptr), int(nbytes), int(device))
            return None
        h = self._h
        if not h:
            return None
        if _load().tcserve_shm_remove(h, k, (name or "").encode()) <= 0 or not ptr:
            return None
        return lambda: bool(self._h) and _load().tcserve_shm_busy(self._h, k, int(ptr)) != 0

    # -- models ----------------------------------------------------------------------
    def register_all(self):
        for entry in list(self.server.repo.values()):
            self._on_model("load", entry)

    def _on_model(self, op, entry, version=None):
        name = entry.name
        if op == "unload":
            if self._versions.get(name) == str(version):
                self.unregister_model(name)
            return
        if not entry.instances:
            return
        v = max(entry.instances)
        inst = entry.instances[v]
        if not getattr(inst, "supports_native", False) or entry.cls.ensemble_steps:
            return
        if name in self._versions:
            self.unregister_model(name)
        from .core import _override_batching

        self.register_model(name, inst, _override_batching(entry, inst.dynamic_batching))

    def register_model(self, name, inst, dynamic_batching=None):
        """Serve ``inst`` (a loaded model exposing execute_native) on the fast
        path; ``dynamic_batching`` replaces the model's own batcher settings
        (a repository load's config override)."""
        db_cfg = inst.dynamic_batching if dynamic_batching is None else dynamic_batching
        ins, outs = inst.inputs, inst.outputs

        def flat(specs):
            nd = (ctypes.c_int32 * max(1, len(specs)))(*[len(s.dims) for s in specs])
            dims = [int(d) for s in specs for d in s.dims]
            return nd, (ctypes.c_int64 * max(1, len(dims)))(*dims)

        in_nd, in_dims = flat(ins)
        out_nd, out_dims = flat(outs)

        def _exec(user, instance, bptr, err, errlen):
            try:
                inst.execute_native(int(instance), bptr.contents)
                return 0
            except Exception as e:  # noqa: BLE001 - reported to the client
                msg = str(e).encode()[: max(0, errlen - 1)]
                ctypes.memmove(err, msg + b"\0", len(msg) + 1)
                return 1

        native = getattr(inst, "native_executor", None)
        native = native() if native is not None else None
        if native is not None:
            # a C executor (e.g. csrc/runtime/graph_exec.hip): tcserve's batcher
            # threads call it directly, no Python per batch
            cb = EXEC_FN(native[0])
            user = ctypes.c_void_p(native[1])
        else:
            cb = EXEC_FN(_exec)
            user = None
        delay = int((db_cfg or {}).get("max_queue_delay_us", 0)) if db_cfg is not None else 0
        err = ctypes.create_string_buffer(512)
        rc = _load().tcserve_add_model(
            self._h, name.encode(), str(inst.version).encode(), int(inst.max_batch_size), delay,
            int(max(1, inst.instance_count)),
            len(ins), _strs([s.name for s in ins]), _strs([s.datatype for s in ins]), in_nd, in_dims,
            len(outs), _strs([s.name for s in outs]), _strs([s.datatype for s in outs]), out_nd, out_dims,
            cb, user, err, 512)
        if rc != 0:
            raise RuntimeError("tcserve: %s" % err.value.decode(errors="replace"))
        pref = [int(x) for x in (db_cfg or {}).get("preferred", [])]
        if pref:
            self.set_preferred(name, pref)
        db = db_cfg or {}
        self.set_idle_dispatch(name, bool(db.get("idle_dispatch", True)), pipelined=bool(db.get("pipelined", False)))
        with self._lock:
            self._cbs[name] = cb
            self._versions[name] = str(inst.version)

    def set_idle_dispatch(self, name, on, pipelined=False):
        """Skip the queue delay while every instance of the model is idle;
        ``pipelined``: a free instance also takes a partial batch once the queue
        holds as many rows as the last batch did."""
        if _load().tcserve_set_idle_dispatch(self._h, name.encode(), int(bool(on)) | (int(bool(pipelined)) << 1)) != 0:
            raise KeyError(name)

    def set_preferred(self, name, sizes):
        """dynamic_batching.preferred_batch_size of a registered model ([] clears)."""
        sizes = [int(x) for x in sizes]
        rc = _load().tcserve_set_preferred(self._h, name.encode(), (ctypes.c_int32 * max(1, len(sizes)))(*sizes),
                                           len(sizes))
        if rc != 0:
            raise KeyError(name)

    def unregister_model(self, name):
        _load().tcserve_remove_model(self._h, name.encode())
        with self._lock:
            self._cbs.pop(name, None)
            self._versions.pop(name, None)

    def model_stats(self, name):
        """Counters of natively served requests for ``name`` (None if not native)."""
        out = (ctypes.c_uint64 * 11)()
        if _load().tcserve_model_stats(self._h, name.encode(), out) != 0:
            return None
        rows = (ctypes.c_uint64 * (7 * 256))()
        n = _load().tcserve_batch_stats(self._h, name.encode(), rows, 256)
        batches = {}
        for i in range(max(0, n)):
            r = rows[7 * i: 7 * i + 7]
            batches[int(r[0])] = (int(r[1]), int(r[2]), int(r[3]), int(r[4]))
        keys = ("inference_count", "execution_count", "success_count", "success_ns", "fail_count", "fail_ns",
                "queue_ns", "compute_input_ns", "compute_infer_ns", "compute_output_ns", "last_inference")
        d = dict(zip(keys, [int(x) for x in out]))
        d["batches"] = batches
        d["version"] = self._versions.get(name)
        return d

    def counters(self):
        out = (ctypes.c_uint64 * 5)()
        _load().tcserve_counters(self._h, out)
        return {"native_requests": int(out[0]), "proxied_calls": int(out[1]), "connections": int(out[2]),
                "inflated_requests": int(out[3]), "compressed_responses": int(out[4])}

    def close(self):
        if self._h:
            for lst, fn in ((self.server.shm_listeners, self._on_shm), (self.server.model_listeners, self._on_model)):
                try:
                    lst.remove(fn)
                except ValueError:
                    pass
            self.server.native_stats = None
            _load().tcserve_destroy(self._h)
            self._h = None
