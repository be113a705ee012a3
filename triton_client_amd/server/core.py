"""Transport-neutral inference core of the in-repo KServe-v2 server.

Responsibilities: model repository (load/unload/override, version policy),
schedulers (direct, dynamic batching, sequence, ensemble, decoupled),
shared-memory registries (POSIX + HIP IPC device regions), output delivery
(binary / JSON / classification / shm), statistics, trace & log settings.

Wire semantics mirror what the reference client expects from a Triton server
(reference src/c++/library/http_client.cc:1393-1764, grpc_client.cc:717-1042).
"""

import asyncio
import base64
import json
import collections
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from tritonclient.grpc import model_config_pb2 as mc

from .types import (
    DeviceView,
    InferResponse,
    OutputTensor,
    ServerError,
    decode_raw,
    internal,
    not_found,
    unavailable,
)

SERVER_NAME = "triton-mi355x"
SERVER_VERSION = "2.51.0"
EXTENSIONS = [
    "classification",
    "sequence",
    "model_repository",
    "model_repository(unload_dependents)",
    "schedule_policy",
    "model_configuration",
    "system_shared_memory",
    "cuda_shared_memory",
    "hip_shared_memory",
    "binary_tensor_data",
    "parameters",
    "statistics",
    "trace",
    "logging",
]


def _now_ns():
    return time.monotonic_ns()


class _Dur:
    __slots__ = ("count", "ns")

    def __init__(self):
        self.count = 0
        self.ns = 0

    def add(self, ns, n=1):
        self.count += n
        self.ns += ns

    def json(self):
        return {"count": self.count, "ns": self.ns}


class ModelStats:
    KEYS = (
        "success",
        "fail",
        "queue",
        "compute_input",
        "compute_infer",
        "compute_output",
        "cache_hit",
        "cache_miss",
    )

    def __init__(self):
        self.lock = threading.Lock()
        self.last_inference = 0
        self.inference_count = 0
        self.execution_count = 0
        self.d = {k: _Dur() for k in self.KEYS}
        self.batch = {}  # batch_size -> {compute_input, compute_infer, compute_output}

    def record_batch(self, batch_size, n_requests, t_in, t_infer, t_out):
        with self.lock:
            self.execution_count += 1
            b = self.batch.setdefault(
                batch_size, {"compute_input": _Dur(), "compute_infer": _Dur(), "compute_output": _Dur()}
            )
            b["compute_input"].add(t_in)
            b["compute_infer"].add(t_infer)
            b["compute_output"].add(t_out)
            self.d["compute_input"].add(t_in, n_requests)
            self.d["compute_infer"].add(t_infer, n_requests)
            self.d["compute_output"].add(t_out, n_requests)

    def record_request(self, ok, total_ns, queue_ns, batch_size):
        with self.lock:
            self.last_inference = int(time.time() * 1000)
            if ok:
                self.inference_count += batch_size
                self.d["success"].add(total_ns)
                self.d["queue"].add(queue_ns)
            else:
                self.d["fail"].add(total_ns)

    def json(self, name, version):
        with self.lock:
            return {
                "name": name,
                "version": str(version),
                "last_inference": self.last_inference,
                "inference_count": self.inference_count,
                "execution_count": self.execution_count,
                "inference_stats": {k: v.json() for k, v in self.d.items()},
                "batch_stats": [
                    {"batch_size": bs, **{k: v.json() for k, v in d.items()}}
                    for bs, d in sorted(self.batch.items())
                ],
                "memory_usage": [],
                "response_stats": {},
            }


# ---------------------------------------------------------------------------
# Shared memory registries
# ---------------------------------------------------------------------------
def _merge_native_stats(d, ns):
    """Fold counters of natively served requests (tcserve) into a stats dict."""
    d["inference_count"] += ns["inference_count"]
    d["execution_count"] += ns["execution_count"]
    d["last_inference"] = max(d["last_inference"], ns["last_inference"])
    st = d["inference_stats"]
    n = ns["success_count"]
    st["success"]["count"] += n
    st["success"]["ns"] += ns["success_ns"]
    st["fail"]["count"] += ns["fail_count"]
    st["fail"]["ns"] += ns["fail_ns"]
    st["queue"]["count"] += n
    st["queue"]["ns"] += ns["queue_ns"]
    for k in ("compute_input", "compute_infer", "compute_output"):
        st[k]["count"] += n
        st[k]["ns"] += ns[k + "_ns"]
    by_bs = {b["batch_size"]: b for b in d["batch_stats"]}
    for bs, (cnt, t_in, t_inf, t_out) in ns["batches"].items():
        b = by_bs.get(bs)
        if b is None:
            b = {"batch_size": bs}
            for k in ("compute_input", "compute_infer", "compute_output"):
                b[k] = {"count": 0, "ns": 0}
            d["batch_stats"].append(b)
            by_bs[bs] = b
        for k, t in (("compute_input", t_in), ("compute_infer", t_inf), ("compute_output", t_out)):
            b[k]["count"] += cnt
            b[k]["ns"] += t
    d["batch_stats"].sort(key=lambda b: b["batch_size"])


class DeferredCloser:
    """Closes unregistered shared-memory regions once no queued or executing
    native request points into them any more (tcserve_shm_busy).  The wait
    runs on this thread, never on the server's event loop or under a registry
    lock."""

    def __init__(self):
        self._cv = threading.Condition()
        self._items = []  # (close_fn, [busy_fn, ...])
        self._thread = None

    def close_when_idle(self, close_fn, busy_fns):
        busy_fns = [b for b in busy_fns if b is not None]
        if not any(b() for b in busy_fns):
            close_fn()
            return
        with self._cv:
            self._items.append((close_fn, busy_fns))
            if self._thread is None:
                self._thread = threading.Thread(target=self._run, name="shm-closer", daemon=True)
                self._thread.start()
            self._cv.notify()

    def pending(self):
        with self._cv:
            return len(self._items)

    def _run(self):
        import time

        while True:
            with self._cv:
                while not self._items:
                    self._cv.wait()
                items = list(self._items)
            done = [it for it in items if not any(b() for b in it[1])]
            for close_fn, _ in done:
                try:
                    close_fn()
                except Exception:  # noqa: BLE001 - a failed unmap must not kill the closer
                    pass
            with self._cv:
                self._items = [it for it in self._items if it not in done]
            if len(done) < len(items):
                time.sleep(0.0005)


def _notify_remove(listeners, kind, name, ptr):
    """Tell the listeners (the native front end) a region is gone; returns the
    busy predicates of those that still have requests pointing into it."""
    busy = []
    for fn in listeners:
        r = fn(kind, "remove", name, ptr)
        if callable(r):
            busy.append(r)
    return busy


class SystemShmRegistry:
    def __init__(self, listeners=None, closer=None):
        self.regions = {}
        self.lock = threading.Lock()
        self.listeners = listeners if listeners is not None else []
        self.closer = closer or DeferredCloser()

    def register(self, name, key, offset, byte_size):
        from tritonclient.utils import shared_memory as shm

        with self.lock:
            if name in self.regions:
                raise ServerError(
                    "shared memory region '%s' already in manager" % name, 400, "ALREADY_EXISTS"
                )
            try:
                region = shm.MappedRegion(key, offset, byte_size)
            except Exception as e:
                raise ServerError(
                    "Unable to open shared memory region: '%s' (%s)" % (key, e), 400, "INVALID_ARGUMENT"
                )
            self.regions[name] = (region, key, offset, byte_size)
            for fn in self.listeners:
                fn("system", "add", name, region.address(0), byte_size, 0)

    def unregister(self, name=""):
        with self.lock:
            names = [name] if name else list(self.regions)
            for n in names:
                entry = self.regions.pop(n, None)
                if entry is not None:
                    busy = _notify_remove(self.listeners, "system", n, entry[0].address(0))
                    self.closer.close_when_idle(entry[0].close, busy)

    def status(self, name=""):
        with self.lock:
            if name:
                if name not in self.regions:
                    raise not_found("Unable to find system shared memory region: '%s'" % name)
                items = [(name, self.regions[name])]
            else:
                items = list(self.regions.items())
            return [
                {"name": n, "key": e[1], "offset": e[2], "byte_size": e[3]} for n, e in items
            ]

    def view(self, name, offset, nbytes):
        with self.lock:
            e = self.regions.get(name)
        if e is None:
            raise ServerError("Unable to find system shared memory region: '%s'" % name)
        if offset < 0 or offset + nbytes > e[3]:
            raise ServerError(
                "Invalid offset + byte size for shared memory region: '%s'" % name
            )
        return e[0].view(offset, nbytes)


class DeviceShmRegistry:
    """HIP IPC regions (wire name: cudasharedmemory)."""

    def __init__(self, listeners=None, closer=None):
        self.regions = {}
        self.lock = threading.Lock()
        self.listeners = listeners if listeners is not None else []
        self.closer = closer or DeferredCloser()

    def register(self, name, raw_handle, device_id, byte_size):
        from triton_client_amd.ops import hip

        with self.lock:
            if name in self.regions:
                raise ServerError(
                    "shared memory region '%s' already in manager" % name, 400, "ALREADY_EXISTS"
                )
            if len(raw_handle) != hip.IPC_HANDLE_SIZE:
                raise ServerError(
                    "raw_handle must be %d bytes, got %d" % (hip.IPC_HANDLE_SIZE, len(raw_handle))
                )
            try:
                ptr = hip.ipc_open(raw_handle, device_id)
            except Exception as e:
                raise ServerError("failed to open HIP IPC handle for '%s': %s" % (name, e))
            self.regions[name] = (ptr, device_id, byte_size)
            for fn in self.listeners:
                fn("device", "add", name, ptr, byte_size, device_id)

    def unregister(self, name=""):
        from triton_client_amd.ops import hip

        with self.lock:
            names = [name] if name else list(self.regions)
            for n in names:
                e = self.regions.pop(n, None)
                if e is not None:
                    busy = _notify_remove(self.listeners, "device", n, e[0])

                    def close(ptr=e[0], dev=e[1]):
                        try:
                            hip.ipc_close(ptr, dev)
                        except Exception:
                            pass

                    self.closer.close_when_idle(close, busy)

    def status(self, name=""):
        with self.lock:
            if name:
                if name not in self.regions:
                    raise not_found("Unable to find cuda shared memory region: '%s'" % name)
                items = [(name, self.regions[name])]
            else:
                items = list(self.regions.items())
            return [{"name": n, "device_id": e[1], "byte_size": e[2]} for n, e in items]

    def view(self, name, offset, nbytes):
        with self.lock:
            e = self.regions.get(name)
        if e is None:
            raise ServerError("Unable to find cuda shared memory region: '%s'" % name)
        if offset < 0 or offset + nbytes > e[2]:
            raise ServerError("Invalid offset + byte size for shared memory region: '%s'" % name)
        return DeviceView(e[0] + offset, nbytes, e[1])


# ---------------------------------------------------------------------------
# Repository
# ---------------------------------------------------------------------------
class ModelEntry:
    def __init__(self, cls, options=None):
        self.cls = cls
        self.options = dict(options or {})
        self.instances = {}  # version -> Model
        self.schedulers = {}  # version -> scheduler
        self.stats = {}  # version -> ModelStats
        self.state = "UNAVAILABLE"
        self.reason = "unloaded"
        self.version_filter = None  # set of versions from config override
        self.config_override = None
        self.lock = threading.Lock()

    @property
    def name(self):
        return self.options.get("name", self.cls.name)

    def versions(self):
        vs = tuple(self.options.get("versions", self.cls.versions))
        if self.version_filter is not None:
            vs = tuple(v for v in vs if v in self.version_filter)
        return vs


def _json_config(cfg):
    """ModelConfig proto -> Triton-style JSON dict (int64 as numbers)."""
    from google.protobuf.json_format import MessageToDict

    d = MessageToDict(cfg, preserving_proto_field_name=True)

    def fix(obj):
        if isinstance(obj, dict):
            return {k: fix(v) for k, v in obj.items()}
        if isinstance(obj, list):
            return [fix(v) for v in obj]
        if isinstance(obj, str) and obj.lstrip("-").isdigit():
            return int(obj)
        return obj

    return fix(d)


class InferenceServer:
    def __init__(self, model_classes=(), model_options=None, executor_workers=16, device_id=0):
        self.device_id = device_id
        self.repo = {}
        self.model_options = model_options or {}
        for cls in model_classes:
            self.add_model(cls, self.model_options.get(cls.name))
        # native front end hooks (server/native_frontend.py)
        self.shm_listeners = []
        self.model_listeners = []
        self.native_stats = None
        self.shm_closer = DeferredCloser()
        # what arrived on the wire through the Python front ends (tests verify
        # client features end to end: JSON tensors, custom parameters)
        self.wire_stats = collections.Counter()
        self.sys_shm = SystemShmRegistry(self.shm_listeners, self.shm_closer)
        self.dev_shm = DeviceShmRegistry(self.shm_listeners, self.shm_closer)
        self.executor = ThreadPoolExecutor(max_workers=executor_workers, thread_name_prefix="tcamd-exec")
        self.trace_settings = {
            "trace_level": ["OFF"],
            "trace_rate": "1000",
            "trace_count": "-1",
            "log_frequency": "0",
            "trace_file": "",
            "trace_mode": "triton",
        }
        self.model_trace = {}
        self.log_settings = {
            "log_file": "",
            "log_info": True,
            "log_warning": True,
            "log_error": True,
            "log_verbose_level": 0,
            "log_format": "default",
        }
        self.ready = True
        self.loop = None
        self.native_frontend = None

    # -- repository ------------------------------------------------------------
    def add_model(self, cls, options=None):
        entry = ModelEntry(cls, options)
        self.repo[entry.name] = entry
        return entry

    def load_all(self):
        for name in list(self.repo):
            self.load_model(name)

    def load_model(self, name, config=None, files=None):
        entry = self.repo.get(name)
        if files and config is None:
            raise ServerError(
                "failed to load '%s', failed to poll from model repository: model configuration "
                "must be provided when loading with override files" % name
            )
        cfg_override = None
        if config is not None:
            try:
                cfg_override = json.loads(config) if isinstance(config, str) else config
                if not isinstance(cfg_override, dict):
                    raise ValueError("config must be a JSON object")
            except Exception as e:
                raise ServerError("failed to load '%s', failed to parse config: %s" % (name, e))
        if entry is None:
            if files:
                entry = self._override_entry(name, cfg_override, files)
            else:
                raise ServerError(
                    "failed to load '%s', failed to poll from model repository" % name, 400, "INVALID_ARGUMENT"
                )
        elif files:
            new_entry = self._override_entry(name, cfg_override, files, base=entry)
            self._unload_entry(entry)
            entry = new_entry
        with entry.lock:
            if cfg_override is not None:
                vp = cfg_override.get("version_policy", {})
                if "specific" in vp:
                    entry.version_filter = set(int(v) for v in vp["specific"].get("versions", []))
                elif "latest" in vp:
                    n = int(vp["latest"].get("num_versions", 1))
                    entry.version_filter = set(sorted(entry.options.get("versions", entry.cls.versions))[-n:])
                else:
                    entry.version_filter = None
                entry.config_override = cfg_override
                for sched in entry.schedulers.values():  # the Python batchers (the native one: its frontend)
                    if isinstance(sched, DynamicBatcher):
                        db = _override_batching(entry, sched.inst.dynamic_batching or {})
                        sched.preferred = sorted(db.get("preferred", []))
                        sched.delay_s = db.get("max_queue_delay_us", 0) / 1e6
            wanted = set(entry.versions())
            for v in list(entry.instances):
                if v not in wanted:
                    self._unload_version(entry, v)
            for v in entry.versions():
                if v in entry.instances:
                    continue
                opts = {k: val for k, val in entry.options.items() if k not in ("name", "versions", "base_cls")}
                try:
                    inst = entry.cls(version=v, **opts)
                    inst._server = self  # lets GPU backends resolve shm targets directly
                    inst.load()
                except Exception as e:
                    entry.state = "UNAVAILABLE"
                    entry.reason = str(e)
                    raise ServerError("failed to load '%s' version %d: %s" % (entry.name, v, e))
                entry.instances[v] = inst
                entry.stats[v] = ModelStats()
                entry.schedulers[v] = make_scheduler(self, entry, inst, entry.stats[v])
            entry.state = "READY"
            entry.reason = ""
        self.repo[entry.name] = entry
        for fn in list(self.model_listeners):
            fn("load", entry)

    def _override_entry(self, name, cfg, files, base=None):
        versions = set()
        blob = None
        for path, content in files.items():
            if not path.startswith("file:"):
                raise ServerError("override file path must start with 'file:': %s" % path)
            rel = path[len("file:") :]
            head = rel.split("/", 1)[0]
            if head.isdigit():
                versions.add(int(head))
            blob = content
        if not versions:
            raise ServerError("override files must include at least one version directory")
        cls = base.cls if base is not None else None
        if blob is not None:
            text = blob.decode("utf-8", "ignore") if isinstance(blob, (bytes, bytearray)) else str(blob)
            # Model files produced by this framework name the builtin they implement
            # ("tcamd-model:<builtin>"); anything else falls back to the base model.
            if text.startswith("tcamd-model:"):
                builtin = text.split(":", 1)[1].strip().split()[0]
                if builtin in self.repo:
                    cls = self.repo[builtin].cls
        if cls is None:
            cls = self.repo["onnx_int32_int32_int32"].cls if "onnx_int32_int32_int32" in self.repo else None
        if cls is None:
            raise ServerError("cannot determine backend for override model '%s'" % name)
        entry = ModelEntry(cls, {"name": name, "versions": tuple(sorted(versions))})
        return entry

    def _unload_version(self, entry, v):
        for fn in list(self.model_listeners):
            fn("unload", entry, v)
        sch = entry.schedulers.pop(v, None)
        if sch is not None:
            sch.close()
        inst = entry.instances.pop(v, None)
        if inst is not None:
            try:
                inst.unload()
            except Exception:
                pass
        entry.stats.pop(v, None)

    def _unload_entry(self, entry):
        with entry.lock:
            for v in list(entry.instances):
                self._unload_version(entry, v)
            entry.state = "UNAVAILABLE"
            entry.reason = "unloaded"

    def unload_model(self, name, unload_dependents=False):
        entry = self.repo.get(name)
        if entry is None:
            raise ServerError("failed to unload '%s', model not found" % name)
        self._unload_entry(entry)
        if unload_dependents and entry.cls.ensemble_steps:
            for step_model, _, _ in entry.cls.ensemble_steps:
                if step_model in self.repo:
                    self._unload_entry(self.repo[step_model])

    def repository_index(self):
        out = []
        for name, e in sorted(self.repo.items()):
            vs = sorted(e.instances) or list(e.versions())
            for v in vs:
                item = {"name": name, "version": str(v), "state": e.state if v in e.instances else "UNAVAILABLE"}
                if item["state"] != "READY":
                    item["reason"] = e.reason or "unloaded"
                out.append(item)
        return out

    def get_instance(self, name, version=""):
        e = self.repo.get(name)
        if e is None:
            raise not_found("Request for unknown model: '%s' is not found" % name)
        if not e.instances:
            raise unavailable("Request for unknown model: '%s' is not ready" % name)
        if version in ("", None, -1, "-1"):
            v = max(e.instances)
        else:
            try:
                v = int(version)
            except ValueError:
                raise ServerError("invalid model version '%s'" % version)
            if v not in e.instances:
                raise unavailable(
                    "Request for unknown model: '%s' version %s is not at ready state" % (name, version)
                )
        return e, v, e.instances[v]

    def is_model_ready(self, name, version=""):
        try:
            self.get_instance(name, version)
            return True
        except ServerError:
            return False

    def model_metadata(self, name, version=""):
        e, v, inst = self.get_instance(name, version)
        ins, outs = inst.metadata_tensors()
        return {
            "name": name,
            "versions": [str(x) for x in sorted(e.instances)],
            "platform": inst.platform,
            "inputs": [{"name": n, "datatype": d, "shape": s} for n, d, s in ins],
            "outputs": [{"name": n, "datatype": d, "shape": s} for n, d, s in outs],
        }

    def model_config_proto(self, name, version=""):
        e, v, inst = self.get_instance(name, version)
        cfg = inst.config()
        cfg.name = name
        if e.version_filter is not None:
            cfg.version_policy.specific.versions[:] = sorted(e.version_filter)
        if e.config_override and "backend" in e.config_override:
            cfg.backend = e.config_override["backend"]
        db = _override_batching(e, {})
        if db and cfg.HasField("dynamic_batching"):
            if "preferred" in db:
                cfg.dynamic_batching.preferred_batch_size[:] = db["preferred"]
            if "max_queue_delay_us" in db:
                cfg.dynamic_batching.max_queue_delay_microseconds = db["max_queue_delay_us"]
        return cfg

    def model_config(self, name, version=""):
        return _json_config(self.model_config_proto(name, version))

    def statistics(self, name="", version=""):
        out = []
        names = [name] if name else sorted(self.repo)
        for n in names:
            e = self.repo.get(n)
            if e is None:
                raise not_found("requested model '%s' is not available" % n)
            if name and not e.instances:
                raise unavailable("requested model '%s' is not available" % n)
            for v, st in sorted(e.stats.items()):
                if version not in ("", None) and str(v) != str(version):
                    continue
                d = st.json(n, v)
                ns = self.native_stats(n) if self.native_stats is not None else None
                if ns and str(ns.get("version")) == str(v):
                    _merge_native_stats(d, ns)
                out.append(d)
            if name and version not in ("", None) and not out:
                raise unavailable("requested model version is not available for model '%s'" % n)
        return {"model_stats": out}

    # -- trace / log --------------------------------------------------------------
    def update_trace(self, model_name, settings):
        target = self.trace_settings if not model_name else self.model_trace.setdefault(
            model_name, dict(self.trace_settings)
        )
        if model_name and model_name not in self.repo:
            raise not_found("Request for unknown model: '%s' is not found" % model_name)
        for k, v in settings.items():
            if v is None:
                # clear: model setting falls back to the global one
                if model_name:
                    target[k] = self.trace_settings.get(k)
                continue
            if k == "trace_level":
                target[k] = [str(x) for x in (v if isinstance(v, list) else [v])]
            else:
                target[k] = str(v[0]) if isinstance(v, list) and len(v) == 1 else (
                    [str(x) for x in v] if isinstance(v, list) else str(v)
                )
        return self.get_trace(model_name)

    def get_trace(self, model_name=None):
        if model_name:
            if model_name not in self.repo:
                raise not_found("Request for unknown model: '%s' is not found" % model_name)
            return dict(self.model_trace.get(model_name, self.trace_settings))
        return dict(self.trace_settings)

    def update_log(self, settings):
        for k, v in settings.items():
            if k not in self.log_settings:
                raise ServerError("Unknown log setting '%s'" % k)
            if v is None:
                continue
            expect = type(self.log_settings[k])
            if expect is bool and not isinstance(v, bool):
                raise ServerError("log setting '%s' must be a boolean" % k)
            if expect is int and (isinstance(v, bool) or not isinstance(v, int)):
                raise ServerError("log setting '%s' must be an unsigned integer" % k)
            if expect is str and not isinstance(v, str):
                raise ServerError("log setting '%s' must be a string" % k)
            self.log_settings[k] = v
        return dict(self.log_settings)

    # -- input / output resolution ------------------------------------------------
    def resolve_shm_input(self, tensor, params):
        region = params.get("shared_memory_region")
        nbytes = int(params.get("shared_memory_byte_size", 0))
        offset = int(params.get("shared_memory_offset", 0))
        if region in self.sys_shm.regions:
            view = self.sys_shm.view(region, offset, nbytes)
            tensor.data = decode_raw(view, tensor.datatype, tensor.shape)
        elif region in self.dev_shm.regions:
            tensor.data = self.dev_shm.view(region, offset, nbytes)
        else:
            raise ServerError("Unable to find shared memory region: '%s'" % region)

    def shm_target(self, region, nbytes, offset):
        if region in self.sys_shm.regions:
            return self.sys_shm.view(region, offset, nbytes)
        if region in self.dev_shm.regions:
            return self.dev_shm.view(region, offset, nbytes)
        raise ServerError("Unable to find shared memory region: '%s'" % region)

    def finalize_outputs(self, request, inst, outputs):
        """Apply requested-output selection, classification and shm delivery."""
        by_name = {o.name: o for o in outputs}
        if request.outputs:
            selected = []
            for ro in request.outputs:
                o = by_name.get(ro.name)
                if o is None:
                    raise ServerError(
                        "unexpected inference output '%s' for model '%s'" % (ro.name, request.model_name)
                    )
                if ro.class_count:
                    o = classify(o, ro.class_count, inst.labels, inst.max_batch_size > 0)
                if ro.shm is not None and o.shm is None:
                    deliver_to_shm(self, o, ro.shm)
                selected.append((o, ro))
            return selected
        return [(o, None) for o in outputs]

    # -- inference entry points -----------------------------------------------------
    _RESERVED_PARAMS = ("sequence_id", "sequence_start", "sequence_end", "priority", "timeout", "binary_data_output",
                        "triton_enable_empty_final_response")

    async def infer(self, request):
        for k, v in request.parameters.items():
            if k not in self._RESERVED_PARAMS:  # custom request parameters, by name / type / value
                self.wire_stats["param:%s:%s:%s" % (k, type(v).__name__, v)] += 1
        entry, version, inst = self.get_instance(request.model_name, request.model_version)
        if inst.decoupled:
            raise ServerError(
                "doesn't support models with decoupled transaction policy", 400, "UNIMPLEMENTED"
            )
        request.model_version = str(version)
        if inst.ensemble_steps:
            return await self._infer_ensemble(request, inst)
        inst.validate(request)
        sch = entry.schedulers[version]
        outputs = await sch.submit(request)
        resp = InferResponse(
            model_name=request.model_name, model_version=str(version), id=request.id
        )
        resp.outputs = self.finalize_outputs(request, inst, outputs)
        return resp

    async def stream_infer(self, request, emit):
        """Run a (possibly decoupled) request; ``await emit(InferResponse)``
        for each response.  Returns after the last response."""
        entry, version, inst = self.get_instance(request.model_name, request.model_version)
        request.model_version = str(version)
        empty_final = bool(request.parameters.get("triton_enable_empty_final_response", False))
        if not inst.decoupled:
            resp = await self.infer(request)
            if empty_final:
                resp.parameters["triton_final_response"] = True
            await emit(resp)
            return
        inst.validate(request)
        loop = asyncio.get_running_loop()
        q = asyncio.Queue()
        t0 = _now_ns()

        def _emit(outs):
            loop.call_soon_threadsafe(q.put_nowait, ("out", outs))

        def _run():
            try:
                inst.execute_decoupled(request, _emit)
                loop.call_soon_threadsafe(q.put_nowait, ("done", None))
            except Exception as e:  # noqa: BLE001
                loop.call_soon_threadsafe(q.put_nowait, ("err", e))

        self.executor.submit(_run)
        stats = entry.stats[version]
        while True:
            kind, payload = await q.get()
            if kind == "out":
                resp = InferResponse(request.model_name, str(version), request.id)
                resp.outputs = self.finalize_outputs(request, inst, payload)
                if empty_final:
                    resp.parameters["triton_final_response"] = False
                await emit(resp)
            elif kind == "done":
                stats.record_request(True, _now_ns() - t0, 0, 1)
                if empty_final:
                    resp = InferResponse(request.model_name, str(version), request.id, final=True)
                    resp.parameters["triton_final_response"] = True
                    await emit(resp)
                return
            else:
                stats.record_request(False, _now_ns() - t0, 0, 1)
                raise payload if isinstance(payload, ServerError) else internal(str(payload))

    async def _infer_ensemble(self, request, inst):
        from .types import InferRequest, InputTensor

        tensors = {t.name: t for t in request.inputs}
        for step_model, imap, omap in inst.ensemble_steps:
            sub = InferRequest(model_name=step_model, id=request.id)
            for model_in, ens_name in imap.items():
                t = tensors.get(ens_name)
                if t is None:
                    raise ServerError("ensemble tensor '%s' is not available" % ens_name)
                sub.inputs.append(InputTensor(model_in, t.datatype, list(t.shape), t.data))
            resp = await self.infer(sub)
            for o, _ in resp.outputs:
                if o.name in omap:
                    ens = omap[o.name]
                    tensors[ens] = InputTensor(ens, o.datatype, list(o.shape), o.data)
        outs = []
        for spec in inst.outputs:
            t = tensors.get(spec.name)
            if t is None:
                raise internal("ensemble output '%s' was not produced" % spec.name)
            outs.append(OutputTensor(spec.name, t.datatype, list(t.shape), t.data))
        resp = InferResponse(request.model_name, request.model_version, request.id)
        resp.outputs = self.finalize_outputs(request, inst, outs)
        return resp


def classify(o, k, labels, batched):
    """Top-k classification strings 'score:index[:label]' (Triton format)."""
    data = o.data
    if data is None:
        raise ServerError("classification of shared-memory outputs is not supported")
    arr = np.asarray(data, dtype=np.float64)
    rows = arr.reshape(arr.shape[0], -1) if batched else arr.reshape(1, -1)
    k = min(k, rows.shape[1])
    res = []
    for row in rows:
        idx = np.argsort(-row, kind="stable")[:k]
        items = []
        for i in idx:
            s = "%f:%d" % (row[i], i)
            if labels is not None and i < len(labels):
                s += ":" + labels[i]
            items.append(s.encode())
        res.append(items)
    out = np.array(res, dtype=np.object_)
    if not batched:
        out = out.reshape(k)
    return OutputTensor(o.name, "BYTES", list(out.shape), out)


def deliver_to_shm(server, o, shm):
    from tritonclient.utils import serialize_bf16_tensor, serialize_byte_tensor

    region, nbytes, offset = shm
    target = server.shm_target(region, nbytes, offset)
    data = o.data
    if hasattr(data, "is_cuda"):  # torch tensor on device
        raw_dev = data.contiguous()
        n = raw_dev.numel() * raw_dev.element_size()
        if n > nbytes:
            raise ServerError("shared memory size specified with the request for output '%s' (%d bytes) should be at least %d bytes" % (o.name, nbytes, n))
        from triton_client_amd.ops import hip

        if isinstance(target, DeviceView):
            hip.memcpy_d2d(target.ptr, raw_dev.data_ptr(), n)
        else:
            host = raw_dev.cpu().numpy().view(np.uint8).reshape(-1)
            target[:n] = host
        o.data = None
        o.shm = shm
        return
    if o.datatype == "BYTES":
        s = serialize_byte_tensor(np.asarray(data, dtype=np.object_))
        raw = np.frombuffer(s.item() if s.size else b"", dtype=np.uint8)
    elif o.datatype == "BF16":
        s = serialize_bf16_tensor(np.asarray(data, dtype=np.float32))
        raw = np.frombuffer(s.item() if s.size else b"", dtype=np.uint8)
    else:
        raw = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    if raw.size > nbytes:
        raise ServerError(
            "shared memory size specified with the request for output '%s' (%d bytes) should be at least %d bytes"
            % (o.name, nbytes, raw.size)
        )
    if isinstance(target, DeviceView):
        from triton_client_amd.ops import hip

        hip.memcpy_h2d(target.ptr, raw, raw.size)
    else:
        target[: raw.size] = raw
    o.data = None
    o.shm = shm


# ---------------------------------------------------------------------------
# Schedulers
# ---------------------------------------------------------------------------
def _batch_size(inst, request):
    if inst.max_batch_size > 0 and request.inputs:
        return int(request.inputs[0].shape[0])
    return 1


class DirectScheduler:
    """One request per execution, ``instance_count`` executions in flight."""

    def __init__(self, server, entry, inst, stats):
        self.server = server
        self.inst = inst
        self.stats = stats
        self.sem = threading.Semaphore(max(1, inst.instance_count))
        self.serial = threading.Lock() if inst.sequence_batching else None
        # GPU backends time their phases with device events and report them
        self.model_reports = bool(getattr(inst, "reports_batch_stats", False))
        if self.model_reports:
            inst._batch_stats = stats.record_batch

    def _run(self, requests, t_enq):
        t_start = _now_ns()
        if self.serial is not None:
            self.serial.acquire()
        self.sem.acquire()
        try:
            t0 = _now_ns()
            results = self.inst.execute(requests)
            t1 = _now_ns()
        finally:
            self.sem.release()
            if self.serial is not None:
                self.serial.release()
        if not self.model_reports:
            bs = sum(_batch_size(self.inst, r) for r in requests)
            self.stats.record_batch(bs, len(requests), 0, t1 - t0, 0)
        return results, t_start - t_enq

    async def submit(self, request):
        loop = asyncio.get_running_loop()
        t_enq = _now_ns()
        results, q_ns = await loop.run_in_executor(self.server.executor, self._run, [request], t_enq)
        res = results[0]
        ok = not isinstance(res, Exception)
        self.stats.record_request(ok, _now_ns() - t_enq, q_ns, _batch_size(self.inst, request))
        if not ok:
            raise res if isinstance(res, ServerError) else internal(str(res))
        return res

    def close(self):
        pass


def _override_preferred(entry):
    """dynamic_batching.preferred_batch_size of a repository load's config
    override (a deployment retuning the batcher of a loaded model: the native
    batcher takes it without reloading the model), or None."""
    db = (entry.config_override or {}).get("dynamic_batching")
    if not isinstance(db, dict) or "preferred_batch_size" not in db:
        return None
    return [int(x) for x in db["preferred_batch_size"]]


def _override_batching(entry, base):
    """The model's batcher settings (``base``: its dynamic_batching dict) with
    a config override's preferred_batch_size / max_queue_delay_microseconds
    applied, or ``base`` itself without an override."""
    db = (entry.config_override or {}).get("dynamic_batching")
    if base is None or not isinstance(db, dict):
        return base
    out = dict(base)
    if "preferred_batch_size" in db:
        out["preferred"] = [int(x) for x in db["preferred_batch_size"]]
    if "max_queue_delay_microseconds" in db:
        out["max_queue_delay_us"] = int(db["max_queue_delay_microseconds"])
    return out


class DynamicBatcher(DirectScheduler):
    """Collect requests into batches of <= max_batch_size rows.

    A batch is dispatched as soon as a preferred size is reached, or when the
    oldest request has waited ``max_queue_delay_us``; ``instance_count``
    batches may execute concurrently (e.g. on separate HIP streams).
    """

    def __init__(self, server, entry, inst, stats):
        super().__init__(server, entry, inst, stats)
        cfg = inst.dynamic_batching or {}
        self.max_bs = inst.max_batch_size
        self.preferred = sorted(cfg.get("preferred", []))
        self.delay_s = cfg.get("max_queue_delay_us", 0) / 1e6
        # idle-aware: wait for more rows only while another batch keeps the device busy
        self.idle_dispatch = bool(cfg.get("idle_dispatch", True))
        self.busy = 0
        self.queue = None
        self.tasks = []
        self.closed = False

    def _ensure(self):
        if self.queue is None:
            self.queue = asyncio.Queue()
            for _ in range(max(1, self.inst.instance_count)):
                self.tasks.append(asyncio.ensure_future(self._worker()))

    async def _worker(self):
        loop = asyncio.get_running_loop()
        pending = None
        while not self.closed:
            first = pending or await self.queue.get()
            pending = None
            batch = [first]
            rows = _batch_size(self.inst, first[0])
            deadline = loop.time() + self.delay_s
            while rows < self.max_bs:
                if self.preferred and rows in self.preferred and self.queue.empty():
                    break
                if self.idle_dispatch and self.busy == 0 and self.queue.empty():
                    break
                try:
                    if self.queue.empty():
                        timeout = deadline - loop.time()
                        if timeout <= 0:
                            break
                        item = await asyncio.wait_for(self.queue.get(), timeout)
                    else:
                        item = self.queue.get_nowait()
                except asyncio.TimeoutError:
                    break
                n = _batch_size(self.inst, item[0])
                if rows + n > self.max_bs:
                    pending = item
                    break
                batch.append(item)
                rows += n
            reqs = [b[0] for b in batch]
            t_enq = min(b[1] for b in batch)
            self.busy += 1
            try:
                results, _ = await loop.run_in_executor(self.server.executor, self._run, reqs, t_enq)
            except Exception as e:  # noqa: BLE001
                results = [e] * len(reqs)
            finally:
                self.busy -= 1
            now = _now_ns()
            for (req, t_in, fut), res in zip(batch, results):
                ok = not isinstance(res, Exception)
                self.stats.record_request(ok, now - t_in, 0, _batch_size(self.inst, req))
                if not fut.done():
                    if ok:
                        fut.set_result(res)
                    else:
                        fut.set_exception(res if isinstance(res, ServerError) else internal(str(res)))

    async def submit(self, request):
        self._ensure()
        fut = asyncio.get_running_loop().create_future()
        self.queue.put_nowait((request, _now_ns(), fut))
        return await fut

    def close(self):
        self.closed = True
        for t in self.tasks:
            t.cancel()


def make_scheduler(server, entry, inst, stats):
    if inst.dynamic_batching is not None and inst.max_batch_size > 0:
        return DynamicBatcher(server, entry, inst, stats)
    return DirectScheduler(server, entry, inst, stats)


def decode_b64(s):
    return base64.b64decode(s)
