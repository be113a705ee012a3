"""KServe-v2 gRPC front end (grpc.aio) for the in-repo server.

Serves every RPC of ``inference.GRPCInferenceService`` (grpc_service.proto).
ModelStreamInfer runs requests concurrently but keeps per-sequence order, and
implements decoupled responses plus ``triton_enable_empty_final_response`` /
``triton_final_response`` (reference src/c++/library/grpc_client.cc:422-446).
"""

import asyncio

import grpc
import numpy as np

from tritonclient.grpc import service_pb2, service_pb2_grpc
from tritonclient.utils import triton_to_np_dtype

from .core import EXTENSIONS, SERVER_NAME, SERVER_VERSION
from .http_frontend import _raw_output
from .types import InferRequest, InputTensor, RequestedOutput, ServerError, decode_raw

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


def _param_value(p):
    which = p.WhichOneof("parameter_choice")
    return getattr(p, which) if which else None


def _set_param(p, v):
    if isinstance(v, bool):
        p.bool_param = v
    elif isinstance(v, int):
        p.int64_param = v
    elif isinstance(v, float):
        p.double_param = v
    else:
        p.string_param = str(v)


def _code(e):
    if isinstance(e, ServerError):
        return getattr(grpc.StatusCode, e.grpc_code, grpc.StatusCode.INVALID_ARGUMENT), e.msg
    return grpc.StatusCode.INTERNAL, str(e)


FAULT_DELAY_KEY = "tc-fault-delay-ms"


class FaultInjector(grpc.aio.ServerInterceptor):
    """Test-server fault knob: a ``tc-fault-delay-ms`` request header delays the
    RPC before it is handled, so client deadlines on control-plane calls can be
    exercised (reference src/c++/tests/client_timeout_test.cc drives every
    API with a timeout against a slow server)."""

    async def intercept_service(self, continuation, handler_call_details):
        for k, v in handler_call_details.invocation_metadata or ():
            if k == FAULT_DELAY_KEY:
                try:
                    await asyncio.sleep(max(0.0, float(v)) / 1000.0)
                except ValueError:
                    pass
        return await continuation(handler_call_details)


class GrpcFrontend(service_pb2_grpc.GRPCInferenceServiceServicer):
    def __init__(self, server):
        self.s = server

    async def _abort(self, context, e):
        code, msg = _code(e)
        await context.abort(code, msg)

    # -- health / metadata ------------------------------------------------------------
    async def ServerLive(self, request, context):
        return service_pb2.ServerLiveResponse(live=True)

    async def ServerReady(self, request, context):
        return service_pb2.ServerReadyResponse(ready=self.s.ready)

    async def ModelReady(self, request, context):
        return service_pb2.ModelReadyResponse(ready=self.s.is_model_ready(request.name, request.version))

    async def ServerMetadata(self, request, context):
        return service_pb2.ServerMetadataResponse(
            name=SERVER_NAME, version=SERVER_VERSION, extensions=EXTENSIONS
        )

    async def ModelMetadata(self, request, context):
        try:
            md = self.s.model_metadata(request.name, request.version)
        except Exception as e:
            await self._abort(context, e)
        resp = service_pb2.ModelMetadataResponse(
            name=md["name"], versions=md["versions"], platform=md["platform"]
        )
        for t in md["inputs"]:
            resp.inputs.add(name=t["name"], datatype=t["datatype"], shape=t["shape"])
        for t in md["outputs"]:
            resp.outputs.add(name=t["name"], datatype=t["datatype"], shape=t["shape"])
        return resp

    async def ModelConfig(self, request, context):
        try:
            cfg = self.s.model_config_proto(request.name, request.version)
        except Exception as e:
            await self._abort(context, e)
        return service_pb2.ModelConfigResponse(config=cfg)

    async def ModelStatistics(self, request, context):
        try:
            st = self.s.statistics(request.name, request.version)
        except Exception as e:
            await self._abort(context, e)
        resp = service_pb2.ModelStatisticsResponse()
        for m in st["model_stats"]:
            ms = resp.model_stats.add(
                name=m["name"],
                version=m["version"],
                last_inference=m["last_inference"],
                inference_count=m["inference_count"],
                execution_count=m["execution_count"],
            )
            for k, v in m["inference_stats"].items():
                getattr(ms.inference_stats, k).count = v["count"]
                getattr(ms.inference_stats, k).ns = v["ns"]
            for b in m["batch_stats"]:
                bs = ms.batch_stats.add(batch_size=b["batch_size"])
                for k in ("compute_input", "compute_infer", "compute_output"):
                    getattr(bs, k).count = b[k]["count"]
                    getattr(bs, k).ns = b[k]["ns"]
        return resp

    # -- repository -----------------------------------------------------------------------
    async def RepositoryIndex(self, request, context):
        resp = service_pb2.RepositoryIndexResponse()
        for m in self.s.repository_index():
            if request.ready and m["state"] != "READY":
                continue
            resp.models.add(
                name=m["name"], version=m["version"], state=m["state"], reason=m.get("reason", "")
            )
        return resp

    async def RepositoryModelLoad(self, request, context):
        config = None
        files = {}
        for k, p in request.parameters.items():
            which = p.WhichOneof("parameter_choice")
            if k == "config":
                config = p.string_param
            elif k.startswith("file:"):
                files[k] = p.bytes_param if which == "bytes_param" else str(_param_value(p)).encode()
        try:
            self.s.load_model(request.model_name, config=config, files=files or None)
        except Exception as e:
            await self._abort(context, e)
        return service_pb2.RepositoryModelLoadResponse()

    async def RepositoryModelUnload(self, request, context):
        dep = False
        if "unload_dependents" in request.parameters:
            dep = bool(request.parameters["unload_dependents"].bool_param)
        try:
            self.s.unload_model(request.model_name, dep)
        except Exception as e:
            await self._abort(context, e)
        return service_pb2.RepositoryModelUnloadResponse()

    # -- shared memory -----------------------------------------------------------------------
    async def SystemSharedMemoryStatus(self, request, context):
        try:
            regions = self.s.sys_shm.status(request.name)
        except Exception as e:
            await self._abort(context, e)
        resp = service_pb2.SystemSharedMemoryStatusResponse()
        for r in regions:
            rs = resp.regions[r["name"]]
            rs.name, rs.key, rs.offset, rs.byte_size = r["name"], r["key"], r["offset"], r["byte_size"]
        return resp

    async def SystemSharedMemoryRegister(self, request, context):
        try:
            self.s.sys_shm.register(request.name, request.key, request.offset, request.byte_size)
        except Exception as e:
            await self._abort(context, e)
        return service_pb2.SystemSharedMemoryRegisterResponse()

    async def SystemSharedMemoryUnregister(self, request, context):
        self.s.sys_shm.unregister(request.name)
        return service_pb2.SystemSharedMemoryUnregisterResponse()

    async def CudaSharedMemoryStatus(self, request, context):
        try:
            regions = self.s.dev_shm.status(request.name)
        except Exception as e:
            await self._abort(context, e)
        resp = service_pb2.CudaSharedMemoryStatusResponse()
        for r in regions:
            rs = resp.regions[r["name"]]
            rs.name, rs.device_id, rs.byte_size = r["name"], r["device_id"], r["byte_size"]
        return resp

    async def CudaSharedMemoryRegister(self, request, context):
        try:
            self.s.dev_shm.register(request.name, request.raw_handle, request.device_id, request.byte_size)
        except Exception as e:
            await self._abort(context, e)
        return service_pb2.CudaSharedMemoryRegisterResponse()

    async def CudaSharedMemoryUnregister(self, request, context):
        self.s.dev_shm.unregister(request.name)
        return service_pb2.CudaSharedMemoryUnregisterResponse()

    # -- trace / log ----------------------------------------------------------------------------
    async def TraceSetting(self, request, context):
        try:
            if request.settings:
                upd = {}
                for k, v in request.settings.items():
                    upd[k] = list(v.value) if len(v.value) else None
                cur = self.s.update_trace(request.model_name, upd)
            else:
                cur = self.s.get_trace(request.model_name)
        except Exception as e:
            await self._abort(context, e)
        resp = service_pb2.TraceSettingResponse()
        for k, v in cur.items():
            vals = v if isinstance(v, list) else [v]
            resp.settings[k].value.extend([str(x) for x in vals if x is not None])
        return resp

    async def LogSettings(self, request, context):
        try:
            if request.settings:
                upd = {k: _param_value(v) for k, v in request.settings.items()}
                cur = self.s.update_log(upd)
            else:
                cur = dict(self.s.log_settings)
        except Exception as e:
            await self._abort(context, e)
        resp = service_pb2.LogSettingsResponse()
        for k, v in cur.items():
            if isinstance(v, bool):
                resp.settings[k].bool_param = v
            elif isinstance(v, int):
                resp.settings[k].uint32_param = v
            else:
                resp.settings[k].string_param = str(v)
        return resp

    # -- inference ---------------------------------------------------------------------------------
    def decode(self, request):
        req = InferRequest(model_name=request.model_name, model_version=request.model_version)
        req.id = request.id
        req.parameters = {k: _param_value(v) for k, v in request.parameters.items()}
        raw_idx = 0
        n_raw = len(request.raw_input_contents)
        for t in request.inputs:
            tp = {k: _param_value(v) for k, v in t.parameters.items()}
            tensor = InputTensor(t.name, t.datatype, list(t.shape))
            if "shared_memory_region" in tp:
                self.s.resolve_shm_input(tensor, tp)
            elif t.HasField("contents"):
                field = _TYPED.get(t.datatype)
                vals = getattr(t.contents, field) if field else []
                if t.datatype == "BYTES":
                    arr = np.empty(len(vals), dtype=np.object_)
                    arr[:] = list(vals)
                else:
                    arr = np.array(vals, dtype=triton_to_np_dtype(t.datatype))
                n = int(np.prod(tensor.shape)) if tensor.shape else 1
                if arr.size != n:
                    raise ServerError(
                        "unexpected number of elements in contents of input '%s'" % t.name
                    )
                tensor.data = arr.reshape(tensor.shape)
            else:
                if raw_idx >= n_raw:
                    raise ServerError("input '%s' has no data" % t.name)
                tensor.data = decode_raw(request.raw_input_contents[raw_idx], t.datatype, tensor.shape)
                raw_idx += 1
            req.inputs.append(tensor)
        if raw_idx != n_raw and n_raw:
            raise ServerError(
                "raw_input_contents count (%d) does not match the inputs without shm/contents (%d)"
                % (n_raw, raw_idx)
            )
        for o in request.outputs:
            op = {k: _param_value(v) for k, v in o.parameters.items()}
            ro = RequestedOutput(o.name, binary=True, class_count=int(op.get("classification", 0) or 0))
            if "shared_memory_region" in op:
                ro.shm = (
                    op["shared_memory_region"],
                    int(op["shared_memory_byte_size"]),
                    int(op.get("shared_memory_offset", 0) or 0),
                )
            req.outputs.append(ro)
        return req

    def encode(self, resp):
        out = service_pb2.ModelInferResponse(
            model_name=resp.model_name, model_version=resp.model_version, id=resp.id
        )
        for k, v in resp.parameters.items():
            _set_param(out.parameters[k], v)
        raws = []
        for o, _ in resp.outputs:
            t = out.outputs.add(name=o.name, datatype=o.datatype, shape=[int(x) for x in o.shape])
            if o.shm is not None:
                region, nbytes, offset = o.shm
                t.parameters["shared_memory_region"].string_param = region
                t.parameters["shared_memory_byte_size"].int64_param = nbytes
                if offset:
                    t.parameters["shared_memory_offset"].int64_param = offset
                raws.append(None)
            else:
                raws.append(bytes(_raw_output(o.data, o.datatype)))
        # raw_output_contents is indexed by output position on the client side
        # (reference grpc/_infer_result.py:62-90): keep positions aligned.
        last = max((i for i, r in enumerate(raws) if r is not None), default=-1)
        for r in raws[: last + 1]:
            out.raw_output_contents.append(r if r is not None else b"")
        return out

    async def ModelInfer(self, request, context):
        try:
            req = self.decode(request)
            resp = await self.s.infer(req)
            return self.encode(resp)
        except Exception as e:
            await self._abort(context, e)

    async def ModelStreamInfer(self, request_iterator, context):
        q = asyncio.Queue()
        seq_locks = {}
        tasks = set()

        async def handle(proto):
            try:
                req = self.decode(proto)
            except Exception as e:
                await q.put(service_pb2.ModelStreamInferResponse(error_message=_code(e)[1]))
                return

            async def emit(resp):
                await q.put(service_pb2.ModelStreamInferResponse(infer_response=self.encode(resp)))

            sid = req.sequence_id
            lock = None
            if sid not in (0, "", None):
                lock = seq_locks.setdefault(sid, asyncio.Lock())
            try:
                if lock is not None:
                    async with lock:
                        await self.s.stream_infer(req, emit)
                else:
                    await self.s.stream_infer(req, emit)
            except Exception as e:
                await q.put(service_pb2.ModelStreamInferResponse(error_message=_code(e)[1]))

        async def reader():
            prev = {}
            async for proto in request_iterator:
                # requests of one sequence must start in arrival order
                sid_p = proto.parameters.get("sequence_id") if "sequence_id" in proto.parameters else None
                key = _param_value(sid_p) if sid_p is not None else None
                t = asyncio.ensure_future(self._ordered(handle, proto, prev.get(key) if key else None))
                if key:
                    prev[key] = t
                tasks.add(t)
                t.add_done_callback(tasks.discard)
            while tasks:
                await asyncio.gather(*list(tasks), return_exceptions=True)
            await q.put(None)

        rt = asyncio.ensure_future(reader())
        try:
            while True:
                item = await q.get()
                if item is None:
                    break
                yield item
        finally:
            rt.cancel()

    @staticmethod
    async def _ordered(handle, proto, prev_task):
        if prev_task is not None:
            try:
                await asyncio.shield(prev_task)
            except Exception:
                pass
        await handle(proto)
