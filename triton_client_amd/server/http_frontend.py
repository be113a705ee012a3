"""KServe-v2 REST front end (aiohttp) for the in-repo server.

Implements every route the reference clients call (SURVEY.md §2.7,
reference src/c++/library/http_client.cc:1393-1764, tritonclient/http/_client.py:340-1217),
including the binary-tensor extension (``Inference-Header-Content-Length``),
gzip/deflate in both directions, system/device shared memory and the
``hipsharedmemory`` alias routes.
"""

import asyncio
import gzip
import json
import zlib

import numpy as np
from aiohttp import web

from tritonclient.utils import (
    serialize_bf16_tensor,
    serialize_byte_tensor,
    serialize_fp8_tensor,
    triton_to_np_dtype,
)

from .core import EXTENSIONS, SERVER_NAME, SERVER_VERSION, decode_b64
from .types import InferRequest, InputTensor, RequestedOutput, ServerError, decode_raw


def _dumps(obj):
    return json.dumps(obj, separators=(",", ":"))


def _err(e):
    if isinstance(e, ServerError):
        return web.Response(status=e.http_status, text=_dumps({"error": e.msg}), content_type="application/json")
    return web.Response(status=500, text=_dumps({"error": str(e)}), content_type="application/json")


def _json_resp(obj):
    return web.Response(body=_dumps(obj).encode(), content_type="application/json")


async def _read_json(request):
    body = await request.read()
    if not body:
        return {}
    try:
        return json.loads(body)
    except Exception as e:
        raise ServerError("failed to parse the request JSON buffer: %s" % e)


def _json_to_array(data, datatype, shape):
    if datatype == "BYTES":
        flat = []

        def walk(x):
            if isinstance(x, list):
                for y in x:
                    walk(y)
            else:
                flat.append(x.encode("utf-8") if isinstance(x, str) else bytes(x))

        walk(data)
        arr = np.empty(len(flat), dtype=np.object_)
        arr[:] = flat
    elif datatype in ("BF16", "FP8_E4M3", "FP8_E5M2"):
        raise ServerError("%s inputs must be sent as binary data" % datatype)
    else:
        dt = triton_to_np_dtype(datatype)
        if dt is None:
            raise ServerError("invalid datatype '%s'" % datatype)
        arr = np.array(data, dtype=dt).reshape(-1)
    n = int(np.prod(shape)) if len(shape) else 1
    if arr.size != n:
        raise ServerError(
            "unexpected number of elements %d in JSON data for shape %s" % (arr.size, list(shape))
        )
    return arr.reshape(shape)


def _array_to_json(arr, datatype):
    if datatype == "BYTES":
        out = []
        for x in np.asarray(arr).reshape(-1).tolist():
            if isinstance(x, bytes):
                try:
                    out.append(x.decode("utf-8"))
                except UnicodeDecodeError:
                    raise ServerError("output contains non-UTF-8 bytes; request it as binary")
            else:
                out.append(str(x))
        return out
    if datatype in ("BF16", "FP8_E4M3", "FP8_E5M2"):
        raise ServerError("%s outputs must be returned as binary data" % datatype)
    return np.asarray(arr).reshape(-1).tolist()


def _raw_output(arr, datatype):
    if hasattr(arr, "is_cuda"):
        arr = arr.detach().cpu().numpy()
    if datatype == "BYTES":
        s = serialize_byte_tensor(np.asarray(arr, dtype=np.object_))
        return s.item() if s.size else b""
    if datatype == "BF16":
        s = serialize_bf16_tensor(np.asarray(arr, dtype=np.float32))
        return s.item() if s.size else b""
    if datatype in ("FP8_E4M3", "FP8_E5M2"):
        s = serialize_fp8_tensor(np.asarray(arr, dtype=np.float32), datatype)
        return s.item() if s.size else b""
    return memoryview(np.ascontiguousarray(arr)).cast("B")


@web.middleware
async def fault_delay(request, handler):
    """Test-server fault knob (see grpc_frontend.FaultInjector): a
    ``tc-fault-delay-ms`` header delays the response."""
    d = request.headers.get("tc-fault-delay-ms")
    if d:
        try:
            await asyncio.sleep(max(0.0, float(d)) / 1000.0)
        except ValueError:
            pass
    return await handler(request)


class HttpFrontend:
    def __init__(self, server):
        self.s = server
        app = web.Application(client_max_size=2**31 - 1, middlewares=[fault_delay])
        r = app.router
        r.add_get("/v2/health/live", self.live)
        r.add_get("/v2/health/ready", self.ready)
        r.add_get("/v2", self.server_metadata)
        r.add_get("/v2/", self.server_metadata)
        r.add_get("/v2/models/stats", self.stats)
        r.add_post("/v2/repository/index", self.repo_index)
        r.add_post("/v2/repository/models/{model}/load", self.load)
        r.add_post("/v2/repository/models/{model}/unload", self.unload)
        r.add_get("/v2/trace/setting", self.get_trace)
        r.add_post("/v2/trace/setting", self.update_trace)
        r.add_get("/v2/logging", self.get_log)
        r.add_post("/v2/logging", self.update_log)
        for kind in ("systemsharedmemory", "cudasharedmemory", "hipsharedmemory"):
            r.add_get("/v2/%s/status" % kind, self.shm_status)
            r.add_get("/v2/%s/region/{region}/status" % kind, self.shm_status)
            r.add_post("/v2/%s/region/{region}/register" % kind, self.shm_register)
            r.add_post("/v2/%s/unregister" % kind, self.shm_unregister)
            r.add_post("/v2/%s/region/{region}/unregister" % kind, self.shm_unregister)
        for base in ("/v2/models/{model}", "/v2/models/{model}/versions/{version}"):
            r.add_get(base, self.model_metadata)
            r.add_get(base + "/ready", self.model_ready)
            r.add_get(base + "/config", self.model_config)
            r.add_get(base + "/stats", self.stats)
            r.add_post(base + "/infer", self.infer)
            r.add_get(base + "/trace/setting", self.get_trace)
            r.add_post(base + "/trace/setting", self.update_trace)
        self.app = app

    # -- health / metadata -----------------------------------------------------------
    async def live(self, request):
        return web.Response(status=200)

    async def ready(self, request):
        return web.Response(status=200 if self.s.ready else 400)

    async def server_metadata(self, request):
        return _json_resp({"name": SERVER_NAME, "version": SERVER_VERSION, "extensions": EXTENSIONS})

    async def model_metadata(self, request):
        try:
            m = request.match_info
            return _json_resp(self.s.model_metadata(m["model"], m.get("version", "")))
        except Exception as e:
            return _err(e)

    async def model_ready(self, request):
        m = request.match_info
        ok = self.s.is_model_ready(m["model"], m.get("version", ""))
        return web.Response(status=200 if ok else 400)

    async def model_config(self, request):
        try:
            m = request.match_info
            return _json_resp(self.s.model_config(m["model"], m.get("version", "")))
        except Exception as e:
            return _err(e)

    async def stats(self, request):
        try:
            m = request.match_info
            return _json_resp(self.s.statistics(m.get("model", ""), m.get("version", "")))
        except Exception as e:
            return _err(e)

    # -- repository -------------------------------------------------------------------
    async def repo_index(self, request):
        return _json_resp(self.s.repository_index())

    async def load(self, request):
        try:
            body = await _read_json(request)
            params = body.get("parameters", {}) if isinstance(body, dict) else {}
            config = params.get("config")
            files = {k: decode_b64(v) for k, v in params.items() if k.startswith("file:")}
            self.s.load_model(request.match_info["model"], config=config, files=files or None)
            return web.Response(status=200)
        except Exception as e:
            return _err(e)

    async def unload(self, request):
        try:
            body = await _read_json(request)
            params = body.get("parameters", {}) if isinstance(body, dict) else {}
            self.s.unload_model(request.match_info["model"], bool(params.get("unload_dependents", False)))
            return web.Response(status=200)
        except Exception as e:
            return _err(e)

    # -- trace / log -----------------------------------------------------------------------
    async def get_trace(self, request):
        try:
            return _json_resp(self.s.get_trace(request.match_info.get("model")))
        except Exception as e:
            return _err(e)

    async def update_trace(self, request):
        try:
            body = await _read_json(request)
            return _json_resp(self.s.update_trace(request.match_info.get("model"), body))
        except Exception as e:
            return _err(e)

    async def get_log(self, request):
        return _json_resp(self.s.log_settings)

    async def update_log(self, request):
        try:
            return _json_resp(self.s.update_log(await _read_json(request)))
        except Exception as e:
            return _err(e)

    # -- shared memory ------------------------------------------------------------------------
    def _reg(self, request):
        return self.s.sys_shm if "/systemsharedmemory/" in request.path else self.s.dev_shm

    async def shm_status(self, request):
        try:
            return _json_resp(self._reg(request).status(request.match_info.get("region", "")))
        except Exception as e:
            return _err(e)

    async def shm_register(self, request):
        try:
            body = await _read_json(request)
            name = request.match_info["region"]
            if "/systemsharedmemory/" in request.path:
                self.s.sys_shm.register(
                    name, body["key"], int(body.get("offset", 0)), int(body["byte_size"])
                )
            else:
                raw = decode_b64(body["raw_handle"]["b64"])
                self.s.dev_shm.register(name, raw, int(body["device_id"]), int(body["byte_size"]))
            return web.Response(status=200)
        except KeyError as e:
            return _err(ServerError("missing field %s in register request" % e))
        except Exception as e:
            return _err(e)

    async def shm_unregister(self, request):
        try:
            self._reg(request).unregister(request.match_info.get("region", ""))
            return web.Response(status=200)
        except Exception as e:
            return _err(e)

    # -- inference -------------------------------------------------------------------------------
    def decode_infer(self, request, body):
        m = request.match_info
        # aiohttp inflates gzip/deflate request bodies itself; only decode here
        # when the payload still carries the compressed framing.
        enc = request.headers.get("Content-Encoding")
        if enc == "gzip" and body[:2] == b"\x1f\x8b":
            body = gzip.decompress(body)
        elif enc == "deflate" and body[:1] == b"\x78":
            try:
                body = zlib.decompress(body)
            except zlib.error:
                pass
        hlen = request.headers.get("Inference-Header-Content-Length")
        if hlen is not None:
            hlen = int(hlen)
            header = json.loads(body[:hlen])
            binary = memoryview(body)[hlen:]
        else:
            header = json.loads(body) if body else {}
            binary = memoryview(b"")
        req = InferRequest(model_name=m["model"], model_version=m.get("version", ""))
        req.id = header.get("id", "")
        params = header.get("parameters", {}) or {}
        req.parameters = dict(params)
        req.binary_data_output = bool(params.get("binary_data_output", False))
        pos = 0
        for t in header.get("inputs", []):
            tp = t.get("parameters", {}) or {}
            tensor = InputTensor(t["name"], t["datatype"], list(t.get("shape", [])))
            if "shared_memory_region" in tp:
                self.s.resolve_shm_input(tensor, tp)
            elif "binary_data_size" in tp:
                n = int(tp["binary_data_size"])
                if pos + n > len(binary):
                    raise ServerError("unexpected end of binary data for input '%s'" % t["name"])
                tensor.data = decode_raw(binary[pos : pos + n], tensor.datatype, tensor.shape)
                pos += n
            elif "data" in t:
                tensor.data = _json_to_array(t["data"], tensor.datatype, tensor.shape)
                self.s.wire_stats["json_input_tensors"] += 1
            else:
                raise ServerError("input '%s' has no data" % t["name"])
            req.inputs.append(tensor)
        for o in header.get("outputs", []) or []:
            op = o.get("parameters", {}) or {}
            ro = RequestedOutput(
                o["name"],
                binary=bool(op.get("binary_data", req.binary_data_output)),
                class_count=int(op.get("classification", 0)),
            )
            if "shared_memory_region" in op:
                ro.shm = (
                    op["shared_memory_region"],
                    int(op["shared_memory_byte_size"]),
                    int(op.get("shared_memory_offset", 0)),
                )
            req.outputs.append(ro)
        return req

    def encode_infer(self, req, resp, accept):
        header = {"model_name": resp.model_name, "model_version": resp.model_version}
        if resp.id:
            header["id"] = resp.id
        if resp.parameters:
            header["parameters"] = resp.parameters
        outs = []
        blobs = []
        for o, ro in resp.outputs:
            d = {"name": o.name, "datatype": o.datatype, "shape": [int(x) for x in o.shape]}
            if o.shm is not None:
                region, nbytes, offset = o.shm
                p = {"shared_memory_region": region, "shared_memory_byte_size": nbytes}
                if offset:
                    p["shared_memory_offset"] = offset
                d["parameters"] = p
            else:
                binary = ro.binary if ro is not None else req.binary_data_output
                if binary:
                    raw = _raw_output(o.data, o.datatype)
                    d["parameters"] = {"binary_data_size": len(raw)}
                    blobs.append(raw)
                else:
                    data = o.data.detach().cpu().numpy() if hasattr(o.data, "is_cuda") else o.data
                    d["data"] = _array_to_json(data, o.datatype)
                    self.s.wire_stats["json_output_tensors"] += 1
            outs.append(d)
        header["outputs"] = outs
        hbytes = _dumps(header).encode()
        headers = {}
        if blobs:
            body = b"".join([hbytes] + [bytes(b) for b in blobs])
            headers["Inference-Header-Content-Length"] = str(len(hbytes))
            ctype = "application/octet-stream"
        else:
            body = hbytes
            ctype = "application/json"
        if accept:
            if "gzip" in accept:
                body = gzip.compress(body, compresslevel=1)
                headers["Content-Encoding"] = "gzip"
            elif "deflate" in accept:
                body = zlib.compress(body, 1)
                headers["Content-Encoding"] = "deflate"
        return web.Response(body=body, headers=headers, content_type=ctype)

    async def infer(self, request):
        try:
            body = await request.read()
            req = self.decode_infer(request, body)
            resp = await self.s.infer(req)
            return self.encode_infer(req, resp, request.headers.get("Accept-Encoding"))
        except json.JSONDecodeError as e:
            return _err(ServerError("failed to parse the request JSON buffer: %s" % e))
        except Exception as e:
            return _err(e)
