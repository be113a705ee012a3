"""asyncio KServe-v2 REST client.

API parity with reference ``tritonclient/http/aio/__init__.py:92-775``: the
same ``InferenceServerClient`` methods as the synchronous client, as
coroutines (``async with`` support, ``close()``), ``generate_request_body`` /
``parse_response_body`` statics, plugins, gzip/deflate.  The request codec is
shared with the sync client (``tritonclient/http/_utils.py``); the body is
sent as one chunked-free payload assembled from the header + tensor buffers.

Transport: an asyncio Protocol keep-alive pool (``_transport.py``) instead of
the reference's aiohttp session; ``conn_limit`` / ``conn_timeout`` / ``ssl`` /
``ssl_context`` keep their meaning.
"""

import asyncio
import base64
import gzip
import json
import ssl as _ssl
import zlib
from urllib.parse import quote

from tritonclient.utils import raise_error

from ..._client import InferenceServerClientBase
from ..._request import Request
from .._infer_input import InferInput
from .._infer_result import InferResult
from .._requested_output import InferRequestedOutput
from .._utils import _dumps, _get_error, _get_inference_request, _get_inference_request_parts, _get_query_string
from ...utils import InferenceServerException  # noqa: F401
from ._transport import HttpTransportError, Pool

__all__ = ["InferenceServerClient", "InferInput", "InferRequestedOutput", "InferResult", "InferenceServerException"]


class _Resp:
    """Adapter so the shared error decoder can read an aiohttp response."""

    def __init__(self, status, body, headers):
        self.status_code = status
        self._body = body
        self.headers = headers

    def read(self):
        return self._body


def _raise_if_error(resp):
    err = _get_error(resp)
    if err is not None:
        raise err


class InferenceServerClient(InferenceServerClientBase):
    """asyncio client; one instance per event loop (not thread-safe)."""

    def __init__(self, url, verbose=False, conn_limit=100, conn_timeout=60.0, ssl=False, ssl_context=None):
        super().__init__()
        if url.startswith("http://") or url.startswith("https://"):
            raise_error("url should not include the scheme")
        scheme = "https://" if ssl else "http://"
        self._url = scheme + (url if url[-1] != "/" else url[:-1])
        hostport, _, prefix = url.partition("/")
        self._prefix = ("/" + prefix.rstrip("/")) if prefix.strip("/") else ""
        host, _, port = hostport.rpartition(":") if ":" in hostport else (hostport, "", "")
        if not port:
            host, port = hostport, ("443" if ssl else "80")
        if ssl and ssl_context is None:
            ssl_context = _ssl.create_default_context()
        self._pool = Pool(host.strip("[]"), int(port), ssl_context if ssl else None, conn_limit)
        self._timeout = conn_timeout
        self._verbose = verbose

    async def __aenter__(self):
        return self

    async def __aexit__(self, type, value, traceback):
        await self.close()

    async def close(self):
        """Close the client's HTTP connections."""
        self._pool.close()

    # -- transport ------------------------------------------------------------------
    def _headers(self, headers):
        request = Request(dict(headers) if headers else {})
        self._call_plugin(request)
        self._validate_headers(request.headers)
        return {k: str(v) for k, v in request.headers.items()}

    def _validate_headers(self, headers):
        if headers and any(k.lower() == "transfer-encoding" for k in headers):
            raise_error(
                "Unsupported HTTP header: 'Transfer-Encoding' is not supported in the Python client "
                "library. Use raw HTTP request libraries or the C++ client instead for this header."
            )

    def _uri(self, request_uri, query_params):
        uri = self._url + "/" + request_uri
        if query_params is not None:
            uri = uri + "?" + _get_query_string(query_params)
        return uri

    def _path(self, request_uri, query_params):
        path = self._prefix + "/" + request_uri
        if query_params is not None:
            path = path + "?" + _get_query_string(query_params)
        return path

    async def _send(self, method, request_uri, headers, query_params, body=None):
        path = self._path(request_uri, query_params)
        try:
            r = await asyncio.wait_for(self._pool.request(method, path, headers, body), self._timeout)
        except asyncio.TimeoutError:
            raise_error("HTTP %s %s timed out after %s s" % (method, self._uri(request_uri, query_params),
                                                             self._timeout))
        except (HttpTransportError, OSError) as e:
            raise_error("HTTP %s %s failed: %s" % (method, self._uri(request_uri, query_params), e))
        return _Resp(r.status, r.body, r.headers)

    async def _get(self, request_uri, headers, query_params):
        headers = self._headers(headers)
        if self._verbose:
            print("GET {}, headers {}".format(self._uri(request_uri, query_params), headers))
        resp = await self._send("GET", request_uri, headers, query_params)
        if self._verbose:
            print(resp.status_code, resp.read())
        return resp

    async def _post(self, request_uri, request_body, headers, query_params):
        headers = self._headers(headers)
        if isinstance(request_body, str):
            request_body = request_body.encode()
        if self._verbose:
            shown = request_body if isinstance(request_body, (bytes, bytearray)) else b"".join(
                bytes(p) for p in request_body)
            print("POST {}, headers {}\n{}".format(self._uri(request_uri, query_params), headers, shown[:256]))
        resp = await self._send("POST", request_uri, headers, query_params, request_body)
        if self._verbose:
            print(resp.status_code, resp.read()[:256])
        return resp

    async def _get_json(self, uri, headers, query_params):
        r = await self._get(uri, headers, query_params)
        _raise_if_error(r)
        return json.loads(r.read())

    async def _post_json(self, uri, body, headers, query_params):
        r = await self._post(uri, body, headers, query_params)
        _raise_if_error(r)
        return json.loads(r.read())

    @staticmethod
    def _model_uri(model_name, model_version, suffix=""):
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        if model_version != "":
            return "v2/models/{}/versions/{}{}".format(quote(model_name), model_version, suffix)
        return "v2/models/{}{}".format(quote(model_name), suffix)

    # -- health / metadata ---------------------------------------------------------
    async def is_server_live(self, headers=None, query_params=None):
        return (await self._get("v2/health/live", headers, query_params)).status_code == 200

    async def is_server_ready(self, headers=None, query_params=None):
        return (await self._get("v2/health/ready", headers, query_params)).status_code == 200

    async def is_model_ready(self, model_name, model_version="", headers=None, query_params=None):
        uri = self._model_uri(model_name, model_version, "/ready")
        return (await self._get(uri, headers, query_params)).status_code == 200

    async def get_server_metadata(self, headers=None, query_params=None):
        return await self._get_json("v2", headers, query_params)

    async def get_model_metadata(self, model_name, model_version="", headers=None, query_params=None):
        return await self._get_json(self._model_uri(model_name, model_version), headers, query_params)

    async def get_model_config(self, model_name, model_version="", headers=None, query_params=None):
        return await self._get_json(self._model_uri(model_name, model_version, "/config"), headers, query_params)

    # -- repository -------------------------------------------------------------------
    async def get_model_repository_index(self, headers=None, query_params=None):
        return await self._post_json("v2/repository/index", "", headers, query_params)

    async def load_model(self, model_name, headers=None, query_params=None, config=None, files=None):
        uri = "v2/repository/models/{}/load".format(quote(model_name))
        load_request = {}
        if config is not None:
            load_request.setdefault("parameters", {})["config"] = config
        if files is not None:
            for path, content in files.items():
                load_request.setdefault("parameters", {})[path] = base64.b64encode(content).decode("ascii")
        r = await self._post(uri, _dumps(load_request), headers, query_params)
        _raise_if_error(r)
        if self._verbose:
            print("Loaded model '{}'".format(model_name))

    async def unload_model(self, model_name, headers=None, query_params=None, unload_dependents=False):
        uri = "v2/repository/models/{}/unload".format(quote(model_name))
        r = await self._post(uri, _dumps({"parameters": {"unload_dependents": unload_dependents}}), headers,
                             query_params)
        _raise_if_error(r)
        if self._verbose:
            print("Unloaded model '{}'".format(model_name))

    # -- statistics / trace / log ----------------------------------------------------
    async def get_inference_statistics(self, model_name="", model_version="", headers=None, query_params=None):
        uri = self._model_uri(model_name, model_version, "/stats") if model_name != "" else "v2/models/stats"
        return await self._get_json(uri, headers, query_params)

    async def update_trace_settings(self, model_name=None, settings={}, headers=None, query_params=None):
        uri = "v2/models/{}/trace/setting".format(quote(model_name)) if model_name else "v2/trace/setting"
        return await self._post_json(uri, _dumps(settings), headers, query_params)

    async def get_trace_settings(self, model_name=None, headers=None, query_params=None):
        uri = "v2/models/{}/trace/setting".format(quote(model_name)) if model_name else "v2/trace/setting"
        return await self._get_json(uri, headers, query_params)

    async def update_log_settings(self, settings, headers=None, query_params=None):
        return await self._post_json("v2/logging", _dumps(settings), headers, query_params)

    async def get_log_settings(self, headers=None, query_params=None):
        return await self._get_json("v2/logging", headers, query_params)

    # -- shared memory ----------------------------------------------------------------
    async def get_system_shared_memory_status(self, region_name="", headers=None, query_params=None):
        uri = ("v2/systemsharedmemory/region/{}/status".format(quote(region_name)) if region_name
               else "v2/systemsharedmemory/status")
        return await self._get_json(uri, headers, query_params)

    async def register_system_shared_memory(self, name, key, byte_size, offset=0, headers=None, query_params=None):
        uri = "v2/systemsharedmemory/region/{}/register".format(quote(name))
        r = await self._post(uri, _dumps({"key": key, "offset": offset, "byte_size": byte_size}), headers,
                             query_params)
        _raise_if_error(r)

    async def unregister_system_shared_memory(self, name="", headers=None, query_params=None):
        uri = ("v2/systemsharedmemory/region/{}/unregister".format(quote(name)) if name
               else "v2/systemsharedmemory/unregister")
        r = await self._post(uri, "", headers, query_params)
        _raise_if_error(r)

    async def get_cuda_shared_memory_status(self, region_name="", headers=None, query_params=None):
        uri = ("v2/cudasharedmemory/region/{}/status".format(quote(region_name)) if region_name
               else "v2/cudasharedmemory/status")
        return await self._get_json(uri, headers, query_params)

    async def register_cuda_shared_memory(self, name, raw_handle, device_id, byte_size, headers=None,
                                          query_params=None):
        uri = "v2/cudasharedmemory/region/{}/register".format(quote(name))
        if isinstance(raw_handle, bytes):
            raw_handle = raw_handle.decode("ascii")
        body = _dumps({"raw_handle": {"b64": raw_handle}, "device_id": device_id, "byte_size": byte_size})
        r = await self._post(uri, body, headers, query_params)
        _raise_if_error(r)

    async def unregister_cuda_shared_memory(self, name="", headers=None, query_params=None):
        uri = ("v2/cudasharedmemory/region/{}/unregister".format(quote(name)) if name
               else "v2/cudasharedmemory/unregister")
        r = await self._post(uri, "", headers, query_params)
        _raise_if_error(r)

    get_hip_shared_memory_status = get_cuda_shared_memory_status
    register_hip_shared_memory = register_cuda_shared_memory
    unregister_hip_shared_memory = unregister_cuda_shared_memory

    # -- inference ------------------------------------------------------------------------
    @staticmethod
    def generate_request_body(inputs, outputs=None, request_id="", sequence_id=0, sequence_start=False,
                              sequence_end=False, priority=0, timeout=None, parameters=None):
        return _get_inference_request(inputs=inputs, request_id=request_id, outputs=outputs,
                                      sequence_id=sequence_id, sequence_start=sequence_start,
                                      sequence_end=sequence_end, priority=priority, timeout=timeout,
                                      custom_parameters=parameters)

    @staticmethod
    def parse_response_body(response_body, verbose=False, header_length=None, content_encoding=None):
        return InferResult.from_response_body(response_body, verbose, header_length, content_encoding)

    async def infer(self, model_name, inputs, model_version="", outputs=None, request_id="", sequence_id=0,
                    sequence_start=False, sequence_end=False, priority=0, timeout=None, headers=None,
                    query_params=None, request_compression_algorithm=None, response_compression_algorithm=None,
                    parameters=None):
        """Run inference; returns :class:`tritonclient.http.InferResult`."""
        parts, json_size = _get_inference_request_parts(
            inputs, request_id=request_id, outputs=outputs, sequence_id=sequence_id,
            sequence_start=sequence_start, sequence_end=sequence_end, priority=priority, timeout=timeout,
            custom_parameters=parameters)
        body = parts  # header + tensor buffers, written with one writelines (no join)
        headers = dict(headers) if headers else {}
        if request_compression_algorithm == "gzip":
            headers["Content-Encoding"] = "gzip"
            body = gzip.compress(b"".join(bytes(p) for p in parts))
        elif request_compression_algorithm == "deflate":
            headers["Content-Encoding"] = "deflate"
            body = zlib.compress(b"".join(bytes(p) for p in parts))
        if response_compression_algorithm == "gzip":
            headers["Accept-Encoding"] = "gzip"
        elif response_compression_algorithm == "deflate":
            headers["Accept-Encoding"] = "deflate"
        if json_size is not None:
            headers["Inference-Header-Content-Length"] = json_size
        uri = self._model_uri(model_name, model_version, "/infer")
        r = await self._post(uri, body, headers, query_params)
        _raise_if_error(r)
        header_length = r.headers.get("Inference-Header-Content-Length")
        return InferResult.from_response_body(r.read(), self._verbose,
                                              int(header_length) if header_length is not None else None,
                                              r.headers.get("Content-Encoding"))
