"""Synchronous KServe-v2 REST client.

Public API parity with reference ``tritonclient/http/_client.py:102-1659``
(control plane, ``infer``/``async_infer``, ``generate_request_body`` /
``parse_response_body``, plugins, gzip/deflate).  Transport differences:

* no gevent: a pooled keep-alive socket transport with ``writev`` bodies
  (``_transport.py``) and a thread pool of ``max_greenlets or concurrency``
  workers behind ``async_infer``;
* no per-call ``gevent.sleep(0.01)`` (reference ``_client.py:1651``), which
  capped the reference's Python async rate at ~100 req/s per caller thread.
"""

import base64
import gzip
import json
import zlib
from concurrent.futures import ThreadPoolExecutor
from concurrent.futures import TimeoutError as _FutTimeout
from urllib.parse import quote

from tritonclient.utils import raise_error

from .._client import InferenceServerClientBase
from .._request import Request
from ._infer_result import InferResult
from ._transport import ConnectionPool, HttpError, make_ssl_context
from ._utils import (
    _dumps,
    _get_inference_request,
    _get_inference_request_parts,
    _get_query_string,
    _raise_if_error,
)


class InferAsyncRequest:
    """Handle to an in-flight :meth:`InferenceServerClient.async_infer`."""

    def __init__(self, future, verbose=False):
        self._future = future
        self._verbose = verbose

    def get_result(self, block=True, timeout=None):
        """Wait for (or poll, ``block=False``) the result; returns InferResult."""
        try:
            if not block:
                if not self._future.done():
                    raise _FutTimeout()
                response = self._future.result()
            else:
                response = self._future.result(timeout=timeout)
        except _FutTimeout:
            raise_error("failed to obtain inference response")
        _raise_if_error(response)
        return InferResult(response, self._verbose)


def _split_url(url, ssl):
    if url.startswith("http://") or url.startswith("https://"):
        raise_error("url should not include the scheme")
    hostport, _, path = url.partition("/")
    host, sep, port = hostport.rpartition(":")
    if not sep or not port.isdigit():
        host, port = hostport, ("443" if ssl else "80")
    if host.startswith("[") and host.endswith("]"):
        host = host[1:-1]
    base = ("/" + path).rstrip("/") if path else ""
    return host, int(port), base


class InferenceServerClient(InferenceServerClientBase):
    """REST client for a KServe-v2 / Triton server.

    Parameters
    ----------
    url : str
        ``host:port[/base]`` (no scheme).
    verbose : bool
        Print requests and responses.
    concurrency : int
        Number of pooled connections (max concurrent requests).
    connection_timeout, network_timeout : float
        Seconds.
    max_greenlets : int
        Worker count for ``async_infer`` (defaults to ``concurrency``).
    ssl, ssl_options, ssl_context_factory, insecure
        TLS configuration (``ssl_options`` accepts ``ca_certs``, ``certfile``,
        ``keyfile``, ``cert_reqs``).
    """

    def __init__(
        self,
        url,
        verbose=False,
        concurrency=1,
        connection_timeout=60.0,
        network_timeout=60.0,
        max_greenlets=None,
        ssl=False,
        ssl_options=None,
        ssl_context_factory=None,
        insecure=False,
    ):
        super().__init__()
        host, port, base = _split_url(url, ssl)
        self._base_uri = base
        ctx = make_ssl_context(ssl_options, ssl_context_factory, insecure) if ssl else None
        self._pool = ConnectionPool(
            host,
            port,
            concurrency=concurrency,
            connection_timeout=connection_timeout,
            network_timeout=network_timeout,
            ssl_context=ctx,
        )
        self._executor = ThreadPoolExecutor(
            max_workers=max_greenlets or max(1, concurrency), thread_name_prefix="tc-http"
        )
        self._verbose = verbose
        self._closed = False

    def __enter__(self):
        return self

    def __exit__(self, type, value, traceback):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def close(self):
        """Close the client; later calls fail."""
        if not getattr(self, "_closed", True):
            self._executor.shutdown(wait=True)
            self._pool.close()
            self._closed = True

    # -- transport ------------------------------------------------------------
    def _uri(self, request_uri, query_params):
        uri = self._base_uri + "/" + request_uri
        if query_params is not None:
            uri = uri + "?" + _get_query_string(query_params)
        return uri

    def _prepare_headers(self, headers):
        request = Request(dict(headers) if headers else {})
        self._call_plugin(request)
        self._validate_headers(request.headers)
        return request.headers

    def _validate_headers(self, headers):
        if headers and any(k.lower() == "transfer-encoding" for k in headers):
            raise_error(
                "Unsupported HTTP header: 'Transfer-Encoding' is not "
                "supported in the Python client library. Use raw HTTP "
                "request libraries or the C++ client instead for this "
                "header."
            )

    def _request(self, method, uri, parts, headers):
        try:
            return self._pool.request(method, uri, parts, headers)
        except (HttpError, OSError) as e:
            raise_error("HTTP %s %s failed: %s" % (method, uri, e))

    def _get(self, request_uri, headers, query_params):
        headers = self._prepare_headers(headers)
        uri = self._uri(request_uri, query_params)
        if self._verbose:
            print("GET {}, headers {}".format(uri, headers))
        response = self._request("GET", uri, (), headers)
        if self._verbose:
            print(response)
        return response

    def _post(self, request_uri, request_body, headers, query_params):
        headers = self._prepare_headers(headers)
        uri = self._uri(request_uri, query_params)
        if isinstance(request_body, str):
            parts = [request_body.encode()]
        elif isinstance(request_body, (list, tuple)):
            parts = list(request_body)
        else:
            parts = [request_body]
        if self._verbose:
            print("POST {}, headers {}\n{}".format(uri, headers, request_body))
        response = self._request("POST", uri, parts, headers)
        if self._verbose:
            print(response)
        return response

    def _get_json(self, request_uri, headers, query_params):
        response = self._get(request_uri, headers, query_params)
        _raise_if_error(response)
        content = response.read()
        if self._verbose:
            print(content)
        return json.loads(content)

    def _post_json(self, request_uri, body, headers, query_params):
        response = self._post(request_uri, body, headers, query_params)
        _raise_if_error(response)
        content = response.read()
        if self._verbose:
            print(content)
        return json.loads(content)

    @staticmethod
    def _model_uri(model_name, model_version, suffix=""):
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        if model_version != "":
            uri = "v2/models/{}/versions/{}".format(quote(model_name), model_version)
        else:
            uri = "v2/models/{}".format(quote(model_name))
        return uri + suffix

    # -- health / metadata ------------------------------------------------------
    def is_server_live(self, headers=None, query_params=None):
        """True if the server is live."""
        return self._get("v2/health/live", headers, query_params).status_code == 200

    def is_server_ready(self, headers=None, query_params=None):
        """True if the server is ready (uses /v2/health/ready; the reference
        C++ client wrongly hits /live, http_client.cc:1416)."""
        return self._get("v2/health/ready", headers, query_params).status_code == 200

    def is_model_ready(self, model_name, model_version="", headers=None, query_params=None):
        """True if ``model_name`` (optionally ``model_version``) is ready."""
        uri = self._model_uri(model_name, model_version, "/ready")
        return self._get(uri, headers, query_params).status_code == 200

    def get_server_metadata(self, headers=None, query_params=None):
        """Server metadata JSON dict."""
        return self._get_json("v2", headers, query_params)

    def get_model_metadata(self, model_name, model_version="", headers=None, query_params=None):
        """Model metadata JSON dict."""
        return self._get_json(self._model_uri(model_name, model_version), headers, query_params)

    def get_model_config(self, model_name, model_version="", headers=None, query_params=None):
        """Model configuration JSON dict."""
        return self._get_json(
            self._model_uri(model_name, model_version, "/config"), headers, query_params
        )

    # -- repository ---------------------------------------------------------------
    def get_model_repository_index(self, headers=None, query_params=None):
        """Repository index (list of model dicts)."""
        return self._post_json("v2/repository/index", "", headers, query_params)

    def load_model(self, model_name, headers=None, query_params=None, config=None, files=None):
        """Load / reload a model, optionally overriding config and files."""
        uri = "v2/repository/models/{}/load".format(quote(model_name))
        load_request = {}
        if config is not None:
            load_request.setdefault("parameters", {})["config"] = config
        if files is not None:
            for path, content in files.items():
                load_request.setdefault("parameters", {})[path] = base64.b64encode(content).decode(
                    "ascii"
                )
        response = self._post(uri, _dumps(load_request), headers, query_params)
        _raise_if_error(response)
        if self._verbose:
            print("Loaded model '{}'".format(model_name))

    def unload_model(self, model_name, headers=None, query_params=None, unload_dependents=False):
        """Unload a model (and its dependents if requested)."""
        uri = "v2/repository/models/{}/unload".format(quote(model_name))
        body = _dumps({"parameters": {"unload_dependents": unload_dependents}})
        response = self._post(uri, body, headers, query_params)
        _raise_if_error(response)
        if self._verbose:
            print("Unloaded model '{}'".format(model_name))

    # -- statistics / trace / log -------------------------------------------------
    def get_inference_statistics(
        self, model_name="", model_version="", headers=None, query_params=None
    ):
        """Inference statistics JSON dict (all models when ``model_name`` is empty)."""
        if model_name != "":
            uri = self._model_uri(model_name, model_version, "/stats")
        else:
            uri = "v2/models/stats"
        return self._get_json(uri, headers, query_params)

    def update_trace_settings(self, model_name=None, settings={}, headers=None, query_params=None):
        """Update trace settings (global when ``model_name`` is empty)."""
        if model_name:
            uri = "v2/models/{}/trace/setting".format(quote(model_name))
        else:
            uri = "v2/trace/setting"
        return self._post_json(uri, _dumps(settings), headers, query_params)

    def get_trace_settings(self, model_name=None, headers=None, query_params=None):
        """Current trace settings."""
        if model_name:
            uri = "v2/models/{}/trace/setting".format(quote(model_name))
        else:
            uri = "v2/trace/setting"
        return self._get_json(uri, headers, query_params)

    def update_log_settings(self, settings, headers=None, query_params=None):
        """Update global log settings."""
        return self._post_json("v2/logging", _dumps(settings), headers, query_params)

    def get_log_settings(self, headers=None, query_params=None):
        """Current global log settings."""
        return self._get_json("v2/logging", headers, query_params)

    # -- system shared memory -----------------------------------------------------
    def get_system_shared_memory_status(self, region_name="", headers=None, query_params=None):
        """Status of one / all registered system shm regions."""
        if region_name != "":
            uri = "v2/systemsharedmemory/region/{}/status".format(quote(region_name))
        else:
            uri = "v2/systemsharedmemory/status"
        return self._get_json(uri, headers, query_params)

    def register_system_shared_memory(
        self, name, key, byte_size, offset=0, headers=None, query_params=None
    ):
        """Register POSIX region ``key`` as ``name``."""
        uri = "v2/systemsharedmemory/region/{}/register".format(quote(name))
        body = _dumps({"key": key, "offset": offset, "byte_size": byte_size})
        response = self._post(uri, body, headers, query_params)
        _raise_if_error(response)
        if self._verbose:
            print("Registered system shared memory with name '{}'".format(name))

    def unregister_system_shared_memory(self, name="", headers=None, query_params=None):
        """Unregister one (or every) system shm region."""
        if name != "":
            uri = "v2/systemsharedmemory/region/{}/unregister".format(quote(name))
        else:
            uri = "v2/systemsharedmemory/unregister"
        response = self._post(uri, "", headers, query_params)
        _raise_if_error(response)
        if self._verbose:
            if name != "":
                print("Unregistered system shared memory with name '{}'".format(name))
            else:
                print("Unregistered all system shared memory regions")

    # -- device (HIP) shared memory; wire name kept as "cuda" ---------------------
    def get_cuda_shared_memory_status(self, region_name="", headers=None, query_params=None):
        """Status of one / all registered device (HIP IPC) regions."""
        if region_name != "":
            uri = "v2/cudasharedmemory/region/{}/status".format(quote(region_name))
        else:
            uri = "v2/cudasharedmemory/status"
        return self._get_json(uri, headers, query_params)

    def register_cuda_shared_memory(
        self, name, raw_handle, device_id, byte_size, headers=None, query_params=None
    ):
        """Register a device region; ``raw_handle`` is the b64 IPC handle
        (``hip_shared_memory.get_raw_handle``)."""
        uri = "v2/cudasharedmemory/region/{}/register".format(quote(name))
        if isinstance(raw_handle, bytes):
            raw_handle = raw_handle.decode("ascii")
        body = _dumps(
            {"raw_handle": {"b64": raw_handle}, "device_id": device_id, "byte_size": byte_size}
        )
        response = self._post(uri, body, headers, query_params)
        _raise_if_error(response)
        if self._verbose:
            print("Registered cuda shared memory with name '{}'".format(name))

    def unregister_cuda_shared_memory(self, name="", headers=None, query_params=None):
        """Unregister one (or every) device region."""
        if name != "":
            uri = "v2/cudasharedmemory/region/{}/unregister".format(quote(name))
        else:
            uri = "v2/cudasharedmemory/unregister"
        response = self._post(uri, "", headers, query_params)
        _raise_if_error(response)
        if self._verbose:
            if name != "":
                print("Unregistered cuda shared memory with name '{}'".format(name))
            else:
                print("Unregistered all cuda shared memory regions")

    # HIP-named aliases (same wire routes)
    get_hip_shared_memory_status = get_cuda_shared_memory_status
    register_hip_shared_memory = register_cuda_shared_memory
    unregister_hip_shared_memory = unregister_cuda_shared_memory

    # -- inference ----------------------------------------------------------------
    @staticmethod
    def generate_request_body(
        inputs,
        outputs=None,
        request_id="",
        sequence_id=0,
        sequence_start=False,
        sequence_end=False,
        priority=0,
        timeout=None,
        parameters=None,
    ):
        """Return ``(body_bytes, json_size or None)`` for an infer request."""
        return _get_inference_request(
            inputs=inputs,
            request_id=request_id,
            outputs=outputs,
            sequence_id=sequence_id,
            sequence_start=sequence_start,
            sequence_end=sequence_end,
            priority=priority,
            timeout=timeout,
            custom_parameters=parameters,
        )

    @staticmethod
    def parse_response_body(response_body, verbose=False, header_length=None, content_encoding=None):
        """Build an :class:`InferResult` from a raw response body."""
        return InferResult.from_response_body(response_body, verbose, header_length, content_encoding)

    def _prepare_infer(
        self,
        model_name,
        inputs,
        model_version,
        outputs,
        request_id,
        sequence_id,
        sequence_start,
        sequence_end,
        priority,
        timeout,
        headers,
        request_compression_algorithm,
        response_compression_algorithm,
        parameters,
    ):
        parts, json_size = _get_inference_request_parts(
            inputs,
            request_id=request_id,
            outputs=outputs,
            sequence_id=sequence_id,
            sequence_start=sequence_start,
            sequence_end=sequence_end,
            priority=priority,
            timeout=timeout,
            custom_parameters=parameters,
        )
        headers = dict(headers) if headers else {}
        if request_compression_algorithm in ("gzip", "deflate"):
            joined = b"".join(bytes(p) for p in parts)
            if request_compression_algorithm == "gzip":
                headers["Content-Encoding"] = "gzip"
                parts = [gzip.compress(joined)]
            else:
                headers["Content-Encoding"] = "deflate"
                parts = [zlib.compress(joined)]
        if response_compression_algorithm == "gzip":
            headers["Accept-Encoding"] = "gzip"
        elif response_compression_algorithm == "deflate":
            headers["Accept-Encoding"] = "deflate"
        if json_size is not None:
            headers["Inference-Header-Content-Length"] = json_size
        uri = self._model_uri(model_name, model_version, "/infer")
        return uri, parts, headers

    def infer(
        self,
        model_name,
        inputs,
        model_version="",
        outputs=None,
        request_id="",
        sequence_id=0,
        sequence_start=False,
        sequence_end=False,
        priority=0,
        timeout=None,
        headers=None,
        query_params=None,
        request_compression_algorithm=None,
        response_compression_algorithm=None,
        parameters=None,
    ):
        """Synchronous inference; returns :class:`InferResult`."""
        uri, parts, headers = self._prepare_infer(
            model_name,
            inputs,
            model_version,
            outputs,
            request_id,
            sequence_id,
            sequence_start,
            sequence_end,
            priority,
            timeout,
            headers,
            request_compression_algorithm,
            response_compression_algorithm,
            parameters,
        )
        response = self._post(uri, parts, headers, query_params)
        _raise_if_error(response)
        return InferResult(response, self._verbose)

    def async_infer(
        self,
        model_name,
        inputs,
        model_version="",
        outputs=None,
        request_id="",
        sequence_id=0,
        sequence_start=False,
        sequence_end=False,
        priority=0,
        timeout=None,
        headers=None,
        query_params=None,
        request_compression_algorithm=None,
        response_compression_algorithm=None,
        parameters=None,
    ):
        """Asynchronous inference; returns :class:`InferAsyncRequest`.

        The request body is built on the caller's thread (so inputs may be
        reused immediately after the call returns), then sent by a pool worker.
        """
        uri, parts, headers = self._prepare_infer(
            model_name,
            inputs,
            model_version,
            outputs,
            request_id,
            sequence_id,
            sequence_start,
            sequence_end,
            priority,
            timeout,
            headers,
            request_compression_algorithm,
            response_compression_algorithm,
            parameters,
        )
        headers = self._prepare_headers(headers)
        full_uri = self._uri(uri, query_params)
        if self._verbose:
            print("POST {}, headers {}".format(full_uri, headers))

        def _run():
            return self._request("POST", full_uri, parts, headers)

        return InferAsyncRequest(self._executor.submit(_run), self._verbose)
