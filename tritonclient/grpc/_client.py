"""Synchronous gRPC client for ``inference.GRPCInferenceService``.

Public API parity with reference ``tritonclient/grpc/_client.py:53-1936``:
control plane (``as_json`` via ``MessageToJson(preserving_proto_field_name)``),
``infer``, ``async_infer`` (cancellable :class:`CallContext`), one bidi stream
per client (``start_stream`` / ``async_stream_infer`` / ``stop_stream``).
"""

import base64
import json
import struct

import grpc
from google.protobuf.json_format import MessageToJson

from tritonclient.grpc import service_pb2, service_pb2_grpc
from tritonclient.utils import raise_error

from .._client import InferenceServerClientBase
from .._request import Request
from ._infer_result import InferResult
from ._infer_stream import StreamSession
from ._utils import (
    _get_inference_request,
    _grpc_compression_type,
    get_cancelled_error,
    get_error_grpc,
    raise_error_grpc,
)

INT32_MAX = 2 ** (struct.Struct("i").size * 8 - 1) - 1
MAX_GRPC_MESSAGE_SIZE = INT32_MAX


class KeepAliveOptions:
    """gRPC keepalive settings (reference _client.py:57-98)."""

    def __init__(
        self,
        keepalive_time_ms=INT32_MAX,
        keepalive_timeout_ms=20000,
        keepalive_permit_without_calls=False,
        http2_max_pings_without_data=2,
    ):
        self.keepalive_time_ms = keepalive_time_ms
        self.keepalive_timeout_ms = keepalive_timeout_ms
        self.keepalive_permit_without_calls = keepalive_permit_without_calls
        self.http2_max_pings_without_data = http2_max_pings_without_data


class CallContext:
    """Handle for cancelling an in-flight :meth:`async_infer`."""

    def __init__(self, grpc_future):
        self.__grpc_future = grpc_future

    def cancel(self):
        """Cancel the RPC (the callback then receives a CANCELLED error)."""
        self.__grpc_future.cancel()


def _default_channel_options(keepalive_options):
    ko = keepalive_options or KeepAliveOptions()
    return [
        ("grpc.max_send_message_length", MAX_GRPC_MESSAGE_SIZE),
        ("grpc.max_receive_message_length", MAX_GRPC_MESSAGE_SIZE),
        ("grpc.keepalive_time_ms", ko.keepalive_time_ms),
        ("grpc.keepalive_timeout_ms", ko.keepalive_timeout_ms),
        ("grpc.keepalive_permit_without_calls", ko.keepalive_permit_without_calls),
        ("grpc.http2.max_pings_without_data", ko.http2_max_pings_without_data),
    ]


def _read(path):
    if path is None:
        return None
    with open(path, "rb") as f:
        return f.read()


def _to_json(msg):
    return json.loads(MessageToJson(msg, preserving_proto_field_name=True))


# -- request builders shared with tritonclient.grpc.aio ------------------------------
def _load_request(model_name, config=None, files=None):
    req = service_pb2.RepositoryModelLoadRequest(model_name=model_name)
    if config is not None:
        req.parameters["config"].string_param = config
    if files is not None:
        for path, content in files.items():
            req.parameters[path].bytes_param = content
    return req


def _unload_request(model_name, unload_dependents=False):
    req = service_pb2.RepositoryModelUnloadRequest(model_name=model_name)
    req.parameters["unload_dependents"].bool_param = unload_dependents
    return req


def _trace_request(model_name=None, settings=None):
    req = service_pb2.TraceSettingRequest()
    if model_name:
        req.model_name = model_name
    for key, value in (settings or {}).items():
        if value is None:
            req.settings[key]  # present-but-empty => clear
        elif isinstance(value, (list, tuple)):
            req.settings[key].value.extend([str(v) for v in value])
        else:
            req.settings[key].value.append(str(value))
    return req


def _log_request(settings=None):
    req = service_pb2.LogSettingsRequest()
    for key, value in (settings or {}).items():
        if value is None:
            req.settings[key]
        elif key in ("log_file", "log_format"):
            req.settings[key].string_param = value
        elif key == "log_verbose_level":
            req.settings[key].uint32_param = value
        else:
            req.settings[key].bool_param = value
    return req


class InferenceServerClient(InferenceServerClientBase):
    """gRPC client for a KServe-v2 / Triton server (``host:port``)."""

    def __init__(
        self,
        url,
        verbose=False,
        ssl=False,
        root_certificates=None,
        private_key=None,
        certificate_chain=None,
        creds=None,
        keepalive_options=None,
        channel_args=None,
    ):
        super().__init__()
        # an empty list means "no channel arguments at all"
        channel_opt = channel_args if channel_args is not None else _default_channel_options(
            keepalive_options
        )
        if creds:
            self._channel = grpc.secure_channel(url, creds, options=channel_opt)
        elif ssl:
            creds = grpc.ssl_channel_credentials(
                root_certificates=_read(root_certificates),
                private_key=_read(private_key),
                certificate_chain=_read(certificate_chain),
            )
            self._channel = grpc.secure_channel(url, creds, options=channel_opt)
        else:
            self._channel = grpc.insecure_channel(url, options=channel_opt)
        self._client_stub = service_pb2_grpc.GRPCInferenceServiceStub(self._channel)
        self._verbose = verbose
        self._stream = None

    def _get_metadata(self, headers):
        request = Request(dict(headers) if headers else {})
        self._call_plugin(request)
        return tuple((k.lower(), v) for k, v in request.headers.items())

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
        """Stop any active stream and close the channel."""
        self.stop_stream()
        if getattr(self, "_channel", None) is not None:
            self._channel.close()
            self._channel = None

    # -- helper -------------------------------------------------------------
    def _unary(self, name, request, headers, client_timeout, as_json=False, verbose_tag=None):
        metadata = self._get_metadata(headers)
        if self._verbose:
            print("{}, metadata {}\n{}".format(verbose_tag or name, metadata, request))
        try:
            response = getattr(self._client_stub, name)(
                request=request, metadata=metadata, timeout=client_timeout
            )
        except grpc.RpcError as rpc_error:
            raise_error_grpc(rpc_error)
        if self._verbose:
            print(response)
        return _to_json(response) if as_json else response

    # -- health / metadata ----------------------------------------------------
    def is_server_live(self, headers=None, client_timeout=None):
        """True if the server is live."""
        return self._unary(
            "ServerLive", service_pb2.ServerLiveRequest(), headers, client_timeout
        ).live

    def is_server_ready(self, headers=None, client_timeout=None):
        """True if the server is ready."""
        return self._unary(
            "ServerReady", service_pb2.ServerReadyRequest(), headers, client_timeout
        ).ready

    def is_model_ready(self, model_name, model_version="", headers=None, client_timeout=None):
        """True if the model (version) is ready."""
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        req = service_pb2.ModelReadyRequest(name=model_name, version=model_version)
        return self._unary("ModelReady", req, headers, client_timeout).ready

    def get_server_metadata(self, headers=None, as_json=False, client_timeout=None):
        """ServerMetadataResponse (or dict)."""
        return self._unary(
            "ServerMetadata", service_pb2.ServerMetadataRequest(), headers, client_timeout, as_json
        )

    def get_model_metadata(
        self, model_name, model_version="", headers=None, as_json=False, client_timeout=None
    ):
        """ModelMetadataResponse (or dict)."""
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        req = service_pb2.ModelMetadataRequest(name=model_name, version=model_version)
        return self._unary("ModelMetadata", req, headers, client_timeout, as_json)

    def get_model_config(
        self, model_name, model_version="", headers=None, as_json=False, client_timeout=None
    ):
        """ModelConfigResponse (or dict)."""
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        req = service_pb2.ModelConfigRequest(name=model_name, version=model_version)
        return self._unary("ModelConfig", req, headers, client_timeout, as_json)

    # -- repository -------------------------------------------------------------
    def get_model_repository_index(self, headers=None, as_json=False, client_timeout=None):
        """RepositoryIndexResponse (or dict)."""
        return self._unary(
            "RepositoryIndex", service_pb2.RepositoryIndexRequest(), headers, client_timeout, as_json
        )

    def load_model(self, model_name, headers=None, config=None, files=None, client_timeout=None):
        """Load / reload a model with optional config + file overrides."""
        req = service_pb2.RepositoryModelLoadRequest(model_name=model_name)
        if config is not None:
            req.parameters["config"].string_param = config
        if self._verbose:
            # the (potentially large) file contents are not printed
            print("load_model, metadata {}\noverride files omitted:\n{}".format(
                self._get_metadata(headers), req))
        if files is not None:
            for path, content in files.items():
                req.parameters[path].bytes_param = content
        metadata = self._get_metadata(headers)
        try:
            self._client_stub.RepositoryModelLoad(
                request=req, metadata=metadata, timeout=client_timeout
            )
        except grpc.RpcError as rpc_error:
            raise_error_grpc(rpc_error)
        if self._verbose:
            print("Loaded model '{}'".format(model_name))

    def unload_model(self, model_name, headers=None, unload_dependents=False, client_timeout=None):
        """Unload a model (and optionally its dependents)."""
        self._unary("RepositoryModelUnload", _unload_request(model_name, unload_dependents), headers,
                    client_timeout, verbose_tag="unload_model")
        if self._verbose:
            print("Unloaded model '{}'".format(model_name))

    # -- statistics / trace / log ------------------------------------------------
    def get_inference_statistics(
        self, model_name="", model_version="", headers=None, as_json=False, client_timeout=None
    ):
        """ModelStatisticsResponse (or dict)."""
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        req = service_pb2.ModelStatisticsRequest(name=model_name, version=model_version)
        return self._unary("ModelStatistics", req, headers, client_timeout, as_json)

    def update_trace_settings(
        self, model_name=None, settings={}, headers=None, as_json=False, client_timeout=None
    ):
        """Update trace settings; a None value clears the setting."""
        return self._unary("TraceSetting", _trace_request(model_name, settings), headers, client_timeout, as_json)

    def get_trace_settings(self, model_name=None, headers=None, as_json=False, client_timeout=None):
        """Current trace settings."""
        req = service_pb2.TraceSettingRequest()
        if model_name:
            req.model_name = model_name
        return self._unary("TraceSetting", req, headers, client_timeout, as_json)

    def update_log_settings(self, settings, headers=None, as_json=False, client_timeout=None):
        """Update global log settings (typed per key as in the reference)."""
        return self._unary("LogSettings", _log_request(settings), headers, client_timeout, as_json)

    def get_log_settings(self, headers=None, as_json=False, client_timeout=None):
        """Current global log settings."""
        return self._unary(
            "LogSettings", service_pb2.LogSettingsRequest(), headers, client_timeout, as_json
        )

    # -- system shared memory ---------------------------------------------------
    def get_system_shared_memory_status(
        self, region_name="", headers=None, as_json=False, client_timeout=None
    ):
        """SystemSharedMemoryStatusResponse (or dict)."""
        req = service_pb2.SystemSharedMemoryStatusRequest(name=region_name)
        return self._unary("SystemSharedMemoryStatus", req, headers, client_timeout, as_json)

    def register_system_shared_memory(
        self, name, key, byte_size, offset=0, headers=None, client_timeout=None
    ):
        """Register POSIX region ``key`` as ``name``."""
        req = service_pb2.SystemSharedMemoryRegisterRequest(
            name=name, key=key, offset=offset, byte_size=byte_size
        )
        self._unary("SystemSharedMemoryRegister", req, headers, client_timeout)
        if self._verbose:
            print("Registered system shared memory with name '{}'".format(name))

    def unregister_system_shared_memory(self, name="", headers=None, client_timeout=None):
        """Unregister one (or every) system region."""
        req = service_pb2.SystemSharedMemoryUnregisterRequest(name=name)
        self._unary("SystemSharedMemoryUnregister", req, headers, client_timeout)
        if self._verbose:
            if name != "":
                print("Unregistered system shared memory with name '{}'".format(name))
            else:
                print("Unregistered all system shared memory regions")

    # -- device (HIP IPC) shared memory — wire name "Cuda" ------------------------
    def get_cuda_shared_memory_status(
        self, region_name="", headers=None, as_json=False, client_timeout=None
    ):
        """CudaSharedMemoryStatusResponse (or dict)."""
        req = service_pb2.CudaSharedMemoryStatusRequest(name=region_name)
        return self._unary("CudaSharedMemoryStatus", req, headers, client_timeout, as_json)

    def register_cuda_shared_memory(
        self, name, raw_handle, device_id, byte_size, headers=None, client_timeout=None
    ):
        """Register a device region; ``raw_handle`` is base64 (as returned by
        ``hip_shared_memory.get_raw_handle``) and is sent as raw 64 bytes."""
        req = service_pb2.CudaSharedMemoryRegisterRequest(
            name=name,
            raw_handle=base64.b64decode(raw_handle),
            device_id=device_id,
            byte_size=byte_size,
        )
        self._unary("CudaSharedMemoryRegister", req, headers, client_timeout)
        if self._verbose:
            print("Registered cuda shared memory with name '{}'".format(name))

    def unregister_cuda_shared_memory(self, name="", headers=None, client_timeout=None):
        """Unregister one (or every) device region."""
        req = service_pb2.CudaSharedMemoryUnregisterRequest(name=name)
        self._unary("CudaSharedMemoryUnregister", req, headers, client_timeout)
        if self._verbose:
            if name != "":
                print("Unregistered cuda shared memory with name '{}'".format(name))
            else:
                print("Unregistered all cuda shared memory regions")

    get_hip_shared_memory_status = get_cuda_shared_memory_status
    register_hip_shared_memory = register_cuda_shared_memory
    unregister_hip_shared_memory = unregister_cuda_shared_memory

    # -- inference --------------------------------------------------------------
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
        client_timeout=None,
        headers=None,
        compression_algorithm=None,
        parameters=None,
    ):
        """Synchronous inference; returns :class:`InferResult`."""
        metadata = self._get_metadata(headers)
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        request = _get_inference_request(
            model_name=model_name,
            inputs=inputs,
            model_version=model_version,
            request_id=request_id,
            outputs=outputs,
            sequence_id=sequence_id,
            sequence_start=sequence_start,
            sequence_end=sequence_end,
            priority=priority,
            timeout=timeout,
            parameters=parameters,
        )
        if self._verbose:
            print("infer, metadata {}\n{}".format(metadata, request))
        try:
            response = self._client_stub.ModelInfer(
                request=request,
                metadata=metadata,
                timeout=client_timeout,
                compression=_grpc_compression_type(compression_algorithm),
            )
        except grpc.RpcError as rpc_error:
            raise_error_grpc(rpc_error)
        if self._verbose:
            print(response)
        return InferResult(response)

    def async_infer(
        self,
        model_name,
        inputs,
        callback,
        model_version="",
        outputs=None,
        request_id="",
        sequence_id=0,
        sequence_start=False,
        sequence_end=False,
        priority=0,
        timeout=None,
        client_timeout=None,
        headers=None,
        compression_algorithm=None,
        parameters=None,
    ):
        """Asynchronous inference; ``callback(result=..., error=...)`` runs on a
        grpc thread. Returns a :class:`CallContext`."""

        def wrapped_callback(call_future):
            result = error = None
            try:
                response = call_future.result()
                if self._verbose:
                    print(response)
                result = InferResult(response)
            except grpc.RpcError as rpc_error:
                error = get_error_grpc(rpc_error)
            except grpc.FutureCancelledError:
                error = get_cancelled_error()
            callback(result=result, error=error)

        metadata = self._get_metadata(headers)
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        request = _get_inference_request(
            model_name=model_name,
            inputs=inputs,
            model_version=model_version,
            request_id=request_id,
            outputs=outputs,
            sequence_id=sequence_id,
            sequence_start=sequence_start,
            sequence_end=sequence_end,
            priority=priority,
            timeout=timeout,
            parameters=parameters,
        )
        if self._verbose:
            print("async_infer, metadata {}\n{}".format(metadata, request))
        try:
            fut = self._client_stub.ModelInfer.future(
                request=request,
                metadata=metadata,
                timeout=client_timeout,
                compression=_grpc_compression_type(compression_algorithm),
            )
        except grpc.RpcError as rpc_error:
            raise_error_grpc(rpc_error)
        if self._verbose:
            msg = "Sent request"
            if request_id != "":
                msg += " '{}'".format(request_id)
            print(msg)
        fut.add_done_callback(wrapped_callback)
        return CallContext(fut)

    # -- streaming --------------------------------------------------------------
    def start_stream(self, callback, stream_timeout=None, headers=None, compression_algorithm=None):
        """Open the (single) bidi stream; responses go to ``callback``."""
        if self._stream is not None:
            raise_error(
                "cannot start another stream with one already running. "
                "'InferenceServerClient' supports only a single active "
                "stream at a given time."
            )
        metadata = self._get_metadata(headers)
        if self._verbose:
            print("start_stream, metadata {}".format(metadata))
        self._stream = StreamSession(callback, self._verbose)
        try:
            response_iterator = self._client_stub.ModelStreamInfer(
                self._stream.outgoing(),
                metadata=metadata,
                timeout=stream_timeout,
                compression=_grpc_compression_type(compression_algorithm),
            )
            self._stream.attach(response_iterator)
        except grpc.RpcError as rpc_error:
            raise_error_grpc(rpc_error)

    def stop_stream(self, cancel_requests=False):
        """Close the stream (blocks for pending responses unless cancelling)."""
        if getattr(self, "_stream", None) is not None:
            self._stream.close(cancel_requests)
        self._stream = None

    def async_stream_infer(
        self,
        model_name,
        inputs,
        model_version="",
        outputs=None,
        request_id="",
        sequence_id=0,
        sequence_start=False,
        sequence_end=False,
        enable_empty_final_response=False,
        priority=0,
        timeout=None,
        parameters=None,
    ):
        """Enqueue one request on the active stream."""
        if self._stream is None:
            raise_error("stream not available, use start_stream() to make one available.")
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        request = _get_inference_request(
            model_name=model_name,
            inputs=inputs,
            model_version=model_version,
            request_id=request_id,
            outputs=outputs,
            sequence_id=sequence_id,
            sequence_start=sequence_start,
            sequence_end=sequence_end,
            priority=priority,
            timeout=timeout,
            parameters=parameters,
        )
        if enable_empty_final_response:
            request.parameters["triton_enable_empty_final_response"].bool_param = True
        if self._verbose:
            print("async_stream_infer\n{}".format(request))
        self._stream.submit(request)
        if self._verbose:
            print("enqueued request {} to stream...".format(request_id))
