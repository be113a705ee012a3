"""asyncio KServe-v2 gRPC client on grpc.aio.

API parity with reference ``tritonclient/grpc/aio/__init__.py:50-810``: the
control plane and ``infer`` as coroutines, and ``stream_infer(inputs_iterator)``
which consumes an async iterator of ``async_stream_infer`` keyword dicts and
returns an async iterator of ``(InferResult, InferenceServerException)`` with
``cancel()``.  Request messages are built by the same helpers as the sync
client (``tritonclient/grpc/_utils.py``, ``_client.py``).
"""

import base64
import json

import grpc
from google.protobuf.json_format import MessageToJson

from tritonclient.utils import raise_error

from ..._client import InferenceServerClientBase
from ..._request import Request
from .. import service_pb2, service_pb2_grpc
from .._client import (
    MAX_GRPC_MESSAGE_SIZE,  # noqa: F401
    KeepAliveOptions,
    _default_channel_options,
    _load_request,
    _log_request,
    _read,
    _trace_request,
    _unload_request,
)
from .._infer_input import InferInput
from .._infer_result import InferResult
from .._requested_output import InferRequestedOutput
from .._utils import _get_inference_request, _grpc_compression_type, get_error_grpc, raise_error_grpc
from ...utils import InferenceServerException  # noqa: F401

__all__ = ["InferenceServerClient", "InferInput", "InferRequestedOutput", "InferResult", "KeepAliveOptions",
           "InferenceServerException"]


def _to_json(msg):
    return json.loads(MessageToJson(msg, preserving_proto_field_name=True))


class InferenceServerClient(InferenceServerClientBase):
    """asyncio gRPC client; one instance per event loop."""

    def __init__(self, url, verbose=False, ssl=False, root_certificates=None, private_key=None,
                 certificate_chain=None, creds=None, keepalive_options=None, channel_args=None):
        super().__init__()
        channel_opt = channel_args if channel_args is not None else _default_channel_options(keepalive_options)
        if creds:
            self._channel = grpc.aio.secure_channel(url, creds, options=channel_opt)
        elif ssl:
            creds = grpc.ssl_channel_credentials(root_certificates=_read(root_certificates),
                                                 private_key=_read(private_key),
                                                 certificate_chain=_read(certificate_chain))
            self._channel = grpc.aio.secure_channel(url, creds, options=channel_opt)
        else:
            self._channel = grpc.aio.insecure_channel(url, options=channel_opt)
        self._client_stub = service_pb2_grpc.GRPCInferenceServiceStub(self._channel)
        self._verbose = verbose

    async def __aenter__(self):
        return self

    async def __aexit__(self, type, value, traceback):
        await self.close()

    async def close(self):
        """Close the channel."""
        await self._channel.close()

    def _get_metadata(self, headers):
        request = Request(dict(headers) if headers else {})
        self._call_plugin(request)
        return tuple((k.lower(), v) for k, v in request.headers.items())

    def _return_response(self, response, as_json):
        return _to_json(response) if as_json else response

    async def _unary(self, name, request, headers, client_timeout, as_json=False):
        metadata = self._get_metadata(headers)
        if self._verbose:
            print("{}, metadata {}\n{}".format(name, metadata, request))
        try:
            response = await getattr(self._client_stub, name)(request=request, metadata=metadata,
                                                               timeout=client_timeout)
        except grpc.RpcError as rpc_error:
            raise_error_grpc(rpc_error)
        if self._verbose:
            print(response)
        return self._return_response(response, as_json)

    # -- health / metadata ---------------------------------------------------------
    async def is_server_live(self, headers=None, client_timeout=None):
        return (await self._unary("ServerLive", service_pb2.ServerLiveRequest(), headers, client_timeout)).live

    async def is_server_ready(self, headers=None, client_timeout=None):
        return (await self._unary("ServerReady", service_pb2.ServerReadyRequest(), headers, client_timeout)).ready

    async def is_model_ready(self, model_name, model_version="", headers=None, client_timeout=None):
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        req = service_pb2.ModelReadyRequest(name=model_name, version=model_version)
        return (await self._unary("ModelReady", req, headers, client_timeout)).ready

    async def get_server_metadata(self, headers=None, as_json=False, client_timeout=None):
        return await self._unary("ServerMetadata", service_pb2.ServerMetadataRequest(), headers, client_timeout,
                                 as_json)

    async def get_model_metadata(self, model_name, model_version="", headers=None, as_json=False,
                                 client_timeout=None):
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        req = service_pb2.ModelMetadataRequest(name=model_name, version=model_version)
        return await self._unary("ModelMetadata", req, headers, client_timeout, as_json)

    async def get_model_config(self, model_name, model_version="", headers=None, as_json=False,
                               client_timeout=None):
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        req = service_pb2.ModelConfigRequest(name=model_name, version=model_version)
        return await self._unary("ModelConfig", req, headers, client_timeout, as_json)

    # -- repository ----------------------------------------------------------------
    async def get_model_repository_index(self, headers=None, as_json=False, client_timeout=None):
        return await self._unary("RepositoryIndex", service_pb2.RepositoryIndexRequest(), headers, client_timeout,
                                 as_json)

    async def load_model(self, model_name, headers=None, config=None, files=None, client_timeout=None):
        await self._unary("RepositoryModelLoad", _load_request(model_name, config, files), headers, client_timeout)
        if self._verbose:
            print("Loaded model '{}'".format(model_name))

    async def unload_model(self, model_name, headers=None, unload_dependents=False, client_timeout=None):
        await self._unary("RepositoryModelUnload", _unload_request(model_name, unload_dependents), headers,
                          client_timeout)
        if self._verbose:
            print("Unloaded model '{}'".format(model_name))

    # -- statistics / trace / log ---------------------------------------------------
    async def get_inference_statistics(self, model_name="", model_version="", headers=None, as_json=False,
                                       client_timeout=None):
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        req = service_pb2.ModelStatisticsRequest(name=model_name, version=model_version)
        return await self._unary("ModelStatistics", req, headers, client_timeout, as_json)

    async def update_trace_settings(self, model_name=None, settings={}, headers=None, as_json=False,
                                    client_timeout=None):
        return await self._unary("TraceSetting", _trace_request(model_name, settings), headers, client_timeout,
                                 as_json)

    async def get_trace_settings(self, model_name=None, headers=None, as_json=False, client_timeout=None):
        return await self._unary("TraceSetting", _trace_request(model_name), headers, client_timeout, as_json)

    async def update_log_settings(self, settings, headers=None, as_json=False, client_timeout=None):
        return await self._unary("LogSettings", _log_request(settings), headers, client_timeout, as_json)

    async def get_log_settings(self, headers=None, as_json=False, client_timeout=None):
        return await self._unary("LogSettings", service_pb2.LogSettingsRequest(), headers, client_timeout, as_json)

    # -- shared memory ----------------------------------------------------------------
    async def get_system_shared_memory_status(self, region_name="", headers=None, as_json=False,
                                              client_timeout=None):
        req = service_pb2.SystemSharedMemoryStatusRequest(name=region_name)
        return await self._unary("SystemSharedMemoryStatus", req, headers, client_timeout, as_json)

    async def register_system_shared_memory(self, name, key, byte_size, offset=0, headers=None,
                                            client_timeout=None):
        req = service_pb2.SystemSharedMemoryRegisterRequest(name=name, key=key, offset=offset, byte_size=byte_size)
        await self._unary("SystemSharedMemoryRegister", req, headers, client_timeout)

    async def unregister_system_shared_memory(self, name="", headers=None, client_timeout=None):
        req = service_pb2.SystemSharedMemoryUnregisterRequest(name=name)
        await self._unary("SystemSharedMemoryUnregister", req, headers, client_timeout)

    async def get_cuda_shared_memory_status(self, region_name="", headers=None, as_json=False,
                                            client_timeout=None):
        req = service_pb2.CudaSharedMemoryStatusRequest(name=region_name)
        return await self._unary("CudaSharedMemoryStatus", req, headers, client_timeout, as_json)

    async def register_cuda_shared_memory(self, name, raw_handle, device_id, byte_size, headers=None,
                                          client_timeout=None):
        req = service_pb2.CudaSharedMemoryRegisterRequest(name=name, raw_handle=base64.b64decode(raw_handle),
                                                          device_id=device_id, byte_size=byte_size)
        await self._unary("CudaSharedMemoryRegister", req, headers, client_timeout)

    async def unregister_cuda_shared_memory(self, name="", headers=None, client_timeout=None):
        req = service_pb2.CudaSharedMemoryUnregisterRequest(name=name)
        await self._unary("CudaSharedMemoryUnregister", req, headers, client_timeout)

    get_hip_shared_memory_status = get_cuda_shared_memory_status
    register_hip_shared_memory = register_cuda_shared_memory
    unregister_hip_shared_memory = unregister_cuda_shared_memory

    # -- inference -----------------------------------------------------------------------
    async def infer(self, model_name, inputs, model_version="", outputs=None, request_id="", sequence_id=0,
                    sequence_start=False, sequence_end=False, priority=0, timeout=None, client_timeout=None,
                    headers=None, compression_algorithm=None, parameters=None):
        """Run inference; returns :class:`tritonclient.grpc.InferResult`."""
        metadata = self._get_metadata(headers)
        if type(model_version) != str:  # noqa: E721
            raise_error("model version must be a string")
        request = _get_inference_request(model_name=model_name, inputs=inputs, model_version=model_version,
                                         request_id=request_id, outputs=outputs, sequence_id=sequence_id,
                                         sequence_start=sequence_start, sequence_end=sequence_end,
                                         priority=priority, timeout=timeout, parameters=parameters)
        if self._verbose:
            print("infer, metadata {}\n{}".format(metadata, request))
        try:
            response = await self._client_stub.ModelInfer(
                request=request, metadata=metadata, timeout=client_timeout,
                compression=_grpc_compression_type(compression_algorithm))
        except grpc.RpcError as rpc_error:
            raise_error_grpc(rpc_error)
        if self._verbose:
            print(response)
        return InferResult(response)

    def stream_infer(self, inputs_iterator, stream_timeout=None, headers=None, compression_algorithm=None):
        """Bidirectional streaming inference.

        ``inputs_iterator`` is an async iterator of dicts holding the keyword
        arguments of :py:meth:`tritonclient.grpc.InferenceServerClient.async_stream_infer`
        (``model_name``, ``inputs``, ...).  Returns an async iterator of
        ``(InferResult, InferenceServerException)`` tuples (one of them None)
        with a ``cancel()`` method.
        """
        metadata = self._get_metadata(headers)
        verbose = self._verbose

        async def _request_iterator(it):
            async for kw in it:
                if type(kw) != dict:  # noqa: E721
                    raise_error("inputs_iterator is not yielding a dict")
                if "model_name" not in kw or "inputs" not in kw:
                    raise_error("model_name and/or inputs is missing")
                enable_empty = bool(kw.get("enable_empty_final_response", False))
                model_version = kw.get("model_version", "")
                if type(model_version) != str:  # noqa: E721
                    raise_error("model version must be a string")
                request = _get_inference_request(
                    model_name=kw["model_name"], inputs=kw["inputs"], model_version=model_version,
                    request_id=kw.get("request_id", ""), outputs=kw.get("outputs"),
                    sequence_id=kw.get("sequence_id", 0), sequence_start=kw.get("sequence_start", False),
                    sequence_end=kw.get("sequence_end", False), priority=kw.get("priority", 0),
                    timeout=kw.get("timeout"), parameters=kw.get("parameters"))
                if enable_empty:
                    request.parameters["triton_enable_empty_final_response"].bool_param = True
                if verbose:
                    print("stream_infer request\n{}".format(request))
                yield request

        call = self._client_stub.ModelStreamInfer(
            _request_iterator(inputs_iterator), metadata=metadata, timeout=stream_timeout,
            compression=_grpc_compression_type(compression_algorithm))

        class _ResponseIterator:
            def __init__(self, grpc_call, verbose):
                self._call = grpc_call
                self._verbose = verbose

            def __aiter__(self):
                return self

            async def __anext__(self):
                try:
                    response = await self._call.read()
                except grpc.RpcError as rpc_error:
                    return None, get_error_grpc(rpc_error)
                if response is grpc.aio.EOF:
                    raise StopAsyncIteration
                if self._verbose:
                    print(response)
                if response.error_message != "":
                    return None, InferenceServerException(msg=response.error_message)
                return InferResult(response.infer_response), None

            def cancel(self):
                return self._call.cancel()

        return _ResponseIterator(call, verbose)
