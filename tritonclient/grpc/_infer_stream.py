"""Bidirectional ModelStreamInfer engine (reference tritonclient/grpc/_infer_stream.py:39-191).

A request queue feeds grpcio's request iterator; one response thread invokes
``callback(result=..., error=...)`` for every stream response (decoupled
models may produce 0..N responses per request).
"""
import queue
import threading

import grpc

from tritonclient.utils import InferenceServerException, raise_error

from ._infer_result import InferResult
from ._utils import get_cancelled_error, get_error_grpc


class _InferStream:
    def __init__(self, callback, verbose):
        self._callback = callback
        self._verbose = verbose
        self._request_queue = queue.Queue()
        self._handler = None
        self._cancelled = False
        self._active = True
        self._response_iterator = None

    def __del__(self):
        try:
            self.close(cancel_requests=True)
        except Exception:
            pass

    def close(self, cancel_requests=False):
        """Close the stream; optionally cancel pending requests."""
        if cancel_requests and self._response_iterator:
            self._response_iterator.cancel()
            self._cancelled = True
        if self._handler is not None:
            if not self._cancelled:
                self._request_queue.put(None)
            if self._handler.is_alive() and self._handler is not threading.current_thread():
                self._handler.join()
                if self._verbose:
                    print("stream stopped...")
            self._handler = None

    def _init_handler(self, response_iterator):
        self._response_iterator = response_iterator
        if self._handler is not None:
            raise_error("Attempted to initialize already initialized InferStream")
        self._handler = threading.Thread(target=self._process_response, daemon=True)
        self._handler.start()
        if self._verbose:
            print("stream started...")

    def _enqueue_request(self, request):
        if self._active:
            self._request_queue.put(request)
        else:
            raise_error(
                "The stream is no longer in valid state, the error detail "
                "is reported through provided callback. A new stream should "
                "be started after stopping the current stream."
            )

    def _get_request(self):
        return self._request_queue.get()

    def _process_response(self):
        try:
            for response in self._response_iterator:
                if self._verbose:
                    print(response)
                result = error = None
                if response.error_message != "":
                    error = InferenceServerException(msg=response.error_message)
                else:
                    result = InferResult(response.infer_response)
                self._callback(result=result, error=error)
        except grpc.RpcError as rpc_error:
            self._active = self._response_iterator.is_active()
            if rpc_error.code() == grpc.StatusCode.CANCELLED:
                error = get_cancelled_error(rpc_error.details())
            else:
                error = get_error_grpc(rpc_error)
            self._callback(result=None, error=error)


class _RequestIterator:
    def __init__(self, stream):
        self._stream = stream

    def __iter__(self):
        return self

    def __next__(self):
        request = self._stream._get_request()
        if request is None:
            raise StopIteration
        return request
