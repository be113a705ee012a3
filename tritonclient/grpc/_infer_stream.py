"""Bidirectional ModelStreamInfer session.

Behaviour contract: reference ``tritonclient/grpc/_infer_stream.py:39-191``
(one active stream per client, responses delivered as
``callback(result=..., error=...)``, 0..N responses per request for decoupled
models, ``stop_stream(cancel_requests=...)``).  The design here is our own:

* a :class:`StreamSession` owns an outbox (``deque`` guarded by one
  ``Condition``) and an explicit lifecycle state::

      IDLE --attach--> OPEN --close()--> DRAINING --server EOF--> CLOSED
                        |  \\--close(cancel)--> CANCELLED ----------/
                        \\--rpc error--> FAILED

* grpcio pulls requests from :meth:`StreamSession.outgoing`, a generator that
  blocks on the condition until a request arrives or the session stops
  accepting work (the half-close is the generator returning, not a sentinel
  object in the queue).
* one dispatch thread consumes the response iterator and runs the user
  callback; the terminal rpc status (if not a clean EOF) is delivered once
  through the same callback and moves the session to FAILED/CANCELLED.
* ``close()`` is idempotent and safe from inside the callback (it never
  joins the dispatch thread from itself).
"""
import collections
import enum
import threading

import grpc

from tritonclient.utils import InferenceServerException, raise_error

from ._infer_result import InferResult
from ._utils import get_cancelled_error, get_error_grpc


class StreamState(enum.Enum):
    IDLE = "idle"            # created, no rpc attached yet
    OPEN = "open"            # accepting requests
    DRAINING = "draining"    # half-closed: no new requests, waiting for the server's EOF
    CANCELLED = "cancelled"  # rpc cancelled by the client
    FAILED = "failed"        # rpc ended with an error (reported via callback)
    CLOSED = "closed"        # clean end of stream


_TERMINAL = (StreamState.CANCELLED, StreamState.FAILED, StreamState.CLOSED)


class StreamSession:
    """One ModelStreamInfer rpc: outbox, dispatch thread and lifecycle."""

    def __init__(self, callback, verbose=False):
        self._callback = callback
        self._verbose = verbose
        self._cv = threading.Condition()
        self._outbox = collections.deque()
        self._state = StreamState.IDLE
        self._call = None
        self._dispatcher = None

    # -- lifecycle ------------------------------------------------------------
    @property
    def state(self):
        return self._state

    def _set_state(self, new):
        # caller holds self._cv
        if self._state in _TERMINAL:
            return
        self._state = new
        self._cv.notify_all()

    def attach(self, call):
        """Bind the rpc returned by ``stub.ModelStreamInfer(self.outgoing())``."""
        with self._cv:
            if self._state is not StreamState.IDLE:
                raise_error("stream session is already attached to an rpc")
            self._call = call
            self._state = StreamState.OPEN
        self._dispatcher = threading.Thread(target=self._dispatch, name="triton-grpc-stream", daemon=True)
        self._dispatcher.start()
        if self._verbose:
            print("stream started...")

    def submit(self, request):
        """Queue one ModelInferRequest for sending."""
        with self._cv:
            if self._state is not StreamState.OPEN:
                raise_error(
                    "The stream is no longer in valid state (%s); the error detail was "
                    "reported through the stream callback. Stop this stream and start a "
                    "new one." % self._state.value
                )
            self._outbox.append(request)
            self._cv.notify_all()

    def close(self, cancel_requests=False):
        """Stop the session.

        ``cancel_requests=False`` half-closes (requests already queued are
        still sent) and waits for every response; ``True`` cancels the rpc,
        dropping queued requests and in-flight responses.
        """
        with self._cv:
            if self._state is StreamState.IDLE:
                self._state = StreamState.CLOSED
                return
            if cancel_requests and self._state not in _TERMINAL:
                self._outbox.clear()
                self._set_state(StreamState.CANCELLED)
                call = self._call
            else:
                call = None
                if self._state is StreamState.OPEN:
                    self._set_state(StreamState.DRAINING)
        if call is not None:
            call.cancel()
        t = self._dispatcher
        if t is not None and t is not threading.current_thread() and t.is_alive():
            t.join()
            if self._verbose:
                print("stream stopped...")

    def __del__(self):
        try:
            self.close(cancel_requests=True)
        except Exception:
            pass

    # -- grpc side ------------------------------------------------------------
    def outgoing(self):
        """Request generator handed to grpcio (runs on grpcio's sender thread)."""
        while True:
            with self._cv:
                while not self._outbox and self._state in (StreamState.IDLE, StreamState.OPEN):
                    self._cv.wait()
                if self._outbox and self._state not in (StreamState.CANCELLED, StreamState.FAILED):
                    req = self._outbox.popleft()
                else:
                    return  # half-close (DRAINING with an empty outbox) or terminal
            yield req

    def _deliver(self, result, error):
        try:
            self._callback(result=result, error=error)
        except Exception as e:  # a faulty callback must not kill the session silently
            if self._verbose:
                print("stream callback raised: %r" % (e,))

    def _dispatch(self):
        call = self._call
        try:
            for response in call:
                if self._verbose:
                    print(response)
                if response.error_message:
                    self._deliver(None, InferenceServerException(msg=response.error_message))
                else:
                    self._deliver(InferResult(response.infer_response), None)
        except grpc.RpcError as rpc_error:
            cancelled = rpc_error.code() == grpc.StatusCode.CANCELLED
            with self._cv:
                self._set_state(StreamState.CANCELLED if cancelled else StreamState.FAILED)
            # a cancel the client asked for is reported too (reference
            # behaviour: the callback sees the CANCELLED status once)
            err = get_cancelled_error(rpc_error.details()) if cancelled else get_error_grpc(rpc_error)
            self._deliver(None, err)
            return
        with self._cv:
            self._set_state(StreamState.CLOSED)


# Names the client module imports (kept for code that reached into them).
_InferStream = StreamSession
