"""CPU model zoo used by the examples and the test-suite.

Behaviour is pinned by the reference's example/test expectations:

* ``simple`` / ``simple_string`` — add/sub of two [1,16] tensors
  (reference src/python/examples/simple_http_infer_client.py:207-290,
  simple_http_string_infer_client.py:41-105).
* ``simple_identity`` — BYTES identity (simple_http_string_infer_client.py:110-141).
* ``onnx_int32_int32_int32`` v1..3 — add/sub; v2,v3 swap the outputs
  (reference src/c++/tests/cc_client_test.cc:435-470).
* ``custom_identity_int32`` — identity with an execution delay, for timeout tests
  (reference src/c++/tests/client_timeout_test.cc:421).
* ``simple_sequence`` / ``simple_dyna_sequence`` / ``simple_string_dyna_sequence``
  — stateful models (simple_grpc_sequence_sync_infer_client.py:186-205).
* ``repeat_int32`` — decoupled: one response per IN element after DELAY[i] ms
  (simple_grpc_custom_repeat.py:78-152).
* ``preprocess_inception`` + ``preprocess_inception_ensemble`` — BYTES image ->
  tensor -> classifier ensemble (ensemble_image_client.py).
"""

import threading
import time

import numpy as np

from .model_base import Model, TensorSpec
from .types import ServerError


class SimpleAddSub(Model):
    name = "simple"
    max_batch_size = 8
    inputs = (TensorSpec("INPUT0", "INT32", [16]), TensorSpec("INPUT1", "INT32", [16]))
    outputs = (TensorSpec("OUTPUT0", "INT32", [16]), TensorSpec("OUTPUT1", "INT32", [16]))
    swap_versions = ()

    def execute(self, requests):
        out = []
        for r in requests:
            try:
                a = r.input("INPUT0").numpy()
                b = r.input("INPUT1").numpy()
                s, d = np.add(a, b, dtype=a.dtype), np.subtract(a, b, dtype=a.dtype)
                if self.version in self.swap_versions:
                    s, d = d, s
                out.append([self.out("OUTPUT0", s), self.out("OUTPUT1", d)])
            except Exception as e:  # per-request failure
                out.append(e)
        return out


class OnnxInt32(SimpleAddSub):
    name = "onnx_int32_int32_int32"
    platform = "onnxruntime_onnx"
    backend = "onnxruntime"
    versions = (1, 2, 3)
    swap_versions = (2, 3)


class SimpleString(Model):
    name = "simple_string"
    max_batch_size = 8
    inputs = (TensorSpec("INPUT0", "BYTES", [16]), TensorSpec("INPUT1", "BYTES", [16]))
    outputs = (TensorSpec("OUTPUT0", "BYTES", [16]), TensorSpec("OUTPUT1", "BYTES", [16]))

    def execute(self, requests):
        res = []
        for r in requests:
            try:
                a = r.input("INPUT0").numpy()
                b = r.input("INPUT1").numpy()
                ai = np.vectorize(lambda x: int(x))(a).astype(np.int64)
                bi = np.vectorize(lambda x: int(x))(b).astype(np.int64)
                s = np.array([str(x).encode() for x in (ai + bi).ravel()], dtype=np.object_)
                d = np.array([str(x).encode() for x in (ai - bi).ravel()], dtype=np.object_)
                res.append([self.out("OUTPUT0", s.reshape(a.shape)), self.out("OUTPUT1", d.reshape(a.shape))])
            except Exception as e:
                res.append(ServerError("simple_string: %s" % e))
        return res


class Identity(Model):
    """Generic identity over one input (datatype set per instance)."""

    name = "simple_identity"
    max_batch_size = 8
    datatype = "BYTES"

    def __init__(self, version=1, **kw):
        super().__init__(version, **kw)
        self.inputs = (TensorSpec("INPUT0", self.datatype, [-1]),)
        self.outputs = (TensorSpec("OUTPUT0", self.datatype, [-1]),)

    def execute(self, requests):
        delay_ms = float(self.options.get("delay_ms", 0))
        if delay_ms:
            time.sleep(delay_ms / 1000.0)
        return [[self.out("OUTPUT0", r.input("INPUT0").numpy())] for r in requests]


class CustomIdentityInt32(Identity):
    name = "custom_identity_int32"
    datatype = "INT32"

    def __init__(self, version=1, **kw):
        kw.setdefault("delay_ms", 500)
        super().__init__(version, **kw)


class IdentityInt32(Identity):
    """custom_identity_int32 without the delay (soak tests)."""

    name = "identity_int32"
    datatype = "INT32"


class IdentityFP32(Identity):
    name = "identity_fp32"
    datatype = "FP32"
    max_batch_size = 0


class IdentityInt8(Identity):
    name = "identity_int8"
    datatype = "INT8"


class IdentityBF16(Identity):
    name = "identity_bf16"
    datatype = "BF16"
    max_batch_size = 0


class SimpleSequence(Model):
    """out = in + 1 on the START request, else out = in (int or string corrid)."""

    name = "simple_sequence"
    max_batch_size = 8
    sequence_batching = True
    inputs = (TensorSpec("INPUT", "INT32", [1]),)
    outputs = (TensorSpec("OUTPUT", "INT32", [1]),)

    def __init__(self, version=1, **kw):
        super().__init__(version, **kw)
        self._state = {}
        self._lock = threading.Lock()

    def _step(self, r, x):
        return x + (1 if r.sequence_start else 0)

    def execute(self, requests):
        res = []
        for r in requests:
            if r.sequence_id in (0, ""):
                res.append(ServerError(
                    "inference request to model '%s' must specify a non-zero or non-empty correlation ID"
                    % self.name))
                continue
            x = r.input("INPUT").numpy()
            with self._lock:
                y = self._step(r, x)
                if r.sequence_end:
                    self._state.pop(r.sequence_id, None)
            res.append([self.out("OUTPUT", np.asarray(y, dtype=np.int32))])
        return res


class SimpleDynaSequence(SimpleSequence):
    """Like simple_sequence, plus the correlation id on the END request."""

    name = "simple_dyna_sequence"

    def _step(self, r, x):
        y = x + (1 if r.sequence_start else 0)
        if r.sequence_end:
            y = y + int(r.sequence_id)
        return y


class SimpleStringDynaSequence(SimpleSequence):
    """Accumulator keyed by a string correlation id that must decode to int."""

    name = "simple_string_dyna_sequence"

    def _step(self, r, x):
        try:
            corr = int(r.sequence_id)
        except (TypeError, ValueError):
            raise ServerError("simple_string_dyna_sequence requires an integer-decodable sequence id")
        if r.sequence_start:
            acc = x.copy()
        else:
            acc = self._state.get(r.sequence_id, np.zeros_like(x)) + x
        self._state[r.sequence_id] = acc
        y = acc
        if r.sequence_end:
            y = acc + corr
        return y


class RepeatInt32(Model):
    """Decoupled: for each element i of IN, sleep DELAY[i] ms then emit OUT=[IN[i]]
    and IDX=[i]; WAIT ms are slept before releasing the request."""

    name = "repeat_int32"
    decoupled = True
    inputs = (
        TensorSpec("IN", "INT32", [-1]),
        TensorSpec("DELAY", "UINT32", [-1]),
        TensorSpec("WAIT", "UINT32", [1]),
    )
    outputs = (TensorSpec("OUT", "INT32", [1]), TensorSpec("IDX", "UINT32", [1]))

    def execute_decoupled(self, request, emit):
        vals = request.input("IN").numpy().ravel()
        d = request.input("DELAY")
        delays = d.numpy().ravel() if d is not None else np.zeros(len(vals), np.uint32)
        w = request.input("WAIT")
        wait = int(w.numpy().ravel()[0]) if w is not None else 0
        if len(delays) != len(vals):
            raise ServerError("repeat_int32: IN and DELAY must have the same length")
        for i, v in enumerate(vals):
            if delays[i]:
                time.sleep(delays[i] / 1000.0)
            emit([
                self.out("OUT", np.array([v], dtype=np.int32)),
                self.out("IDX", np.array([i], dtype=np.uint32)),
            ])
        if wait:
            time.sleep(wait / 1000.0)


class PreprocessInception(Model):
    """Decode a raw image (BYTES: PPM/PGM or raw HxWx3 uint8 with a header) and
    produce INCEPTION-scaled FP32 NCHW [3,224,224]."""

    name = "preprocess_inception"
    max_batch_size = 8
    inputs = (TensorSpec("INPUT", "BYTES", [1]),)
    outputs = (TensorSpec("OUTPUT", "FP32", [3, 224, 224]),)

    def execute(self, requests):
        from triton_client_amd.utils.image import decode_image, inception_preprocess

        res = []
        for r in requests:
            blobs = r.input("INPUT").numpy().reshape(-1)
            outs = []
            for b in blobs:
                img = decode_image(b)
                outs.append(inception_preprocess(img, 224, 224, "NCHW"))
            res.append([self.out("OUTPUT", np.stack(outs).astype(np.float32))])
        return res


class AddSubBatched(Model):
    """INT32 add/sub with dynamic batching; also served on the native fast path.

    ``execute_native`` receives one batch from tcserve (csrc/cpp/server) with
    host pointers (in-band tensors or system shared memory) and writes the
    outputs in place.
    """

    name = "add_sub_batched"
    max_batch_size = 8
    inputs = (TensorSpec("INPUT0", "INT32", [16]), TensorSpec("INPUT1", "INT32", [16]))
    outputs = (TensorSpec("OUTPUT0", "INT32", [16]), TensorSpec("OUTPUT1", "INT32", [16]))
    dynamic_batching = {"preferred": [], "max_queue_delay_us": 200}
    instance_count = 2
    supports_native = True
    native_delay_s = 0.0  # tests: hold each native batch this long (region-lifetime checks)

    def execute(self, requests):
        out = []
        for r in requests:
            try:
                a = r.input("INPUT0").numpy()
                b = r.input("INPUT1").numpy()
                out.append([self.out("OUTPUT0", a + b), self.out("OUTPUT1", a - b)])
            except Exception as e:  # per-request failure
                out.append(e)
        return out

    def execute_native(self, instance, b):
        import ctypes
        import time

        t0 = time.monotonic_ns()
        if self.native_delay_s:
            time.sleep(self.native_delay_s)
        ni, no = b.n_inputs, b.n_outputs
        for r in range(b.n_requests):
            rows = b.rows[r]
            arrs = []
            for k in range(ni):
                ref = b.inputs[r * ni + k]
                if ref.kind != 0:
                    raise ServerError("add_sub_batched runs on host memory only")
                arrs.append(np.ctypeslib.as_array((ctypes.c_int32 * (rows * 16)).from_address(ref.ptr)))
            res = (arrs[0] + arrs[1], arrs[0] - arrs[1])
            for k in range(no):
                ref = b.outputs[r * no + k]
                if ref.ptr:
                    if ref.kind != 0:
                        raise ServerError("add_sub_batched runs on host memory only")
                    np.ctypeslib.as_array((ctypes.c_int32 * (rows * 16)).from_address(ref.ptr))[:] = res[k]
        t1 = time.monotonic_ns()
        b.timing_ns[0] = 0
        b.timing_ns[1] = t1 - t0
        b.timing_ns[2] = 0


class AddSubPipelined(AddSubBatched):
    """add_sub_batched with every tcserve batcher rule engaged: 2 instances,
    a preferred batch of 8 rows (full batches -> staggered starts), idle-aware
    and pipelined dispatch of partial batches.  Exists so the threaded
    batcher's rules run under the sanitizers (tools/sanitize_tcserve.py) and
    the CPU tests; the rules themselves are unit-tested on scripted arrivals
    (tests/test_batch_policy.py)."""

    name = "add_sub_pipelined"
    dynamic_batching = {"preferred": [8], "max_queue_delay_us": 300, "pipelined": True}
    instance_count = 2
    native_delay_s = 0.0002  # each batch holds its instance ~0.2 ms: queues build, rules fire


class FrontendSink(Model):
    """densenet_onnx-shaped model that does no compute: FP32 [3,224,224] in,
    FP32 [1000] out (first input value broadcast).  Served natively, it
    measures what the tcserve front end and the transport alone sustain for
    the headline request shape, with no GPU involved."""

    name = "frontend_sink"
    max_batch_size = 8
    inputs = (TensorSpec("data_0", "FP32", [3, 224, 224]),)
    outputs = (TensorSpec("fc6_1", "FP32", [1000]),)
    dynamic_batching = {"preferred": [], "max_queue_delay_us": 100}
    instance_count = 2
    supports_native = True

    def execute(self, requests):
        out = []
        for r in requests:
            x = r.input("data_0").numpy()
            out.append([self.out("fc6_1", np.repeat(x.reshape(x.shape[0], -1)[:, :1], 1000, axis=1))])
        return out

    def execute_native(self, instance, b):
        import ctypes

        for r in range(b.n_requests):
            rows = b.rows[r]
            src, dst = b.inputs[r], b.outputs[r]
            if src.kind != 0 or (dst.ptr and dst.kind != 0):
                raise ServerError("frontend_sink runs on host memory only")
            if not dst.ptr:
                continue
            x = np.ctypeslib.as_array((ctypes.c_float * (rows * 3 * 224 * 224)).from_address(src.ptr))
            y = np.ctypeslib.as_array((ctypes.c_float * (rows * 1000)).from_address(dst.ptr)).reshape(rows, 1000)
            y[:] = x.reshape(rows, -1)[:, :1]
        b.timing_ns[0] = b.timing_ns[1] = b.timing_ns[2] = 0


class BertSink(Model):
    """bert_large-shaped model that does no compute: INT32 [384] input_ids /
    attention_mask / token_type_ids in, FP32 [384] start/end logits out (the
    mask as float).  The CPU stand-in of bench.py's bert_large sweep, so the
    multi-rank launch + fan-out + sweep aggregation path runs without a GPU."""

    name = "bert_sink"
    max_batch_size = 64
    SEQ = 384
    inputs = (TensorSpec("input_ids", "INT32", [384]), TensorSpec("attention_mask", "INT32", [384]),
              TensorSpec("token_type_ids", "INT32", [384]))
    outputs = (TensorSpec("start_logits", "FP32", [384]), TensorSpec("end_logits", "FP32", [384]))
    dynamic_batching = {"preferred": [], "max_queue_delay_us": 100}
    instance_count = 2
    supports_native = True

    def execute(self, requests):
        out = []
        for r in requests:
            m = r.input("attention_mask").numpy().astype(np.float32)
            out.append([self.out("start_logits", m), self.out("end_logits", -m)])
        return out

    def execute_native(self, instance, b):
        import ctypes

        n = self.SEQ
        for r in range(b.n_requests):
            rows = b.rows[r]
            src = b.inputs[r * 3 + 1]
            if src.kind != 0:
                raise ServerError("bert_sink runs on host memory only")
            m = np.ctypeslib.as_array((ctypes.c_int32 * (rows * n)).from_address(src.ptr)).astype(np.float32)
            for k, sign in ((0, 1.0), (1, -1.0)):
                dst = b.outputs[r * 2 + k]
                if not dst.ptr:
                    continue
                if dst.kind != 0:
                    raise ServerError("bert_sink runs on host memory only")
                np.ctypeslib.as_array((ctypes.c_float * (rows * n)).from_address(dst.ptr))[:] = sign * m
        b.timing_ns[0] = b.timing_ns[1] = b.timing_ns[2] = 0


CPU_MODELS = [
    FrontendSink,
    BertSink,
    SimpleAddSub,
    OnnxInt32,
    SimpleString,
    Identity,
    CustomIdentityInt32,
    IdentityInt32,
    IdentityFP32,
    IdentityBF16,
    IdentityInt8,
    SimpleSequence,
    SimpleDynaSequence,
    SimpleStringDynaSequence,
    RepeatInt32,
    PreprocessInception,
    AddSubBatched,
    AddSubPipelined,
]
