"""GPU model backends of the bench server (torch-ROCm + in-tree HIP kernels).

``densenet_onnx`` — the BASELINE model (FP32 ``data_0`` [3,224,224] NCHW in,
FP32 ``fc6_1`` [1000] out; same I/O contract as Triton's densenet_onnx example)
served with dynamic batching on one MI355X:

  request inputs (device shm views / host tensors)
    --pointer table (one 1 KB H2D)--> HIP graph replay of DenseNet-121 on
        hand-written MFMA kernels whose first kernel reads every image
        straight from its request's fp32 NCHW region (the batch is never
        assembled).  engine="fp32" (default, the model's FP32 contract):
        split-precision bf16x3 kernels K8x-K10x (models/densenet_fp32.py),
        logits within ~4e-5 rel-L2 of the fp32 module.  engine="fused": the
        bf16 K8-K10 kernels (models/densenet_fused.py), ~2.2x faster, ~3e-2
        off fp32 — a labelled reduced-precision operating point.
        engine="torch" keeps the MIOpen per-op bf16 module, fed by K6
        layout_pack (gather+transpose+cvt into one bf16 NHWC batch buffer)
    --K7 batched_copy--> each request's fp32 logits straight into its output
                         device-shm region (one launch per batch)

Host (non-shm) inputs are staged through pinned memory; host outputs come back
with one D2H of the whole batch.  Each model instance owns a torch stream, its
graphs (one per batch bucket) and static buffers, so ``instance_count``
batches pipeline on separate HIP streams.
"""

import os
import threading

import numpy as np

from triton_client_amd.utils import roctx

from .model_base import Model, TensorSpec
from .types import DeviceView, OutputTensor, ServerError

# HIP-graph batch buckets: powers of two up to 16, then every 8 rows to 128 and
# every 16 to 256.  A batch runs the smallest bucket that holds it, and the
# padding rows cost full compute: under the headline load (bs8 requests, 128-row
# preferred batches) batches average 109-124 rows, which power-of-two buckets
# padded to 128 (3-15% of the device time spent on padding)
BUCKETS = (1, 2, 4, 8, 12, 16, 20) + tuple(range(24, 129, 8)) + tuple(range(144, 257, 16))


class DensenetOnnx(Model):
    name = "densenet_onnx"
    platform = "onnxruntime_onnx"
    backend = "onnxruntime"
    max_batch_size = 128
    inputs = (TensorSpec("data_0", "FP32", [3, 224, 224], fmt="NCHW"),)
    outputs = (TensorSpec("fc6_1", "FP32", [1000], label_filename="densenet_labels.txt"),)
    # pipelined: tcserve dispatches a partial batch to a free instance once the
    # queue holds as many rows as the last batch (bs1 closed loops)
    dynamic_batching = {"preferred": [], "max_queue_delay_us": 500, "pipelined": True}
    instance_kind = "KIND_GPU"
    instance_count = 2
    gpus = (0,)
    labels = ["class_%d" % i for i in range(1000)]

    C, H, W = 3, 224, 224
    OUT = 1000

    ENGINES = ("fp32", "fused", "torch")

    def __init__(self, version=1, device_id=0, buckets=BUCKETS, use_graphs=True, engine="fp32", max_batch_size=0,
                 **kw):
        super().__init__(version, **kw)
        if engine not in self.ENGINES:
            raise ServerError("unknown densenet engine %r" % engine)
        self.engine = engine
        self.device_id = int(kw.get("device", device_id))
        if max_batch_size:
            # option max_batch_size: the HIP-graph buckets up to it (BUCKETS).  The fused engine's device throughput keeps growing with the
            # rows per forward: on MI355X (tools/engine_streams_bench.py) ~64k
            # img/s with 128-row forwards on 3-4 streams, ~70k with 256-row
            # forwards on 2 streams.
            if int(max_batch_size) not in buckets:
                raise ServerError("max_batch_size must be one of %s" % (tuple(buckets),))
            self.max_batch_size = int(max_batch_size)
        self.buckets = tuple(b for b in buckets if b <= self.max_batch_size)
        self.use_graphs = use_graphs
        self._slots = []
        self._free = []
        self._cv = threading.Condition()

    # -- load ----------------------------------------------------------------------
    def load(self):
        import torch

        from triton_client_amd.models import densenet
        from triton_client_amd.ops import hip

        if not torch.cuda.is_available():
            raise ServerError("densenet_onnx requires a GPU")
        hip.lib()  # fail loudly if the native kernels are missing
        torch.cuda.set_device(self.device_id)
        self.torch = torch
        dev = torch.device("cuda", self.device_id)
        if self.engine == "fp32":
            from triton_client_amd.models import densenet_fp32

            self.model, _ = densenet_fp32.build(max(self.buckets), device=dev)
        elif self.engine == "fused":
            from triton_client_amd.models import densenet_fused

            self.model, _ = densenet_fused.build(max(self.buckets), device=dev)
        else:
            self.model = densenet.build(device=dev)
        self.scale = None
        # the instances' streams run concurrently: engines route small batches for that
        self.model.concurrent_streams = max(1, self.instance_count)
        for _ in range(max(1, self.instance_count)):
            self._slots.append(self._make_slot(dev))
        self._free = list(range(len(self._slots)))
        self._pgx = None
        if self.engine != "torch" and self.use_graphs and os.environ.get("TCAMD_NATIVE_EXEC", "1") != "0":
            self._pgx = self._make_executor()

    def _make_executor(self):
        """C++ per-batch dispatch (csrc/runtime/graph_exec.hip): pointer table,
        graph replay, output scatter and the completion wait run in the server's
        batcher thread without Python (the GIL stays out of the request path)."""
        from triton_client_amd.ops import hip

        x = hip.PtrGraphExecutor(self.device_id, len(self._slots), self.C * self.H * self.W * 4, self.OUT * 4,
                                 self.buckets)
        for i, slot in enumerate(self._slots):
            execs = [slot["graphs"][b].raw_cuda_graph_exec() for b in self.buckets]
            x.bind(i, slot["stream"].cuda_stream, execs, slot["net"].ptrs.data_ptr(), slot["stage_dev"].data_ptr(),
                   slot["out"].data_ptr(), slot["pad_ptrs"])
        return x

    def native_executor(self):
        """(tcserve_exec_fn address, user pointer) of the C++ executor, or None."""
        if self._pgx is None:
            return None
        return self._pgx.fn_address, self._pgx.handle

    def executor_stats(self):
        return None if self._pgx is None else self._pgx.stats()

    def _make_slot(self, dev):
        torch = self.torch
        from triton_client_amd.ops import hip

        net = self.model
        if self.engine != "torch" and self._slots:
            net = self.model.with_workspace()  # own activation buffers per concurrent stream
        slot = {"stream": torch.cuda.Stream(device=dev), "graphs": {}, "net": net,
                "ev": [torch.cuda.Event(enable_timing=True) for _ in range(4)]}
        maxb = max(self.buckets)
        img_bytes = self.C * self.H * self.W * 4
        fused = self.engine != "torch"  # pointer-table engines (fp32 / bf16 fused kernels)
        slot["out"] = torch.zeros(maxb, self.OUT, device=dev, dtype=torch.float32)
        slot["stage_host"] = hip.host_alloc(maxb * img_bytes)
        slot["stage_dev"] = torch.zeros(maxb * self.C * self.H * self.W, device=dev, dtype=torch.float32)
        slot["out_host"] = hip.host_alloc(maxb * self.OUT * 4)
        if fused:
            # padded rows of a bucket read (finite) staging images, never a stale request region
            pad = np.arange(maxb, dtype=np.int64) * img_bytes + slot["stage_dev"].data_ptr()
            slot["pad_ptrs"] = pad
            slot["ptrs_host"] = hip.host_alloc(maxb * 8)
            slot["ptrs_tbl"] = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_int64 * maxb).from_address(
                slot["ptrs_host"]))
            net.ptrs.copy_(torch.from_numpy(pad))

            def run(b):
                return net.forward_ptrs(b, out=slot["out"])
        else:
            slot["inp"] = torch.zeros(maxb, self.H, self.W, self.C, device=dev, dtype=torch.bfloat16)

            def run(b):
                x = slot["inp"][:b].permute(0, 3, 1, 2)  # NCHW view of NHWC memory
                return slot["out"][:b].copy_(net(x).float())
        with torch.cuda.stream(slot["stream"]), torch.no_grad():
            for b in self.buckets:
                for _ in range(2):  # warm up library kernel selection
                    run(b)
                if self.use_graphs:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=slot["stream"]):
                        run(b)
                    slot["graphs"][b] = g
        slot["stream"].synchronize()
        return slot

    def unload(self):
        from triton_client_amd.ops import hip

        if getattr(self, "_pgx", None) is not None:
            self._pgx.close()
            self._pgx = None
        for s in self._slots:
            try:
                hip.host_free(s["stage_host"])
                hip.host_free(s["out_host"])
                if "ptrs_host" in s:
                    hip.host_free(s["ptrs_host"])
            except Exception:
                pass
        self._slots = []

    # -- execute ----------------------------------------------------------------------
    def _acquire(self):
        with self._cv:
            while not self._free:
                self._cv.wait()
            return self._free.pop()

    def _release(self, i):
        with self._cv:
            self._free.append(i)
            self._cv.notify()

    def forward_device(self, slot, srcs, rows):
        """Assemble ``rows`` images from device pointers and run the model."""
        with roctx.range("densenet_onnx.forward rows=%d" % rows):
            return self._forward_device(slot, srcs, rows)

    def _forward_device(self, slot, srcs, rows):
        torch = self.torch
        from triton_client_amd.ops import hip

        bucket = next(b for b in self.buckets if b >= rows)
        stream = slot["stream"]
        sh = stream.cuda_stream
        fused = self.engine != "torch"
        slot["ev"][0].record(stream)
        if fused:
            tbl = slot["ptrs_tbl"]
            tbl[:rows] = srcs
            tbl[rows:bucket] = slot["pad_ptrs"][rows:bucket]
            hip.memcpy_async(slot["net"].ptrs.data_ptr(), slot["ptrs_host"], bucket * 8, sh)
        else:
            hip.layout_pack(srcs, "FP32", "NCHW", slot["inp"].data_ptr(), "BF16", "NHWC",
                            self.C, self.H, self.W, rounding="rne", stream=sh)
        slot["ev"][1].record(stream)
        if self.use_graphs:
            with torch.cuda.stream(stream):
                slot["graphs"][bucket].replay()
        else:
            with torch.cuda.stream(stream), torch.no_grad():
                if fused:
                    slot["net"].forward_ptrs(bucket, out=slot["out"])
                else:
                    x = slot["inp"][:bucket].permute(0, 3, 1, 2)
                    slot["out"][:bucket].copy_(slot["net"](x).float())
        slot["ev"][2].record(stream)
        return bucket

    def execute(self, requests):
        torch = self.torch
        from triton_client_amd.ops import hip

        img_bytes = self.C * self.H * self.W * 4
        out_row = self.OUT * 4
        rows = 0
        plan = []  # (request, first_row, nrows)
        for r in requests:
            t = r.input("data_0")
            n = int(t.shape[0])
            plan.append((r, rows, n))
            rows += n
        if rows > max(self.buckets):
            return [ServerError("batch of %d rows exceeds the largest bucket" % rows)] * len(requests)
        if getattr(self, "_pgx", None) is not None:
            return self._execute_pgx(plan, rows, img_bytes, out_row)
        i = self._acquire()
        slot = self._slots[i]
        try:
            stream = slot["stream"]
            sh = stream.cuda_stream
            srcs = []
            host_rows = 0
            for r, first, n in plan:
                t = r.input("data_0")
                if isinstance(t.data, DeviceView):
                    if t.data.nbytes < n * img_bytes:
                        raise ServerError("input region too small for data_0")
                    srcs += [t.data.ptr + k * img_bytes for k in range(n)]
                else:
                    a = np.ascontiguousarray(t.data, dtype=np.float32)
                    dst = slot["stage_host"] + host_rows * img_bytes
                    np.copyto(np.ctypeslib.as_array((np.ctypeslib.ctypes.c_float * a.size).from_address(dst)),
                              a.reshape(-1))
                    srcs += [slot["stage_dev"].data_ptr() + (host_rows + k) * img_bytes for k in range(n)]
                    host_rows += n
            if host_rows:
                hip.memcpy_async(slot["stage_dev"].data_ptr(), slot["stage_host"], host_rows * img_bytes, sh)
            self.forward_device(slot, srcs, rows)
            # outputs: device-shm targets get a K7 scatter, the rest one D2H
            out_base = slot["out"].data_ptr()
            c_src, c_dst, c_n = [], [], []
            need_host = False
            results = []
            for r, first, n in plan:
                ro = next((o for o in r.outputs if o.name == "fc6_1"), None)
                target = None
                if ro is not None and ro.shm is not None and ro.class_count == 0:
                    target = self._server_target(r, ro)
                if isinstance(target, DeviceView):
                    if target.nbytes < n * out_row:
                        raise ServerError(
                            "shared memory size specified with the request for output 'fc6_1' "
                            "(%d bytes) should be at least %d bytes" % (target.nbytes, n * out_row)
                        )
                    c_src.append(out_base + first * out_row)
                    c_dst.append(target.ptr)
                    c_n.append(n * out_row)
                    results.append(("shm", ro))
                else:
                    need_host = True
                    results.append(("host", None))
            if c_src:
                hip.batched_copy(c_src, c_dst, c_n, sh)
            if need_host:
                hip.memcpy_async(slot["out_host"], out_base, rows * out_row, sh)
            slot["ev"][3].record(stream)
            stream.synchronize()
            if self._batch_stats is not None:
                ev = slot["ev"]
                ms_in, ms_inf, ms_out = (ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]),
                                         ev[2].elapsed_time(ev[3]))
                self._batch_stats(rows, len(requests), int(ms_in * 1e6), int(ms_inf * 1e6), int(ms_out * 1e6))
            host_all = None
            if need_host:
                host_all = np.ctypeslib.as_array(
                    (np.ctypeslib.ctypes.c_float * (rows * self.OUT)).from_address(slot["out_host"])
                ).reshape(rows, self.OUT).copy()
            out = []
            for (r, first, n), (kind, ro) in zip(plan, results):
                if kind == "shm":
                    o = OutputTensor("fc6_1", "FP32", [n, self.OUT], None, shm=ro.shm)
                else:
                    o = OutputTensor("fc6_1", "FP32", [n, self.OUT], host_all[first : first + n])
                out.append([o])
            return out
        except ServerError as e:
            return [e] * len(requests)
        finally:
            self._release(i)

    def _execute_pgx(self, plan, rows, img_bytes, out_row):
        """Python-scheduled batch through the same C++ executor tcserve uses."""
        import ctypes

        from .native_frontend import TcBatch, TcRef

        n = len(plan)
        ins = (TcRef * n)()
        outs = (TcRef * n)()
        keep, results = [], []
        try:
            for j, (r, first, k) in enumerate(plan):
                t = r.input("data_0")
                if isinstance(t.data, DeviceView):
                    if t.data.nbytes < k * img_bytes:
                        raise ServerError("input region too small for data_0")
                    ins[j] = TcRef(1, self.device_id, t.data.ptr, t.data.nbytes)
                else:
                    a = np.ascontiguousarray(t.data, dtype=np.float32)
                    keep.append(a)
                    ins[j] = TcRef(0, 0, a.ctypes.data, a.nbytes)
                ro = next((o for o in r.outputs if o.name == "fc6_1"), None)
                target = None
                if ro is not None and ro.shm is not None and ro.class_count == 0:
                    target = self._server_target(r, ro)
                if isinstance(target, DeviceView):
                    if target.nbytes < k * out_row:
                        raise ServerError(
                            "shared memory size specified with the request for output 'fc6_1' "
                            "(%d bytes) should be at least %d bytes" % (target.nbytes, k * out_row)
                        )
                    outs[j] = TcRef(1, self.device_id, target.ptr, target.nbytes)
                    results.append(("shm", ro, None))
                else:
                    host = np.empty((k, self.OUT), dtype=np.float32)
                    outs[j] = TcRef(0, 0, host.ctypes.data, host.nbytes)
                    results.append(("host", None, host))
            nrows = (ctypes.c_int32 * n)(*[k for _, _, k in plan])
            timing = (ctypes.c_uint64 * 3)()
            b = TcBatch(n, rows, nrows, 1, ins, 1, outs, timing)
            i = self._acquire()
            try:
                self._pgx.execute(i, ctypes.addressof(b))
            except RuntimeError as e:
                raise ServerError(str(e)) from e
            finally:
                self._release(i)
        except ServerError as e:
            return [e] * n
        if self._batch_stats is not None:
            self._batch_stats(rows, n, int(timing[0]), int(timing[1]), int(timing[2]))
        out = []
        for (r, first, k), (kind, ro, host) in zip(plan, results):
            if kind == "shm":
                out.append([OutputTensor("fc6_1", "FP32", [k, self.OUT], None, shm=ro.shm)])
            else:
                out.append([OutputTensor("fc6_1", "FP32", [k, self.OUT], host)])
        return out

    # -- native fast path (tcserve, csrc/cpp/server) ------------------------------------
    supports_native = True

    def execute_native(self, instance, b):
        """One dynamic batch assembled by the C++ front end: raw device / host
        pointers in, outputs written straight to their targets."""
        import ctypes

        from triton_client_amd.ops import hip

        img_bytes = self.C * self.H * self.W * 4
        out_row = self.OUT * 4
        total = int(b.total_rows)
        if total > max(self.buckets):
            raise ServerError("batch of %d rows exceeds the largest bucket" % total)
        i = self._acquire()
        slot = self._slots[i]
        try:
            stream = slot["stream"]
            sh = stream.cuda_stream
            srcs, plan = [], []
            host_rows = first = 0
            stage_dev = slot["stage_dev"].data_ptr()
            for r in range(b.n_requests):
                rows = int(b.rows[r])
                ref = b.inputs[r * b.n_inputs]
                if ref.kind == 1:
                    srcs += [ref.ptr + k * img_bytes for k in range(rows)]
                else:  # in-band tensor or system shm: stage through pinned memory
                    ctypes.memmove(slot["stage_host"] + host_rows * img_bytes, ref.ptr, rows * img_bytes)
                    srcs += [stage_dev + (host_rows + k) * img_bytes for k in range(rows)]
                    host_rows += rows
                plan.append((first, rows))
                first += rows
            if host_rows:
                hip.memcpy_async(stage_dev, slot["stage_host"], host_rows * img_bytes, sh)
            self.forward_device(slot, srcs, total)
            out_base = slot["out"].data_ptr()
            c_src, c_dst, c_n, host_outs = [], [], [], []
            for r, (f, rows) in enumerate(plan):
                ref = b.outputs[r * b.n_outputs]
                if not ref.ptr:
                    continue
                if ref.kind == 1:
                    c_src.append(out_base + f * out_row)
                    c_dst.append(ref.ptr)
                    c_n.append(rows * out_row)
                else:
                    host_outs.append((ref.ptr, f, rows))
            if c_src:
                hip.batched_copy(c_src, c_dst, c_n, sh)
            if host_outs:
                hip.memcpy_async(slot["out_host"], out_base, total * out_row, sh)
            ev = slot["ev"]
            ev[3].record(stream)
            hip.stream_synchronize(sh)  # ctypes call: the GIL is released while the GPU runs
            for ptr, f, rows in host_outs:
                ctypes.memmove(ptr, slot["out_host"] + f * out_row, rows * out_row)
            b.timing_ns[0] = int(ev[0].elapsed_time(ev[1]) * 1e6)
            b.timing_ns[1] = int(ev[1].elapsed_time(ev[2]) * 1e6)
            b.timing_ns[2] = int(ev[2].elapsed_time(ev[3]) * 1e6)
        finally:
            self._release(i)

    _server = None
    # set by the scheduler: (rows, n_requests, compute_input_ns, compute_infer_ns, compute_output_ns)
    _batch_stats = None
    reports_batch_stats = True

    def _server_target(self, r, ro):
        region, nbytes, offset = ro.shm
        return self._server.shm_target(region, nbytes, offset)


class PreprocessInceptionEnsemble(Model):
    """Ensemble: raw image bytes -> preprocess_inception -> densenet_onnx
    (the model the reference's ensemble_image_client drives,
    src/python/examples/ensemble_image_client.py)."""

    name = "preprocess_inception_ensemble"
    platform = "ensemble"
    backend = ""
    max_batch_size = 8
    inputs = (TensorSpec("INPUT", "BYTES", [1]),)
    outputs = (TensorSpec("OUTPUT", "FP32", [1000], label_filename="densenet_labels.txt"),)
    ensemble_steps = [
        ("preprocess_inception", {"INPUT": "INPUT"}, {"OUTPUT": "preprocessed_image"}),
        ("densenet_onnx", {"data_0": "preprocessed_image"}, {"fc6_1": "OUTPUT"}),
    ]
    labels = DensenetOnnx.labels

    def load(self):
        pass

    def execute(self, requests):  # pragma: no cover - the server runs ensembles step by step
        raise ServerError("ensemble models are scheduled by the server")


class BertLarge(Model):
    """``bert_large`` — BERT-large SQuAD-style QA (models/bert.py), the model of
    BASELINE.json's concurrency-sweep config.  INT32 [384] input_ids /
    attention_mask / token_type_ids in, FP32 [384] start/end logits out;
    dynamic batching into HIP-graph buckets.  Inputs from device shm are
    gathered with K7 batched_copy (one launch per input tensor), outputs are
    scattered the same way; both the Python scheduler and the native front end
    (execute_native) use it."""

    name = "bert_large"
    platform = "pytorch_libtorch"
    backend = "pytorch"
    # 128: a bs128 HIP-graph forward runs 4,292 seq/s against 4,095 at bs64
    # (tools/bert_probe.py --graphs, profiles/r6_bert_batching/)
    max_batch_size = 128
    SEQ = 384
    inputs = (TensorSpec("input_ids", "INT32", [384]), TensorSpec("attention_mask", "INT32", [384]),
              TensorSpec("token_type_ids", "INT32", [384]))
    outputs = (TensorSpec("start_logits", "FP32", [384]), TensorSpec("end_logits", "FP32", [384]))
    dynamic_batching = {"preferred": [], "max_queue_delay_us": 1000}
    instance_kind = "KIND_GPU"
    instance_count = 1
    supports_native = True
    # HIP-graph buckets: a batch runs the smallest one that holds it.  Steps of
    # 4 rows from 8 to 32 (where c64's batches land), 8 above: closed-loop loads
    # batch anything from 1 to 64 rows, and
    # with power-of-two buckets a 33-row batch paid for 64 (served c64: 33 rows
    # per batch at 11.5 ms vs 7.9 ms for a 32-row forward)
    BUCKETS = (1, 2, 4, 8, 12, 16, 20, 24, 28, 32, 40, 48, 56, 64, 80, 96, 112, 128)
    # a second, unmasked ("dense") graph for the buckets from DENSE_FROM rows,
    # picked per batch when no real row is padded.  Below that every batch
    # runs the masked graph: K12 classifies its key chunks, so an all-ones
    # mask runs the unmasked math (bs1 9.8 vs 9.7-10.8 us), while picking the
    # dense graph costs a device reduction and a host sync per batch on
    # HIP-shm inputs (~40 us of compute_input at c1).  At 64 rows the
    # unmasked kernel is still 4-8 % faster (78-80 vs 82-87 us,
    # profiles/r6_k12/k12_allones.log), worth the sync.
    DENSE_FROM = 32

    def __init__(self, version=1, device_id=0, use_graphs=True, layers=24, **kw):
        super().__init__(version, **kw)
        self.device_id = int(kw.get("device", device_id))
        self.use_graphs = use_graphs
        self.layers = int(layers)
        self._slots = []
        self._free = []
        self._cv = threading.Condition()

    def load(self):
        import torch

        from triton_client_amd.models import bert
        from triton_client_amd.ops import hip

        if not torch.cuda.is_available():
            raise ServerError("bert_large requires a GPU")
        hip.lib()
        torch.cuda.set_device(self.device_id)
        self.torch = torch
        dev = torch.device("cuda", self.device_id)
        self.model = self._build_model(bert, dev)
        # before the warm-up runs and graph captures below pick their GEMM solutions
        self.tuned_gemms = bert.use_tuned_gemms()
        for _ in range(max(1, self.instance_count)):
            self._slots.append(self._make_slot(dev))
        self._free = list(range(len(self._slots)))

    def _build_model(self, bert, dev):
        return bert.build(device=dev, layers=self.layers)

    def _make_slot(self, dev):
        torch = self.torch
        from triton_client_amd.ops import hip

        n, s = self.max_batch_size, self.SEQ
        slot = {"stream": torch.cuda.Stream(device=dev), "graphs": {},
                "ins": [torch.zeros(n, s, device=dev, dtype=torch.int32) for _ in range(3)],
                "outs": [torch.zeros(n, s, device=dev, dtype=torch.float32) for _ in range(2)],
                "ev": [torch.cuda.Event(enable_timing=True) for _ in range(4)]}
        slot["ins"][1].fill_(1)
        slot["stage_host"] = hip.host_alloc(3 * n * s * 4)
        slot["out_host"] = hip.host_alloc(2 * n * s * 4)

        def run(b, dense=False):
            ids, mask, tt = (t[:b] for t in slot["ins"])
            # synthetic load generators send arbitrary INT32: keep indices in range
            # (an out-of-range embedding index is a device fault, not an error)
            st, en = self.model(ids.long().remainder(30522), mask.clamp(0, 1), tt.long().clamp(0, 1), dense=dense)
            slot["outs"][0][:b].copy_(st)
            slot["outs"][1][:b].copy_(en)

        slot["run"] = run
        # one graph per bucket with the key-padding mask, plus a "dense" one
        # without it from DENSE_FROM rows (no padding in any real row)
        with torch.cuda.stream(slot["stream"]), torch.no_grad():
            for b in self.BUCKETS:
                for dense in ((False, True) if b >= self.DENSE_FROM else (False,)):
                    run(b, dense)
                    if self.use_graphs:
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g, stream=slot["stream"]):
                            run(b, dense)
                        slot["graphs"][(b, dense)] = g
        slot["stream"].synchronize()
        return slot

    def unload(self):
        from triton_client_amd.ops import hip

        for sl in self._slots:
            for k in ("stage_host", "out_host"):
                try:
                    hip.host_free(sl[k])
                except Exception:
                    pass
        self._slots = []

    def _acquire(self):
        with self._cv:
            while not self._free:
                self._cv.wait()
            return self._free.pop()

    def _release(self, i):
        with self._cv:
            self._free.append(i)
            self._cv.notify()

    def _mask_all_ones(self, slot, parts, total):
        """True when every real row's attention_mask is >= 1 everywhere (the
        model clamps it to [0, 1]).  Host-staged parts are scanned in place;
        if any part came from device memory (HIP shm) the staged device rows
        are checked on the slot stream (one small reduction + sync)."""
        import ctypes

        on_device = False
        for kind, ptr, rows in parts:
            if kind == 1:
                on_device = True
                continue
            a = np.ctypeslib.as_array((ctypes.c_int32 * (rows * self.SEQ)).from_address(ptr))
            if a.min() < 1:
                return False
        if not on_device:
            return True
        torch = self.torch
        with torch.cuda.stream(slot["stream"]):
            return not bool((slot["ins"][1][:total] < 1).any().item())

    def _run_batch(self, slot, srcs, outs, total):
        """srcs: per input a list of (kind, ptr, rows) in row order; outs: per
        output a list of (kind, ptr, first_row, rows).  Returns timings (ns)."""
        import ctypes

        from triton_client_amd.ops import hip

        row = self.SEQ * 4
        bucket = next(b for b in self.BUCKETS if b >= total)
        stream = slot["stream"]
        sh = stream.cuda_stream
        ev = slot["ev"]
        ev[0].record(stream)
        for k, parts in enumerate(srcs):
            base = slot["ins"][k].data_ptr()
            c_src, c_dst, c_n = [], [], []
            host_off = 0
            first = 0
            stage = slot["stage_host"] + k * self.max_batch_size * row
            for kind, ptr, rows in parts:
                if kind == 1:
                    c_src.append(ptr)
                    c_dst.append(base + first * row)
                    c_n.append(rows * row)
                else:
                    ctypes.memmove(stage + host_off, ptr, rows * row)
                    hip.memcpy_async(base + first * row, stage + host_off, rows * row, sh)
                    host_off += rows * row
                first += rows
            if c_src:
                hip.batched_copy(c_src, c_dst, c_n, sh)
            if bucket > total:  # padding rows: keep them deterministic (mask 1, ids 0)
                hip.memset_async(base + total * row, 0, (bucket - total) * row, sh)
        dense = bucket >= self.DENSE_FROM and self._mask_all_ones(slot, srcs[1], total)
        ev[1].record(stream)
        with self.torch.cuda.stream(stream), self.torch.no_grad():
            if self.use_graphs:
                slot["graphs"][(bucket, dense)].replay()
            else:
                slot["run"](bucket, dense)
        ev[2].record(stream)
        host_outs = []
        for k, parts in enumerate(outs):
            base = slot["outs"][k].data_ptr()
            c_src, c_dst, c_n = [], [], []
            for kind, ptr, first, rows in parts:
                if not ptr:
                    continue
                if kind == 1:
                    c_src.append(base + first * row)
                    c_dst.append(ptr)
                    c_n.append(rows * row)
                else:
                    host_outs.append((k, ptr, first, rows))
            if c_src:
                hip.batched_copy(c_src, c_dst, c_n, sh)
        if host_outs:
            for k in range(2):
                hip.memcpy_async(slot["out_host"] + k * self.max_batch_size * row, slot["outs"][k].data_ptr(),
                                 total * row, sh)
        ev[3].record(stream)
        hip.stream_synchronize(sh)
        for k, ptr, first, rows in host_outs:
            ctypes.memmove(ptr, slot["out_host"] + k * self.max_batch_size * row + first * row, rows * row)
        return [int(ev[0].elapsed_time(ev[1]) * 1e6), int(ev[1].elapsed_time(ev[2]) * 1e6),
                int(ev[2].elapsed_time(ev[3]) * 1e6)]

    def execute_native(self, instance, b):
        total = int(b.total_rows)
        if total > self.max_batch_size:
            raise ServerError("batch of %d rows exceeds max_batch_size" % total)
        srcs = [[] for _ in range(3)]
        outs = [[] for _ in range(2)]
        first = 0
        for r in range(b.n_requests):
            rows = int(b.rows[r])
            for k in range(3):
                ref = b.inputs[r * b.n_inputs + k]
                srcs[k].append((ref.kind, ref.ptr, rows))
            for k in range(2):
                ref = b.outputs[r * b.n_outputs + k]
                outs[k].append((ref.kind, ref.ptr, first, rows))
            first += rows
        i = self._acquire()
        try:
            t = self._run_batch(self._slots[i], srcs, outs, total)
        finally:
            self._release(i)
        for k in range(3):
            b.timing_ns[k] = t[k]

    def execute(self, requests):
        import ctypes

        total = 0
        plan = []
        for r in requests:
            n = int(r.input("input_ids").shape[0])
            plan.append((r, total, n))
            total += n
        if total > self.max_batch_size:
            return [ServerError("batch of %d rows exceeds max_batch_size" % total)] * len(requests)
        names = [s.name for s in self.inputs]
        srcs = [[] for _ in range(3)]
        keep = []
        for r, first, n in plan:
            for k, nm in enumerate(names):
                t = r.input(nm)
                if isinstance(t.data, DeviceView):
                    srcs[k].append((1, t.data.ptr, n))
                else:
                    a = np.ascontiguousarray(t.data, dtype=np.int32)
                    keep.append(a)
                    srcs[k].append((0, a.ctypes.data, n))
        # outputs come back to host; shm targets are filled by the server (deliver_to_shm)
        res = np.empty((2, total, self.SEQ), dtype=np.float32)
        outs = [[(0, res[k].ctypes.data, 0, total)] for k in range(2)]
        i = self._acquire()
        try:
            t = self._run_batch(self._slots[i], srcs, outs, total)
        finally:
            self._release(i)
        if self._batch_stats is not None:
            self._batch_stats(total, len(requests), *t)
        del ctypes
        return [[OutputTensor("start_logits", "FP32", [n, self.SEQ], res[0, f:f + n]),
                 OutputTensor("end_logits", "FP32", [n, self.SEQ], res[1, f:f + n])] for _, f, n in plan]

    _batch_stats = None
    reports_batch_stats = True


class BertLargeFP32(BertLarge):
    """``bert_large_fp32`` — the same BERT-large QA model (same seed, same
    inputs and outputs) with fp32-parity compute, the way densenet_onnx has
    one: fp32 weights and activations, every projection one bf16x3 GEMM on
    the bf16 MFMA (models/bert.py prepare_x3: x_hi W_hi + x_hi W_lo + x_lo W_hi,
    fp32 accumulate), LayerNorm / GELU / softmax attention in fp32.  Served
    logits match an fp32 forward of the fp32 weights to ~1e-5
    (tests/test_bert_accuracy_gpu.py); ~3x the bf16 model's GEMM work.  The
    bf16 ``bert_large`` stays the config-4 serving default."""

    name = "bert_large_fp32"
    # 64 rows, as before bert_large went to 128: a bs128 fp32-parity forward
    # (~110 ms) outlasts the sweep's queue delay, so c256 ran partial 88-row
    # batches at 1,142 infer/s against 1,200 with 64-row ones
    # (profiles/r6_bert_batching/)
    max_batch_size = 64
    BUCKETS = tuple(b for b in BertLarge.BUCKETS if b <= 64)

    def _build_model(self, bert, dev):
        import torch

        return bert.prepare_x3(bert.build(device=dev, dtype=torch.float32, layers=self.layers))


GPU_MODELS = [DensenetOnnx, PreprocessInceptionEnsemble, BertLarge]
# loaded only when --models names them: bert_large_fp32 adds ~2 GB of bf16x3
# weights and 28 captured HIP graphs per instance (round-5 advisor finding)
OPT_IN_GPU_MODELS = [BertLargeFP32]
