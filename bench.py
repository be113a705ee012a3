#!/usr/bin/env python3
"""Flagship serving benchmark (BASELINE.json metric): perf_analyzer-style
inferences/sec + p99 latency for ``densenet_onnx`` at bs=8 and bs=1 over gRPC
with HIP shared memory, FP32 in / FP32 out / fp32-parity compute.

One process per GPU.  ``python bench.py --gpus N`` with no ``WORLD_SIZE`` in
the environment starts ``torch.distributed.run`` with N ranks as a CHILD
process (this process never touches the GPU) and exits with its code; under
``torch.distributed.run`` (the driver's N>1 launch) each rank:

  * spawns the KServe-v2 bench server pinned to its GPU (child process: HIP
    IPC needs two processes) with the fp32-parity DenseNet engine
    (models/densenet_fp32.py, split-precision bf16x3 MFMA kernels);
  * allocates a HIP shm input region; rank 0 fills it with K1 Philox normal
    data on its GPU and RCCL-broadcasts it into every rank's region (X1;
    ``--fanout p2p`` = the xGMI peer-copy star X2), replicas verified;
  * drives the native C++ load generator (csrc/cpp/perf, in-process through
    ctypes, no Python on the request path) with ``concurrency`` requests in
    flight against its own server.

A "step" is one perf_analyzer count window: ``--window`` x concurrency
requests of ``--batch`` images.  W warmup steps, then EXACTLY K timed steps
as ONE continuous closed-loop run between barrier + device sync; the K
windows are cut from the requests' completion times (no drain between
windows), and the run is "stable" when the 3 windows before the last (which
holds the final drain) are within 10% of their mean (perf_analyzer's rule).  value = total
images/s over all ranks (elapsed = MAX over ranks); p50/p90/p99 over every
rank's requests.  After the timed bs=8 region: a bs=1 point (HIP shm, same
server) and, unless ``--no-bf16`` (or on more than one GPU), the bf16 engine as a labelled
reduced-precision operating point.

``--cpu`` runs the same pipeline with no GPU (CPU ``frontend_sink`` model,
system shm, gloo): the multi-rank CPU test of the launch/aggregation path.

``--model bert_large`` is BASELINE.json's concurrency-sweep config instead
(bert-large seq 384, HIP shm fanned out over RCCL): the three INT32 input
regions are filled on rank 0 (K1: random token ids, all-ones mask, zero
segment ids) and broadcast to every rank, then each rank sweeps
``--sweep`` concurrencies against its own server; per point ``--steps``
windows of max(64, 8 x concurrency) requests, aggregated over ranks.  The
JSON ``value`` is the aggregate infer/s at the highest concurrency; every
point is listed under ``sweep``.  (``--cpu`` covers it on the CPU with the
``bert_sink`` shape model.)
"""

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "perf_analyzer inferences/sec + p99 latency, densenet_onnx bs=1/8 via HIP shm"
BERT_METRIC = "perf_analyzer concurrency sweep 1-256 inferences/sec + p99 latency, bert_large seq384 via HIP shm"


def log(*a):
    print("[bench rank %s]" % os.environ.get("RANK", "0"), *a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="images per request (densenet_onnx bs)")
    ap.add_argument("--concurrency", type=int, default=48, help="requests in flight per GPU")
    ap.add_argument("--window", type=int, default=16, help="requests per step = window x concurrency")
    ap.add_argument("--bs1-concurrency", type=int, default=64)
    ap.add_argument("--lanes", type=int, default=1,
                    help="client lanes (connection + worker thread each) sharing the headline concurrency")
    ap.add_argument("--bs1-preferred", default="auto",
                    help="preferred batch rows for the bs=1 point (comma list; auto = bs1 concurrency / instances; "
                         "none = keep the headline's), set on the loaded model through the repository API's config "
                         "override before that point: c64 on 2 instances 23.6k -> 26.3k infer/s, p99 3.5 -> 3.2 ms "
                         "(profiles/r6_bench/bs1_preferred_ab.md)")
    ap.add_argument("--bs1-lanes", type=int, default=2,
                    help="client lanes (connection + worker thread each) sharing the bs=1 concurrency; with the "
                         "preferred size at rows per instance, 2 lanes return each 32-row group fast enough that every "
                         "batch is full: c64 25.3-26.8k -> 28.6-29.2k infer/s, p99 3.1-3.4 -> 2.3-2.4 ms "
                         "(profiles/r6_bench/bs1_preferred_ab.md)")
    ap.add_argument("--fanout", default="rccl", choices=["rccl", "p2p", "local"])
    ap.add_argument("--fanout-fallback", default="none", choices=["none", "local"],
                    help="none (default): a failed RCCL broadcast ends the run non-zero with the error; "
                         "local: ranks agree over a gloo control group and refill locally (labelled)")
    ap.add_argument("--engine", default="fp32", choices=["fp32", "fused", "torch"],
                    help="densenet_onnx engine for the headline (fp32 = fp32-parity split-precision kernels)")
    ap.add_argument("--no-bf16", action="store_true", help="skip the bf16-engine secondary measurement")
    ap.add_argument("--same-input", action="store_true",
                    help="every request reads the same bs images (default: each concurrency slot has its own "
                         "images and output slice, and every slot's output is checked after the run)")
    # 2 instances (2 HIP streams): full 128-row batches on two overlapping
    # streams beat 4 instances' ~110-row batches on four (one box: 42.1k infer/s
    # p99 9.7 ms vs 40.5k p99 11.5 ms; the engine alone at bs128 makes 42.0k img/s
    # on 2 streams, 40.9k on 4: profiles/r3_instances.md)
    ap.add_argument("--instance-count", type=int, default=2)
    ap.add_argument("--max-queue-delay-us", type=int, default=2000)
    ap.add_argument("--max-batch-size", type=int, default=0)
    ap.add_argument("--preferred", default="128")
    ap.add_argument("--idle-dispatch", default="on", choices=["on", "off"])
    ap.add_argument("--cpu", action="store_true", help="no GPU: CPU frontend_sink model, system shm, gloo")
    ap.add_argument("--rehearse", action="store_true",
                    help="one-GPU rehearsal of the N-GPU launch: every rank (and its server) on GPU 0, gloo "
                         "process group, p2p/host fan-out (RCCL cannot put two ranks on one device)")
    ap.add_argument("--pin", default="auto", choices=["auto", "on", "off"],
                    help="pin each rank (server child + load generator threads) to CPUs of its GPU's NUMA node "
                         "(auto: when more than one rank runs on this host)")
    ap.add_argument("--server-log", default="")
    ap.add_argument("--model", default="densenet_onnx", choices=["densenet_onnx", "bert_large"])
    ap.add_argument("--sweep", default="1,4,16,64,256", help="bert_large: concurrencies per GPU")
    ap.add_argument("--bert-preferred-from", type=int, default=2,
                    help="bert_large sweep: rows per instance from which --bert-preferred auto applies")
    ap.add_argument("--bert-lanes", type=int, default=1,
                    help="bert_large sweep: client lanes per point (from 8 requests per lane)")
    ap.add_argument("--bert-preferred", default="auto", choices=["auto", "none"],
                    help="bert_large sweep: per point, the batcher's preferred size = concurrency / instances (capped "
                         "at the model's max batch; a repository config override, as for the bs=1 point); none = the "
                         "model's own setting for every point")
    ap.add_argument("--bert-instance-count", type=int, default=2)
    ap.add_argument("--bert-queue-delay-us", type=int, default=500)
    ap.add_argument("--loop-timeout", type=float, default=600.0,
                    help="seconds a timed loop may wait for its requests before the run fails (server stacks dumped)")
    ap.add_argument("--bert-precision", default="bf16", choices=["bf16", "fp32"],
                    help="bert_large: bf16 (the config-4 default) or fp32 parity (serves bert_large_fp32: bf16x3 "
                         "projections on the hand-written GEMMs, fp32 LayerNorm / attention)")
    return ap.parse_args(argv)


def spawn_ranks(args):
    """Parent of a multi-GPU run: torch.distributed.run as a child process."""
    from triton_client_amd.perf.harness import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    log("spawning %d ranks: %s" % (args.gpus, " ".join(cmd)))
    return subprocess.call(cmd, env=env)


def bs1_preferred_rows(spec, concurrency, instances):
    """--bs1-preferred: "auto" = one full group per instance (concurrency /
    instances, when it divides), "none"/"" = keep the headline's setting, else
    the comma list given.  Returns the list or None."""
    if spec == "auto":
        n = max(1, instances)
        return [concurrency // n] if concurrency >= n and concurrency % n == 0 else None
    if spec in ("", "none"):
        return None
    return [int(x) for x in spec.split(",")]


def bert_point_preferred(mode, concurrency, instances, from_rows, max_batch=64):
    """Preferred batch rows of one bert sweep point (--bert-preferred auto):
    concurrency / instances, capped at the model's max batch, from
    ``from_rows`` rows per instance; None otherwise."""
    n = max(1, instances)
    if mode != "auto" or concurrency % n or concurrency < max(1, from_rows) * n:
        return None
    return min(max_batch, concurrency // n)


class Point:
    """One load point of the native engine against one server."""

    def __init__(self, srv, model, bs, conc, region, nbytes, device, cpu, inputs=None, out_bytes=None, outputs=None):
        from triton_client_amd.perf.native import PerfSession

        self.bs, self.conc = bs, conc
        out_bytes = out_bytes or bs * 1000 * 4
        args = ["-m", model, "-i", "grpc", "-u", srv.grpc_url, "-b", bs,
                "--shared-memory", "system" if cpu else "hip", "--device", device,
                "--output-shared-memory-size", out_bytes, "--concurrency-range", conc]
        # a list value pins entry s % n to concurrency slot s (REGION@OFFSET slices)
        for name, reg in (inputs or {"data_0": region}).items():
            args += ["--shared-memory-input", "%s=%s" % (name, ",".join(reg) if isinstance(reg, list) else reg)]
        for name, reg in (outputs or {}).items():
            args += ["--shared-memory-output", "%s=%s" % (name, ",".join(reg) if isinstance(reg, list) else reg)]
        self.s = PerfSession(args)

    def run(self, n):
        return self.s.run_timed(self.conc, n)

    # ---- continuous closed loop (measure): no restart between warm-up and timing ----
    def start(self):
        self.s.loop_start(self.conc)

    def marks(self):
        return [self.s.loop_count()]

    timeout_s = 600.0

    def wait_after(self, marks, n):
        self.s.loop_wait(marks[0][0] + n, timeout_s=self.timeout_s, log=log)

    def take(self, marks, n, t0_ns):
        """The first n requests completed after ``marks``: latencies (ns) and
        completion times (ns after t0_ns on the engine clock), completion order."""
        st, en, ok = self.s.loop_records(marks[0][0], n)
        if len(en) < n or not ok.all():
            raise RuntimeError("the loop lost requests (%d of %d, %d failed)" % (len(en), n, int((ok == 0).sum())))
        return en - st, en.astype("int64") - int(t0_ns)

    def stop(self):
        self.s.loop_stop()

    def close(self):
        self.s.close()


class Lanes:
    """`sum(conc)` requests in flight over several client lanes against one
    server: each lane is its own Point (gRPC connection, I/O thread, engine
    worker thread), the way perf_analyzer spreads a concurrency over its worker
    threads.  run(n) runs n / lanes requests on every lane at once."""

    def __init__(self, points):
        self.points = points
        self.conc = sum(p.conc for p in points)
        self.s = points[0].s  # server statistics are per model, any lane reads them

    def run(self, n):
        """Per-request latencies and completion times of all lanes on ONE
        clock: each lane's end_ns counts from its own run's start, so every
        lane's times are shifted to the earliest lane start (a lane's start =
        its return time minus its elapsed run time) before they are merged --
        the window statistics sort them as one timeline."""
        import threading
        import time

        import numpy as np

        k = len(self.points)
        out = [None] * k
        back = [0] * k
        errs = []

        def go(i):
            try:
                out[i] = self.points[i].run(n // k)
                back[i] = time.perf_counter_ns()
            except Exception as e:  # noqa: BLE001 -- re-raised below
                errs.append(e)

        th = [threading.Thread(target=go, args=(i,)) for i in range(k)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]
        return merge_lanes(out, back)

    # ---- continuous closed loop: every lane at once ----
    def start(self):
        for p in self.points:
            p.start()

    def marks(self):
        return [p.s.loop_count() for p in self.points]

    def wait_after(self, marks, n):
        k = len(self.points)
        for p, m in zip(self.points, marks):  # equal concurrency per lane: each takes its share
            p.s.loop_wait(m[0] + -(-n // k), timeout_s=p.timeout_s, log=log)

    def take(self, marks, n, t0_ns):
        """All lanes' completions since ``marks`` merged on the engine clock
        (one steady clock in this process); the first n by completion time."""
        import numpy as np

        lat, end = [], []
        for p, m in zip(self.points, marks):
            cnt, _ = p.s.loop_count()
            st, en, ok = p.s.loop_records(m[0], cnt - m[0])
            if not ok.all():
                raise RuntimeError("a lane's loop had failed requests")
            lat.append(en - st)
            end.append(en.astype(np.int64) - int(t0_ns))
        lat, end = np.concatenate(lat), np.concatenate(end)
        if len(end) < n:
            raise RuntimeError("the lanes completed %d of %d requests" % (len(end), n))
        order = np.argsort(end, kind="stable")[:n]
        return lat[order], end[order]

    def stop(self):
        for p in self.points:
            p.stop()

    def close(self):
        for p in self.points:
            p.close()


def merge_lanes(out, back_ns):
    """Lane results [(lat_ns, end_ns, elapsed_s)] and each lane's return time
    (perf_counter ns) -> one (lat_ns, end_ns, elapsed_s) with every end_ns on
    the clock of the earliest-starting lane."""
    import numpy as np

    starts = [b - int(o[2] * 1e9) for o, b in zip(out, back_ns)]
    t0 = min(starts)
    ends = [o[1].astype(np.int64) + (st - t0) for o, st in zip(out, starts)]
    span = max(b - t0 for b in back_ns) * 1e-9
    return np.concatenate([o[0] for o in out]), np.concatenate(ends).astype(np.uint64), span


def windows(end_ns, per, k):
    """Throughputs (requests/s) of k back-to-back windows of `per` requests."""
    import numpy as np

    e = np.sort(end_ns.astype(np.float64))
    out, t_prev = [], 0.0
    for i in range(k):
        t = e[min(len(e), (i + 1) * per) - 1]
        out.append(per / max((t - t_prev) * 1e-9, 1e-9))
        t_prev = t
    return out


def window_percentiles(lat_ns, end_ns, per, k):
    """p50 and p99 (us) of the requests that completed in each of the k
    windows of `per` requests (completion order, as :func:`windows`)."""
    import numpy as np

    from triton_client_amd.perf.loadgen import percentile_us

    order = np.argsort(end_ns, kind="stable")
    lat = lat_ns.astype(np.float64)[order]
    p50, p99 = [], []
    for i in range(k):
        w = lat[i * per:(i + 1) * per]
        if len(w) == 0:
            break
        p50.append(round(percentile_us(w, 50), 1))
        p99.append(round(percentile_us(w, 99), 1))
    return p50, p99


def stats_delta(a, b):
    d = {k: b[k] - a[k] for k in a}
    execs = max(d["execution_count"], 1)
    reqs = max(d["success_count"], 1)
    return {
        "avg_rows_per_batch": round(d["inference_count"] / execs, 2),
        "queue_us_per_request": round(d["queue_ns"] / reqs / 1e3, 1),
        "compute_input_us_per_batch": round(d["compute_input_ns"] / execs / 1e3, 1),
        "compute_infer_us_per_batch": round(d["compute_infer_ns"] / execs / 1e3, 1),
        "compute_output_us_per_batch": round(d["compute_output_ns"] / execs / 1e3, 1),
        "server_us_per_request": round(d["success_ns"] / reqs / 1e3, 1),
    }


def batch_stats(client, model):
    """Per batch size: (executions, compute_input_ns, compute_infer_ns, compute_output_ns)."""
    st = client.get_inference_statistics(model, as_json=True)
    out = {}
    for m in st.get("model_stats", []):
        for b in m.get("batch_stats", []):
            bs = int(b["batch_size"])
            cnt = int(b.get("compute_infer", {}).get("count", 0))
            ns = [int(b.get(k, {}).get("ns", 0)) for k in ("compute_input", "compute_infer", "compute_output")]
            c0, i0, f0, o0 = out.get(bs, (0, 0, 0, 0))
            out[bs] = (c0 + cnt, i0 + ns[0], f0 + ns[1], o0 + ns[2])
    return out


def weighted_compute_us(a, b, rows_per_request):
    """Request-weighted device time of the batches between two batch_stats
    snapshots: a request of a 128-row batch waits for that batch's whole
    execution, so per-request server time must be compared with batch times
    weighted by the requests they carry, not with the plain per-batch mean
    (large batches run longer and carry more requests)."""
    num = den = 0.0
    for bs, (c1, i1, f1, o1) in b.items():
        c0, i0, f0, o0 = a.get(bs, (0, 0, 0, 0))
        reqs = max(bs / float(rows_per_request), 1.0)
        num += reqs * ((i1 - i0) + (f1 - f0) + (o1 - o0))
        den += reqs * (c1 - c0)
    return num / den / 1e3 if den else 0.0


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    rehearse = args.rehearse and world > 1
    # the GPU this rank drives (and its server runs on)
    dev = 0 if args.rehearse else local_rank
    if rehearse and args.fanout == "rccl":
        args.fanout = "p2p"
    if world != args.gpus:
        raise SystemExit("WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

    import numpy as np

    from triton_client_amd.perf.harness import ServerProcess
    from triton_client_amd.perf.loadgen import percentile_us

    cpu = args.cpu
    Point.timeout_s = args.loop_timeout
    bert = args.model == "bert_large"
    if bert:
        model = "bert_sink" if cpu else ("bert_large_fp32" if args.bert_precision == "fp32" else "bert_large")
    else:
        model = "frontend_sink" if cpu else "densenet_onnx"
    bs, conc = args.batch, args.concurrency
    log_dir = os.path.join(REPO, "gpurun_out")
    os.makedirs(log_dir, exist_ok=True)

    # host placement BEFORE the server is spawned (the child inherits it): the
    # CPUs of this rank's GPU's NUMA node, split among the ranks sharing it
    from triton_client_amd.parallel import placement

    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    place = placement.plan(dev if args.rehearse else local_rank, 1 if args.rehearse else local_world)
    if args.pin == "on" or (args.pin == "auto" and local_world > 1 and not args.rehearse):
        place = placement.apply(place)
    else:
        place["applied"] = False
    place.pop("cpus", None)
    log("placement: %s" % place)

    def start_server(engine, tag):
        if bert:
            extra = ["--instance-count", str(args.bert_instance_count), "--max-queue-delay-us",
                     str(args.bert_queue_delay_us)]
        else:
            extra = ["--instance-count", str(args.instance_count), "--max-queue-delay-us",
                     str(args.max_queue_delay_us), "--idle-dispatch", args.idle_dispatch]
        if not cpu and not bert:
            extra += ["--engine", engine]
            if args.preferred:
                extra += ["--preferred-batch-sizes", args.preferred]
            if args.max_batch_size:
                extra += ["--max-batch-size", str(args.max_batch_size)]
        path = args.server_log or os.path.join(log_dir, "bench_server_%s_r%d.log" % (tag, rank))
        # spawned before this process touches the GPU; per-rank port stripes
        return ServerProcess(device=dev, gpu=not cpu, models=model, extra_args=extra, log_path=path,
                             port_stripe=local_rank if world > 1 else None), path

    srv, srv_log = start_server(args.engine, "bert" if bert else args.engine)
    place["grpc_port"] = srv.grpc_port

    import torch
    import torch.distributed as dist

    if not cpu:
        torch.cuda.set_device(dev)
    if world > 1:
        if cpu or rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        from triton_client_amd.parallel import fanout as _fo

        _fo.cpu_group()  # the gloo control group (collective creation: every rank, now)

    import tritonclient.grpc as grpcclient
    from triton_client_amd.parallel import fanout

    if cpu:
        from tritonclient.utils import shared_memory as shmod
    else:
        from tritonclient.utils import hip_shared_memory as shmod

    regions, points = [], []
    state = {"client": None}

    def make_input(name, n_img):
        """Input region of n_img images, filled on rank 0 and fanned out."""
        elems = n_img * 3 * 224 * 224
        nbytes = elems * 4
        if cpu:
            key = "/%s_r%d_%d" % (name, rank, os.getpid())
            r = shmod.create_shared_memory_region(name, key, nbytes)
            regions.append(r)
            data = np.random.default_rng(1234).standard_normal(elems, dtype=np.float32) if rank == 0 \
                else np.zeros(elems, np.float32)
            host = data.view(np.uint8)
            method = fanout.fanout_host(host)
            shmod.set_shared_memory_region(r, [host.view(np.float32)])
            if not fanout.verify_host_replicas(host):
                raise RuntimeError("fan-out replicas differ across ranks")
            state["client"].register_system_shared_memory(name, key, nbytes)
        else:
            r = shmod.create_shared_memory_region(name, nbytes, dev)
            regions.append(r)
            method = fanout.fill_and_fanout(r, "FP32", elems, seed=1234, mode="normal", lo=0.0, hi=1.0,
                                            method=args.fanout, fallback=args.fanout_fallback)
            if not fanout.verify_replicas(r, nbytes, over_cpu=method == fanout.LOCAL_FALLBACK):
                raise RuntimeError("fan-out replicas differ across ranks")
            state["client"].register_cuda_shared_memory(name, shmod.get_raw_handle(r), dev, nbytes)
        return method, nbytes

    def measure(point, warm_n, steps, per, snap=None):
        """One continuous closed loop: `warm_n` untimed warm-up requests, then
        EXACTLY `steps` windows of `per` requests between barrier + sync, in
        the SAME loop (no restart, so the timed windows start in steady state
        instead of with a refilling pipeline; round 5's first window carried
        that refill's tail).  `snap()` (server statistics) is read right
        before the timed start and right after the last timed completion.
        Returns latencies, completion times (ns after the timed start),
        elapsed (max over ranks) and the two snapshots."""
        point.start()
        try:
            return _measure(point, warm_n, steps, per, snap)
        except Exception:
            log("timed loop failed: asking the server for its thread stacks (log %s)" % srv_log)
            try:
                srv.dump_stacks()
            except Exception as e:  # noqa: BLE001
                log("stack dump failed: %s" % e)
            raise
        finally:
            try:
                point.stop()
            except Exception as e:  # noqa: BLE001 -- the loop's own error is the one to report
                log("loop stop: %s -- asking the server for its thread stacks" % e)
                try:
                    srv.dump_stacks()
                except Exception as e2:  # noqa: BLE001
                    log("stack dump failed: %s" % e2)

    def _measure(point, warm_n, steps, per, snap):
        point.wait_after(point.marks(), warm_n)
        s0 = snap() if snap else None  # outside the timed windows: its RPC would ride in window 0
        if world > 1:
            fanout.barrier()
        if not cpu:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = point.marks()
        point.wait_after(m, steps * per)
        s1 = snap() if snap else None
        if not cpu:
            torch.cuda.synchronize()
        if world > 1:
            fanout.barrier()
        elapsed = time.perf_counter() - t0
        lat, end = point.take(m, steps * per, m[0][1])
        return lat, end, fanout.max_over_ranks(elapsed), (s0, s1)

    try:
        log("waiting for server (log %s)" % srv_log)
        srv.wait_ready(timeout=1500, model=model)
        log("server ready")
        client = grpcclient.InferenceServerClient(srv.grpc_url)
        state["client"] = client
        if bert:
            return bert_sweep(args, srv, model, client, shmod, regions, points, measure, fanout, rank, world,
                              dev, cpu)
        # one region of `nslots` x bs distinct images (one fan-out); concurrency
        # slot s reads slice s and writes output slice s, so a batch of 16
        # requests mixes 16 different inputs and a row mix-up is visible below
        nslots = 1 if args.same_input else conc
        req_bytes = bs * 3 * 224 * 224 * 4
        method, in_total = make_input("data_0_in", bs * nslots)
        in_bytes = req_bytes
        in_list = ["data_0_in@%d" % (i * req_bytes) for i in range(nslots)] if nslots > 1 else "data_0_in"
        out_list = None
        if not cpu:
            ob = bs * 1000 * 4
            ro = shmod.create_shared_memory_region("fc6_1_out", nslots * ob, dev)
            regions.append(ro)
            client.register_cuda_shared_memory("fc6_1_out", shmod.get_raw_handle(ro), dev, nslots * ob)
            out_list = ["fc6_1_out@%d" % (i * ob) for i in range(nslots)]

        def slots(c, lo=0):
            return {"data_0": in_list[lo:c] if isinstance(in_list, list) else in_list}, \
                ({"fc6_1": out_list[lo:c]} if out_list else None)

        fan = {"method": method, "replicas_verified": True, "bytes": in_total}
        if not cpu and world > 1:
            # X1 (RCCL broadcast) vs X2 (xGMI one-hop star), once, on the headline input
            # region; a rehearsal on one GPU times p2p and host staging
            fan["timings"] = fanout.time_fanout(
                regions[0], in_total, ["p2p", "host"] if rehearse else
                (["p2p"] if method == fanout.LOCAL_FALLBACK else ["rccl", "p2p"]))
            fan["errors"] = fanout.fanout_errors(fan["timings"])
            if not fanout.verify_replicas(regions[0], in_total, over_cpu=method == fanout.LOCAL_FALLBACK):
                raise RuntimeError("fan-out replicas differ across ranks after the fan-out timing")
            t_used = fan["timings"].get(method, {})
            if "us" in t_used:
                fan["fanout_us"] = t_used["us"]
            log("fan-out timings: %s" % fan["timings"])
        if not cpu:
            _sanity_check(client, shmod, bs, dev, regions)

        # ---- headline: bs=8 -------------------------------------------------------
        per = args.window * conc
        nl8 = max(1, args.lanes)
        if conc % nl8 or per % nl8:
            raise SystemExit("--concurrency (and window x concurrency) must be a multiple of --lanes")
        # lane i drives concurrency slots [i c / n, (i + 1) c / n): its own connection and worker thread
        lanes8 = []
        for i in range(nl8):
            ins, outs = slots((i + 1) * conc // nl8, i * conc // nl8)
            lanes8.append(Point(srv, model, bs, conc // nl8, None, in_bytes, dev, cpu, inputs=ins, outputs=outs))
        p8 = Lanes(lanes8)
        points.extend(lanes8)
        lat, end, elapsed, ((st0, bst0), (st1, bst1)) = measure(
            p8, max(args.warmup, 1) * per, args.steps, per,
            snap=lambda: (p8.s.server_stats(), batch_stats(client, model)))
        wins = windows(end, per, args.steps)
        # the last window holds the closed loop's drain (no new issues), so the
        # stability rule looks at the three windows before it
        last3 = wins[-4:-1] if len(wins) >= 4 else wins[-3:]
        mean3 = sum(last3) / len(last3)
        stable = all(abs(w - mean3) <= 0.10 * mean3 for w in last3)
        all_lat = fanout.gather_arrays(lat.astype(np.int64)).astype(np.float64)
        # per-window p50 / p99 (rank 0, requests binned by completion time into
        # the same windows as the throughputs): a wide tail is then visible as
        # one bad window or as the whole run
        win_p = window_percentiles(lat, end, per, args.steps)
        value = world * args.steps * per * bs / elapsed
        breakdown = stats_delta(st0, st1)
        breakdown["client_overhead_us_per_request"] = round(
            float(np.mean(lat)) / 1e3 - breakdown["server_us_per_request"], 1)
        # per-request accounting: queue + the request-weighted device time of
        # the batch it rode in; what is left is host time nobody timed
        wc = weighted_compute_us(bst0, bst1, bs)
        breakdown["compute_us_per_request_weighted"] = round(wc, 1)
        breakdown["unattributed_us_per_request"] = round(
            breakdown["server_us_per_request"] - breakdown["queue_us_per_request"] - wc, 1)
        # every slot's output slice must be the logits of ITS images (checked
        # against the same server running that request alone, outside the timing)
        slot_check = None if (cpu or out_list is None) else _verify_slots(client, shmod, regions, nslots, bs, dev)

        # ---- best throughput with p99 <= 10 ms (same server, lower concurrency) ---------
        p99c = {"p99_target_us": 10000.0, "points": [
            {"concurrency": args.concurrency, "infer_per_sec": round(value, 1),
             "p50_latency_us": round(percentile_us(all_lat, 50), 1),
             "p99_latency_us": round(percentile_us(all_lat, 99), 1)}]}
        if not cpu:
            for c in (32, 24, 16):
                ins_c, outs_c = slots(c)
                pc = Point(srv, model, bs, c, None, in_bytes, dev, cpu, inputs=ins_c, outputs=outs_c)
                points.append(pc)
                perc = 16 * c
                lc_, _, elc, ((sp0, bp0), (sp1, bp1)) = measure(
                    pc, perc, 4, perc, snap=lambda: (pc.s.server_stats(), batch_stats(client, model)))
                lg = fanout.gather_arrays(lc_.astype(np.int64)).astype(np.float64)
                row = {"concurrency": c, "infer_per_sec": round(world * 4 * perc * bs / elc, 1),
                       "p50_latency_us": round(percentile_us(lg, 50), 1),
                       "p99_latency_us": round(percentile_us(lg, 99), 1)}
                # why a probe lands where it does: rows per executed batch
                # (how the c x bs rows in flight split into batches over the
                # instances), queueing and device time per batch (rank 0)
                bdp = stats_delta(sp0, sp1)
                bdp["batch_rows_histogram"] = {str(k): int(bp1[k][0] - bp0.get(k, (0,))[0]) for k in sorted(bp1)
                                               if bp1[k][0] - bp0.get(k, (0,))[0] > 0}
                row["breakdown_rank0"] = bdp
                p99c["points"].append(row)
                log("p99-constrained probe c%d: %.0f infer/s p99 %.0f us" % (c, row["infer_per_sec"],
                                                                             row["p99_latency_us"]))
            ok = [r for r in p99c["points"] if r["p99_latency_us"] <= p99c["p99_target_us"]]
            if ok:
                best = max(ok, key=lambda r: r["infer_per_sec"])
                p99c.update({"concurrency": best["concurrency"], "infer_per_sec": best["infer_per_sec"],
                             "p99_latency_us": best["p99_latency_us"]})

        # ---- bs=1 on the same server -------------------------------------------------
        bs1_rows = bs1_preferred_rows(args.bs1_preferred, args.bs1_concurrency, args.instance_count)
        if bs1_rows and not cpu:
            # a deployment tuned for this load: the batcher's preferred size
            # (Triton's dynamic_batching.preferred_batch_size) = the closed
            # loop's rows per instance, so the loop settles into one full group
            # per instance instead of ~3 groups of ~21 rows; applied to the
            # loaded model by a repository load with a config override
            client.load_model(model, config=json.dumps({"dynamic_batching": {"preferred_batch_size": bs1_rows}}))
            log("bs=1 point: preferred batch rows %s" % bs1_rows)
        _, in1 = make_input("data_1_in", 1)
        nl = max(1, args.bs1_lanes)
        if args.bs1_concurrency % nl:
            raise SystemExit("--bs1-concurrency must be a multiple of --bs1-lanes")
        p1 = Lanes([Point(srv, model, 1, args.bs1_concurrency // nl, "data_1_in", in1, dev, cpu) for _ in range(nl)])
        points.extend(p1.points)
        n1 = 64 * args.bs1_concurrency  # ~0.2 s at 20k infer/s: the batch groups of a closed loop need time to settle
        l1, e1, el1, ((s10, b10), (s11, b11)) = measure(
            p1, n1 // 4, 4, n1 // 4, snap=lambda: (p1.s.server_stats(), batch_stats(client, model)))
        bs1 = {"concurrency": args.bs1_concurrency, "client_lanes": nl, "infer_per_sec": round(world * n1 / el1, 1),
               "preferred_batch_rows": args.preferred if cpu or not bs1_rows else ",".join(map(str, bs1_rows))}
        # where a bs=1 request's latency goes at this concurrency: rows per
        # batch, queueing, and the request-weighted device time of its batch
        bd64 = stats_delta(s10, s11)
        bd64["client_overhead_us_per_request"] = round(float(np.mean(l1)) / 1e3 - bd64["server_us_per_request"], 1)
        wc1 = weighted_compute_us(b10, b11, 1)
        bd64["compute_us_per_request_weighted"] = round(wc1, 1)
        bd64["unattributed_us_per_request"] = round(
            bd64["server_us_per_request"] - bd64["queue_us_per_request"] - wc1, 1)
        # executed batches by rows (a closed loop of 64 settles into groups: ~2 of ~32 or ~3 of ~21)
        bd64["batch_rows_histogram"] = {str(k): int(b11[k][0] - b10.get(k, (0,))[0]) for k in sorted(b11)
                                        if b11[k][0] - b10.get(k, (0,))[0] > 0}
        bs1["breakdown_rank0"] = bd64
        l1g = fanout.gather_arrays(l1.astype(np.int64)).astype(np.float64)
        bs1.update({"p50_latency_us": round(percentile_us(l1g, 50), 1),
                    "p99_latency_us": round(percentile_us(l1g, 99), 1)})
        pc1 = Point(srv, model, 1, 1, "data_1_in", in1, dev, cpu)
        points.append(pc1)
        pc1.run(20)
        sc0 = pc1.s.server_stats()
        lc, _, _ = pc1.run(200)
        sc1 = pc1.s.server_stats()
        lcg = fanout.gather_arrays(lc.astype(np.int64)).astype(np.float64)
        bs1["concurrency1_p50_latency_us"] = round(percentile_us(lcg, 50), 1)
        bs1["concurrency1_p99_latency_us"] = round(percentile_us(lcg, 99), 1)
        # where one bs=1 request's latency goes (server-stat deltas over the 200 requests)
        bd1 = stats_delta(sc0, sc1)
        bd1["client_overhead_us_per_request"] = round(float(np.mean(lc)) / 1e3 - bd1["server_us_per_request"], 1)
        bs1["concurrency1_breakdown_rank0"] = bd1

        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "infer/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if (cpu or args.engine == "fp32") else "bf16",
            "data": ("synthetic (host normal, fanned out by %s), no model weights (CPU frontend_sink)" % method if cpu
                     else "synthetic (K1 Philox normal on device: %d distinct images, %d per concurrency slot, "
                          "fanned out by %s), random-init weights" % (nslots * bs, bs, method)),
            "config": {
                "model": model,
                "global_batch": world * conc * bs,
                "seq_len": None,
                "parallelism": "dp%d" % world,
                "batch_size": bs,
                "concurrency_per_gpu": conc,
                "protocol": "grpc",
                "shared_memory": "system" if cpu else "hip",
                "engine": args.engine,
                "compute": ("split-precision bf16x3 MFMA, fp32 accumulate (rel-L2 vs fp32 module ~4e-5)"
                            if args.engine == "fp32" else args.engine),
                "loadgen": "native C++ (csrc/cpp/perf)", "client_lanes": args.lanes,
                "server_instances": args.instance_count,
                "preferred_batch_rows": args.preferred,
                "max_queue_delay_us": args.max_queue_delay_us,
                "requests_per_step": per,
            },
            "p50_latency_us": round(percentile_us(all_lat, 50), 1),
            "p90_latency_us": round(percentile_us(all_lat, 90), 1),
            "p99_latency_us": round(percentile_us(all_lat, 99), 1),
            "stable": bool(fanout.max_over_ranks(0.0 if stable else 1.0) == 0.0),
            "window_infer_per_sec_rank0": [round(w * bs, 1) for w in wins],
            "window_p50_latency_us_rank0": win_p[0],
            "window_p99_latency_us_rank0": win_p[1],
            "placement": fanout.gather_objects(place),
            "server_breakdown_rank0": breakdown,
            "p99_constrained": p99c,
            "bs1": bs1,
            "fanout": fan,
            "distinct_inputs": {"slots": nslots, "images": nslots * bs,
                                "outputs_checked": slot_check},
            "fanout_errors": fan.get("errors", {}),
            "world_size_reported_by_process_group": dist.get_world_size() if world > 1 else 1,
        }
        for p in points:
            p.close()
        points.clear()

        # ---- bf16 engine: labelled reduced-precision operating point -------------------
        # (one GPU only: a multi-GPU scaling run stays on the headline engine)
        if not cpu and not args.no_bf16 and args.engine == "fp32" and world == 1:
            client.unregister_cuda_shared_memory()
            client.close()
            state["client"] = None
            srv.stop()
            srv, srv_log = start_server("fused", "bf16")
            srv.wait_ready(timeout=1500, model=model)
            client = grpcclient.InferenceServerClient(srv.grpc_url)
            state["client"] = client
            client.register_cuda_shared_memory("data_0_in", shmod.get_raw_handle(regions[0]), dev, in_total)
            client.register_cuda_shared_memory("fc6_1_out", shmod.get_raw_handle(regions[1]), dev,
                                               nslots * bs * 1000 * 4)
            ins, outs = slots(conc)
            pb = Point(srv, model, bs, conc, None, in_bytes, dev, cpu, inputs=ins, outputs=outs)
            points.append(pb)
            _, _, elb, _ = measure(pb, per, max(2, args.steps // 4), per)
            res["bf16_engine_infer_per_sec"] = round(world * max(2, args.steps // 4) * per * bs / elb, 1)
            res["bf16_engine_note"] = "same pipeline, bf16 K8-K10 kernels: ~3e-2 rel-L2 off fp32 (not the headline)"
        if rehearse:
            res["rehearsal"] = ("%d ranks on ONE GPU over gloo (launch/fan-out/aggregation rehearsal; "
                                "not a scaling measurement)" % world)
        if rank == 0:
            print(json.dumps(res), flush=True)
        return 0
    finally:
        for p in points:
            try:
                p.close()
            except Exception as e:  # noqa: BLE001
                log("perf session cleanup error: %s" % e)
        try:
            if state["client"] is not None:
                if cpu:
                    state["client"].unregister_system_shared_memory()
                else:
                    state["client"].unregister_cuda_shared_memory()
                state["client"].close()
        except Exception as e:  # noqa: BLE001
            log("cleanup error: %s" % e)
        for r in regions:
            try:
                shmod.destroy_shared_memory_region(r)
            except Exception:
                pass
        srv.stop()
        if world > 1 and dist.is_initialized():
            dist.destroy_process_group()


BERT_SEQ = 384


def bert_sweep(args, srv, model, client, shmod, regions, points, measure, fanout, rank, world, local_rank, cpu):
    """Config 4: bert_large seq-384 concurrency sweep, inputs fanned out by RCCL."""
    import numpy as np

    from triton_client_amd.perf.loadgen import percentile_us

    nbytes = BERT_SEQ * 4  # one request (bs 1) per region
    specs = (("input_ids", "random", 0.0, 30521.0), ("attention_mask", "constant", 1.0, 1.0),
             ("token_type_ids", "zero", 0.0, 0.0))
    inputs, method = {}, "local"
    for name, mode, lo, hi in specs:
        reg = "bert_%s" % name
        if cpu:
            key = "/%s_r%d_%d" % (reg, rank, os.getpid())
            r = shmod.create_shared_memory_region(reg, key, nbytes)
            regions.append(r)
            if mode == "random":
                data = np.random.default_rng(1234).integers(0, int(hi) + 1, BERT_SEQ, dtype=np.int32)
            else:
                data = np.full(BERT_SEQ, int(lo), np.int32)
            host = data if rank == 0 else np.zeros(BERT_SEQ, np.int32)
            method = fanout.fanout_host(host.view(np.uint8))
            shmod.set_shared_memory_region(r, [host])
            if not fanout.verify_host_replicas(host.view(np.uint8)):
                raise RuntimeError("fan-out replicas differ across ranks")
            client.register_system_shared_memory(reg, key, nbytes)
        else:
            r = shmod.create_shared_memory_region(reg, nbytes, local_rank)
            regions.append(r)
            method = fanout.fill_and_fanout(r, "INT32", BERT_SEQ, seed=1234, mode=mode, lo=lo, hi=hi,
                                            method=args.fanout, fallback=args.fanout_fallback)
            if not fanout.verify_replicas(r, nbytes, over_cpu=method == fanout.LOCAL_FALLBACK):
                raise RuntimeError("fan-out replicas differ across ranks")
            client.register_cuda_shared_memory(reg, shmod.get_raw_handle(r), local_rank, nbytes)
        inputs[name] = reg
    fan = {"method": method, "replicas_verified": True, "bytes": nbytes}
    if not cpu and world > 1:
        # X1 vs X2 on the token-id region, as the densenet run does on its batch
        rehearse = args.rehearse
        fan["timings"] = fanout.time_fanout(regions[0], nbytes, ["p2p", "host"] if rehearse else
                                            (["p2p"] if method == fanout.LOCAL_FALLBACK else ["rccl", "p2p"]))
        fan["errors"] = fanout.fanout_errors(fan["timings"])
        if not fanout.verify_replicas(regions[0], nbytes, over_cpu=method == fanout.LOCAL_FALLBACK):
            raise RuntimeError("fan-out replicas differ across ranks after the fan-out timing")
    sweep = []
    bert_max_batch = 64
    if not cpu:
        bert_max_batch = int(client.get_model_config(model, as_json=True)["config"].get("max_batch_size", 64))
    for c in [int(v) for v in args.sweep.split(",") if v]:
        # the batcher's preferred size for this load: one equal group per
        # instance (e.g. c16 on 2 instances ran as 5- and 11-row batches)
        n_inst = max(1, args.bert_instance_count)
        # (from 2 rows per instance: c4 1,312 -> 1,566 infer/s; without the longer
        # queue delay the 2-row preference had run mostly 1-row batches)
        pref = bert_point_preferred(args.bert_preferred, c, n_inst, args.bert_preferred_from, bert_max_batch)
        if pref and not cpu:
            # with a delay long enough for a partial group to wait for the next
            # group to come back (one batch), the loop converges on full groups
            client.load_model(model, config=json.dumps({"dynamic_batching": {
                "preferred_batch_size": [pref], "max_queue_delay_microseconds": max(args.bert_queue_delay_us, 20000)}}))
        nl = max(1, args.bert_lanes)
        if nl > 1 and c % nl == 0 and c >= 8 * nl:  # read-only input regions: the lanes may share them
            pt = Lanes([Point(srv, model, 1, c // nl, None, nbytes, local_rank, cpu, inputs=inputs,
                              out_bytes=BERT_SEQ * 4) for _ in range(nl)])
            points.extend(pt.points)
        else:
            pt = Point(srv, model, 1, c, None, nbytes, local_rank, cpu, inputs=inputs, out_bytes=BERT_SEQ * 4)
        if isinstance(pt, Point):
            points.append(pt)
        per = max(64, 8 * c)
        lat, _, elapsed, ((s0, b0), (s1, b1)) = measure(
            pt, max(args.warmup, 1) * per, args.steps, per, snap=lambda: (pt.s.server_stats(), batch_stats(client, model)))
        all_lat = fanout.gather_arrays(lat.astype(np.int64)).astype(np.float64)
        row = {"concurrency": c, "infer_per_sec": round(world * args.steps * per / elapsed, 1),
               "p50_latency_us": round(percentile_us(all_lat, 50), 1),
               "p99_latency_us": round(percentile_us(all_lat, 99), 1), "ms_per_step": round(1e3 * elapsed / args.steps, 3),
               "preferred_batch_rows": pref if pref and not cpu else None,
               "client_lanes": len(pt.points) if isinstance(pt, Lanes) else 1}
        # rank 0's server over the timed window: rows per executed batch, queueing, device time per batch
        bd = stats_delta(s0, s1)
        bd["batch_rows_histogram"] = {str(k): int(b1[k][0] - b0.get(k, (0,))[0]) for k in sorted(b1)
                                      if b1[k][0] - b0.get(k, (0,))[0] > 0}
        row["breakdown_rank0"] = bd
        sweep.append(row)
        log("bert c%d: %.1f infer/s p99 %.0f us" % (c, row["infer_per_sec"], row["p99_latency_us"]))
    top = sweep[-1]
    res = {
        "metric": BERT_METRIC,
        "value": top["infer_per_sec"],
        "unit": "infer/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": top["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32" if (cpu or args.bert_precision == "fp32") else "bf16",
        "data": ("synthetic INT32 (host, fanned out by %s), CPU %s" % (method, model) if cpu else
                 "synthetic INT32 token ids / all-ones mask / zero segments (K1 on device, fanned out by %s), "
                 "random-init weights" % method),
        "config": {"model": model, "global_batch": world * top["concurrency"], "seq_len": BERT_SEQ,
                   "parallelism": "dp%d" % world, "batch_size": 1, "protocol": "grpc",
                   "shared_memory": "system" if cpu else "hip", "loadgen": "native C++ (csrc/cpp/perf)",
                   "server_instances": args.bert_instance_count, "max_queue_delay_us": args.bert_queue_delay_us},
        "p99_latency_us": top["p99_latency_us"],
        "sweep": sweep,
        "fanout": fan,
    }
    if not cpu:
        res["config"]["compute"] = ("fp32 parity: bf16x3 projections and attention products (x_hi W_hi + x_hi W_lo + "
                                    "x_lo W_hi, fp32 accumulate), fp32 LayerNorm / softmax"
                                    if args.bert_precision == "fp32"
                                    else "bf16 (fp32 accumulate)")
        from triton_client_amd.models import bert as _bert

        res["config"]["gemm_routing"] = _bert.GEMM
    if args.rehearse and world > 1:
        res["rehearsal"] = ("%d ranks on ONE GPU over gloo (launch/fan-out/aggregation rehearsal; "
                            "not a scaling measurement)" % world)
    if rank == 0:
        print(json.dumps(res), flush=True)
    return 0


def _verify_slots(client, hipshm, regions, nslots, bs, dev):
    """After the timed run, output slice s holds the logits the server produced
    for slot s's images inside a mixed 128-row batch.  Re-run each slot's
    images alone (one bs-row request, its own HIP-graph bucket) and compare: a
    pointer-table or scatter row mix-up gives another image's logits (rel-L2
    ~1); split-K plans differ between buckets, so the bound is fp32-class."""
    import numpy as np
    import tritonclient.grpc as grpcclient

    ob = bs * 1000 * 4
    outs = hipshm.get_contents_as_numpy(regions[1], np.float32, [nslots, bs, 1000]).copy()
    chk = hipshm.create_shared_memory_region("fc6_1_slotchk", ob, dev)
    regions.append(chk)
    client.register_cuda_shared_memory("fc6_1_slotchk", hipshm.get_raw_handle(chk), dev, ob)
    worst = 0.0
    for s in range(nslots):
        x = grpcclient.InferInput("data_0", [bs, 3, 224, 224], "FP32")
        x.set_shared_memory("data_0_in", bs * 3 * 224 * 224 * 4, offset=s * bs * 3 * 224 * 224 * 4)
        o = grpcclient.InferRequestedOutput("fc6_1")
        o.set_shared_memory("fc6_1_slotchk", ob)
        client.infer("densenet_onnx", [x], outputs=[o])
        ref = hipshm.get_contents_as_numpy(chk, np.float32, [bs, 1000]).astype(np.float64)
        got = outs[s].astype(np.float64)
        rel = np.linalg.norm(got - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-30)
        worst = max(worst, float(rel.max()))
    client.unregister_cuda_shared_memory("fc6_1_slotchk")
    if not worst < 1e-3:
        raise RuntimeError("served outputs do not match their own inputs (worst per-row rel-L2 %.3g)" % worst)
    return {"slots": nslots, "rows": nslots * bs, "max_row_rel_l2_vs_unbatched": float("%.3g" % worst)}


def _sanity_check(client, hipshm, bs, dev, regions):
    """One python-client request over the same regions: finite logits land in our output region."""
    import numpy as np
    import tritonclient.grpc as grpcclient

    out_bytes = bs * 1000 * 4
    chk = hipshm.create_shared_memory_region("fc6_1_check", out_bytes, dev)
    regions.append(chk)
    client.register_cuda_shared_memory("fc6_1_check", hipshm.get_raw_handle(chk), dev, out_bytes)
    x = grpcclient.InferInput("data_0", [bs, 3, 224, 224], "FP32")
    x.set_shared_memory("data_0_in", bs * 3 * 224 * 224 * 4)
    o = grpcclient.InferRequestedOutput("fc6_1")
    o.set_shared_memory("fc6_1_check", out_bytes)
    client.infer("densenet_onnx", [x], outputs=[o])
    o0 = hipshm.get_contents_as_numpy(chk, np.float32, [bs, 1000])
    if not np.isfinite(o0).all() or not np.abs(o0).max() > 0:
        raise RuntimeError("bad logits in output region")


if __name__ == "__main__":
    sys.exit(main())
