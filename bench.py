#!/usr/bin/env python3
"""Flagship serving benchmark: perf_analyzer-style inferences/sec + p99 latency
for ``densenet_onnx`` over gRPC with HIP shared memory (BASELINE.json metric).

One process per GPU (``torch.distributed.run`` for N>1; RCCL over xGMI):

  rank r: spawns the KServe-v2 bench server pinned to GPU r (child process,
          HIP IPC needs two processes), allocates a HIP shm input region and
          one output region per in-flight slot, receives the synthetic input
          batch (K1 Philox on rank 0 -> RCCL broadcast into every rank's
          region), registers the regions, then drives `concurrency` requests
          in flight (closed loop) against its own server.

A "step" = every in-flight slot completes one request (concurrency requests,
each carrying `--batch` images).  W warmup steps, then EXACTLY K timed steps
between barrier + device sync; elapsed = MAX over ranks; value = total images
per second over all ranks (weak scaling: per-GPU work is fixed).
"""

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)


def log(*a):
    print("[bench rank %s]" % os.environ.get("RANK", "0"), *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=8, help="images per request (densenet_onnx bs)")
    ap.add_argument("--concurrency", type=int, default=48, help="requests in flight per GPU")
    ap.add_argument("--fanout", default="rccl", choices=["rccl", "p2p", "local"])
    # operating point from tools/gpu_bench_sweep.sh on MI355X (profiles/r1_operating_points.md):
    # four model instances (HIP streams) each running full 128-row batches overlap
    # well on the 256 CUs (~1.3x one stream's throughput)
    ap.add_argument("--instance-count", type=int, default=4)
    ap.add_argument("--max-queue-delay-us", type=int, default=2000)
    ap.add_argument("--max-batch-size", type=int, default=0, help="server densenet_onnx max_batch_size (0 = model default 128)")
    ap.add_argument("--preferred", default="128", help="server preferred batch sizes (comma-separated rows; '' = none)")
    # a closed-loop saturation run wants full batches: no early dispatch of partial ones
    ap.add_argument("--idle-dispatch", default="off", choices=["on", "off"],
                    help="server: dispatch partial batches at once while every instance is idle")
    ap.add_argument("--engine", default="fused", choices=["fused", "torch"],
                    help="densenet_onnx engine in the server (fused HIP/MFMA kernels or torch/MIOpen)")
    ap.add_argument("--loadgen", default="native", choices=["native", "python"],
                    help="native: C++ perf engine (csrc/cpp/perf) in-process via ctypes; python: grpc.aio loop")
    ap.add_argument("--server-log", default="")
    ap.add_argument("--server-url", default="", help="use an already running server (gRPC host:port, HTTP port = +1 unless --http-url)")
    ap.add_argument("--http-url", default="")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

    from triton_client_amd.perf.harness import ExternalServer, ServerProcess

    bs, conc = args.batch, args.concurrency
    log_path = args.server_log or os.path.join(REPO, "gpurun_out", "bench_server_r%d.log" % rank)
    os.makedirs(os.path.dirname(log_path), exist_ok=True)
    # spawn the server before this process touches the GPU
    if args.server_url:
        srv = ExternalServer(args.server_url, args.http_url)
    else:
        srv = ServerProcess(
            device=local_rank,
            models="densenet_onnx",
            extra_args=["--instance-count", str(args.instance_count), "--engine", args.engine,
                        "--max-queue-delay-us", str(args.max_queue_delay_us)]
            + (["--preferred-batch-sizes", args.preferred] if args.preferred else [])
            + (["--max-batch-size", str(args.max_batch_size)] if args.max_batch_size else [])
            + ["--idle-dispatch", args.idle_dispatch],
            log_path=log_path,
            # per-rank port range: N ranks start their servers at once
            port_stripe=local_rank if world > 1 else None,
        )

    import numpy as np
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import tritonclient.grpc as grpcclient
    from tritonclient.utils import hip_shared_memory as hipshm
    from triton_client_amd.parallel import fanout
    from triton_client_amd.perf.loadgen import ConcurrencyRun, percentile_us
    regions = []
    sessions = []
    client = None
    try:
        log("waiting for server (log %s)" % log_path)
        srv.wait_ready(timeout=1500, model="densenet_onnx")
        log("server ready")
        client = grpcclient.InferenceServerClient(srv.grpc_url)

        in_elems = bs * 3 * 224 * 224
        in_bytes = in_elems * 4
        out_bytes = bs * 1000 * 4
        inp = hipshm.create_shared_memory_region("data_0_in", in_bytes, local_rank)
        regions.append(inp)
        method = fanout.fill_and_fanout(inp, "FP32", in_elems, seed=1234, mode="normal", lo=0.0, hi=1.0,
                                        method=args.fanout)
        if not fanout.verify_replicas(inp, in_bytes):
            raise RuntimeError("fan-out replicas differ across ranks")
        client.register_cuda_shared_memory("data_0_in", hipshm.get_raw_handle(inp), local_rank, in_bytes)
        # one python-client request first: sanity of the whole shm path (finite logits land in our region)
        chk = hipshm.create_shared_memory_region("fc6_1_check", out_bytes, local_rank)
        regions.append(chk)
        client.register_cuda_shared_memory("fc6_1_check", hipshm.get_raw_handle(chk), local_rank, out_bytes)
        x = grpcclient.InferInput("data_0", [bs, 3, 224, 224], "FP32")
        x.set_shared_memory("data_0_in", in_bytes)
        o = grpcclient.InferRequestedOutput("fc6_1")
        o.set_shared_memory("fc6_1_check", out_bytes)
        client.infer("densenet_onnx", [x], outputs=[o])
        o0 = hipshm.get_contents_as_numpy(chk, np.float32, [bs, 1000])
        if not np.isfinite(o0).all() or not np.abs(o0).max() > 0:
            raise RuntimeError("bad logits in output region")

        if args.loadgen == "native":
            from triton_client_amd.perf.native import PerfSession

            perf = PerfSession(["-m", "densenet_onnx", "-i", "grpc", "-u", srv.grpc_url, "-b", bs,
                                "--shared-memory", "hip", "--device", local_rank,
                                "--shared-memory-input", "data_0=data_0_in",
                                "--output-shared-memory-size", out_bytes, "--concurrency-range", conc])
            sessions.append(perf)

            def run(steps):
                lat_ns, el = perf.run_fixed(conc, steps * conc)
                return lat_ns.astype(np.float64), []
        else:
            outs = []
            for s in range(conc):
                name = "fc6_1_out_%d" % s
                r = hipshm.create_shared_memory_region(name, out_bytes, local_rank)
                regions.append(r)
                client.register_cuda_shared_memory(name, hipshm.get_raw_handle(r), local_rank, out_bytes)
                o = grpcclient.InferRequestedOutput("fc6_1")
                o.set_shared_memory(name, out_bytes)
                outs.append([o])
            runner = ConcurrencyRun(client, "densenet_onnx", [x], outs, conc)

            def run(steps):
                lat, errs, _ = runner.run(steps)
                return lat, errs

        lat, errs = run(max(args.warmup, 1))
        if errs:
            raise RuntimeError("warmup errors: %s" % errs[0])
        log("warmup done (%s loadgen): p50 %.0f us" % (args.loadgen, percentile_us(lat, 50)))

        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lat, errs = run(args.steps)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if errs:
            raise RuntimeError("%d request errors, first: %s" % (len(errs), errs[0]))
        elapsed_max = fanout.max_over_ranks(elapsed)
        all_lat = fanout.gather_arrays(lat)
        images = world * args.steps * conc * bs
        value = images / elapsed_max
        stats = client.get_inference_statistics("densenet_onnx", as_json=True)
        if rank == 0:
            ms = stats["model_stats"][0]
            execs = int(ms.get("execution_count", 0))
            infers = int(ms.get("inference_count", 0))
            bst = ms.get("batch_stats", [])
            nb = sum(int(b["compute_infer"].get("count", 0)) for b in bst) or 1
            gpu_ms = {k: sum(int(b[k].get("ns", 0)) for b in bst) / nb / 1e6
                      for k in ("compute_input", "compute_infer", "compute_output")}
            log("server per-batch device ms: %s  avg rows %.1f" % (
                {k: round(v, 3) for k, v in gpu_ms.items()}, infers / max(execs, 1)))
            res = {
                "metric": "perf_analyzer inferences/sec (densenet_onnx, HIP shm)",
                "value": round(value, 2),
                "unit": "infer/sec",
                "n_gpus": world,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": round(1000.0 * elapsed_max / args.steps, 3),
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": None,
                "dtype": "bf16",
                "data": "synthetic (K1 Philox normal on device, fanned out by %s), random-init weights" % method,
                "config": {
                    "model": "densenet_onnx",
                    "global_batch": world * conc * bs,
                    "seq_len": None,
                    "parallelism": "dp%d" % world,
                    "batch_size": bs,
                    "concurrency_per_gpu": conc,
                    "protocol": "grpc",
                    "shared_memory": "hip",
                    "engine": args.engine,
                    "loadgen": args.loadgen,
                    "server_instances": args.instance_count,
                    "preferred_batch_rows": args.preferred,
                    "max_queue_delay_us": args.max_queue_delay_us,
                    "server_max_batch_rows": args.max_batch_size or 128,
                    "idle_dispatch": args.idle_dispatch,
                },
                "p50_latency_us": round(percentile_us(all_lat, 50), 1),
                "p90_latency_us": round(percentile_us(all_lat, 90), 1),
                "p99_latency_us": round(percentile_us(all_lat, 99), 1),
                "requests_per_sec": round(value / bs, 2),
                "server_avg_batch_rows_rank0": round(infers / max(execs, 1), 2),
                "server_device_ms_per_batch_rank0": {k: round(v, 3) for k, v in gpu_ms.items()},
            }
            print(json.dumps(res), flush=True)
        return 0
    finally:
        for p in sessions:
            try:
                p.close()
            except Exception as e:  # noqa: BLE001
                log("perf session cleanup error: %s" % e)
        try:
            if client is not None:
                client.unregister_cuda_shared_memory()
                client.close()
        except Exception as e:  # noqa: BLE001
            log("cleanup error: %s" % e)
        for r in regions:
            try:
                hipshm.destroy_shared_memory_region(r)
            except Exception:
                pass
        srv.stop()
        if world > 1 and dist.is_initialized():
            dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
