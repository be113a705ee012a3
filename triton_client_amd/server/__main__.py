"""``python -m triton_client_amd.server`` — run the KServe-v2 test/bench server.

Example::

    python -m triton_client_amd.server --http-port 8000 --grpc-port 8001 --gpu --device 0
"""
import argparse
import asyncio
import json
import os
import signal
import sys


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--http-port", type=int, default=8000, help="0 disables HTTP")
    ap.add_argument("--grpc-port", type=int, default=8001, help="0 disables gRPC")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--gpu", action="store_true", help="also load the GPU model zoo")
    ap.add_argument("--device", type=int, default=0, help="GPU for the GPU models")
    ap.add_argument("--models", default="", help="comma-separated subset of models to load")
    ap.add_argument("--instance-count", type=int, default=0, help="override GPU model instance count")
    ap.add_argument("--max-queue-delay-us", type=int, default=-1)
    ap.add_argument("--idle-dispatch", default="on", choices=["on", "off"],
                    help="dispatch queued requests at once while every model instance is idle (else wait the delay)")
    ap.add_argument("--preferred-batch-sizes", default="",
                    help="override dynamic_batching.preferred_batch_size of the GPU models (comma-separated)")
    ap.add_argument("--max-batch-size", type=int, default=0,
                    help="override densenet_onnx max_batch_size (one of gpu_models.BUCKETS, <= 256; HIP-graph buckets up to it)")
    ap.add_argument("--no-graphs", action="store_true", help="disable HIP graph capture")
    ap.add_argument("--engine", default="fp32", choices=["fp32", "fused", "torch"],
                    help="densenet_onnx engine: fp32 = fp32-parity split-precision HIP/MFMA kernels (default), "
                         "fused = bf16 HIP/MFMA kernels, torch = the bf16 torch/MIOpen module")
    ap.add_argument("--ready-file", default="", help="touch this file once serving")
    ap.add_argument("--native-grpc", default="auto", choices=["auto", "on", "off"],
                    help="serve the gRPC port with tcserve (C++ front end, csrc/cpp/server)")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="HIP hardware queues for this process (sets GPU_MAX_HW_QUEUES, overriding an inherited "
                         "value such as the pool's 4; 0 = leave the environment alone).  Each model instance replays its graphs on its own stream; with 4 "
                         "instances plus copy streams on 4 queues, ready batches waited for a queue: 1.6 ms of "
                         "every request's server time was outside queue and compute (profiles/r3_hw_queues.md)")
    args = ap.parse_args(argv)
    if args.hw_queues > 0:
        # before anything initialises HIP in this process.  The GPU boxes
        # export GPU_MAX_HW_QUEUES=4 (HIP's own default) into every job, so a
        # setdefault here never took effect under bench.py there: the r3
        # 4 -> 8 A/B set it by hand
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(args.hw_queues, 32))

    # `kill -USR1 <server>` dumps every thread's Python stack into the server
    # log (the bench asks for it when a timed loop stops completing)
    import faulthandler
    import signal

    faulthandler.register(signal.SIGUSR1, all_threads=True)

    from .app import default_models, serve
    from .core import InferenceServer

    models = default_models(gpu=args.gpu, names=args.models.split(",") if args.models else None)
    opts = {}
    for m in models:
        if getattr(m, "instance_kind", "") == "KIND_GPU":
            o = {"device": args.device}
            if m.name == "densenet_onnx":
                o["engine"] = args.engine
                if args.max_batch_size:
                    o["max_batch_size"] = args.max_batch_size
            if args.no_graphs:
                o["use_graphs"] = False
            opts[m.name] = o
            if args.instance_count:
                m.instance_count = args.instance_count
            if args.max_queue_delay_us >= 0 and m.dynamic_batching is not None:
                m.dynamic_batching = dict(m.dynamic_batching, max_queue_delay_us=args.max_queue_delay_us)
            if m.dynamic_batching is not None:
                m.dynamic_batching = dict(m.dynamic_batching, idle_dispatch=args.idle_dispatch == "on")
            if args.preferred_batch_sizes and m.dynamic_batching is not None:
                pref = sorted(int(x) for x in args.preferred_batch_sizes.split(",") if x)
                m.dynamic_batching = dict(m.dynamic_batching, preferred=pref)
    server = InferenceServer(models, opts, device_id=args.device)
    server.load_all()

    async def run():
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGINT, signal.SIGTERM):
            loop.add_signal_handler(sig, stop.set)
        ready = asyncio.Event()
        task = asyncio.ensure_future(
            serve(server, args.http_port or None, args.grpc_port or None, args.host, ready, stop,
                  native_grpc={"auto": None, "on": True, "off": False}[args.native_grpc])
        )
        await ready.wait()
        print("SERVER READY http=%s grpc=%s" % (args.http_port, args.grpc_port), flush=True)
        if args.ready_file:
            with open(args.ready_file, "w") as f:
                f.write(str(os.getpid()))
        await task

    asyncio.run(run())
    # host-side phase totals of the native batch executors (graph_exec.hip)
    for entry in list(server.repo.values()):
        for inst in list(entry.instances.values()):
            fn = getattr(inst, "executor_stats", None)
            st = fn() if fn is not None else None
            if st and st.get("batches"):
                print("EXECUTOR STATS %s %s" % (entry.name, json.dumps(st)), flush=True)
    server.sys_shm.unregister()
    server.dev_shm.unregister()
    return 0


if __name__ == "__main__":
    sys.exit(main())
