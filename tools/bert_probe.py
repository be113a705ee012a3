"""Time one BERT-large (seq 384) forward per batch size on the GPU; run under
``rocprofv3 --kernel-trace --stats`` for the per-kernel split.

  python tools/bert_probe.py --batch 64 --iters 10
  python tools/bert_probe.py --batch 1 8 64 --gemm lib,auto,ours --graphs   # projection routing A/B, HIP graphs
"""

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from triton_client_amd.models import bert  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[64])
    ap.add_argument("--seq", type=int, default=384)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tuned-table", default="",
                    help="A/B against TunableOp reading this solution table (tuning off), e.g. "
                         "triton_client_amd/models/tuned/bert_large_gfx950.csv")
    ap.add_argument("--tunable", default="",
                    help="A/B against PyTorch TunableOp (hipBLASLt / rocBLAS solution search per GEMM shape); "
                         "the tuned results go to this CSV path")
    ap.add_argument("--gemm", default="", help="A/B the projection routing modes (bert.GEMM), e.g. lib,auto,ours")
    ap.add_argument("--graphs", action="store_true", help="time HIP-graph replays of the forward (as served)")
    ap.add_argument("--fp32", action="store_true", help="the fp32-parity model (bert_large_fp32: bf16x3 projections)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = (bert.prepare_x3(bert.build(device=dev, dtype=torch.float32)) if a.fp32 else bert.build(device=dev))
    for b in a.batch:
        ids = torch.randint(0, bert.VOCAB, (b, a.seq), device=dev)
        mask = torch.ones(b, a.seq, device=dev, dtype=torch.int64)
        tt = torch.zeros(b, a.seq, device=dev, dtype=torch.int64)
        variants = {"default": 0}
        if a.gemm:
            variants = {m: 0 for m in a.gemm.split(",")}
        tun = None
        if a.tuned_table:
            import torch.cuda.tunable as tun

            assert bert.use_tuned_gemms(a.tuned_table), "the table does not load in this process"
            variants = {"default": 0, "tunableop": 0}
        elif a.tunable:
            import torch.cuda.tunable as tun

            tun.set_filename(a.tunable)
            variants = {"default": 0, "tunableop": 0}
            with torch.no_grad():  # tune every GEMM shape of this batch once, outside the timed rounds
                tun.enable(True)
                tun.tuning_enable(True)
                model(ids, mask, tt)
                torch.cuda.synchronize()
                tun.tuning_enable(False)
                tun.enable(False)
        ts = {k: [] for k in variants}
        graphs = {}
        with torch.no_grad():
            for name in variants:
                if tun is not None:
                    tun.enable(name == "tunableop")
                if a.gemm:
                    bert.GEMM = name
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):  # warm-up on the capture stream (K17 allocates its workspace there)
                    for _ in range(2):
                        model(ids, mask, tt)
                torch.cuda.current_stream().wait_stream(s)
                if a.graphs:
                    with torch.cuda.stream(s):
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g, stream=s):
                            model(ids, mask, tt)
                    torch.cuda.current_stream().wait_stream(s)
                    graphs[name] = g
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for name in variants:
                    if tun is not None:
                        tun.enable(name == "tunableop")
                    if a.gemm:
                        bert.GEMM = name
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(a.iters):
                        if a.graphs:
                            graphs[name].replay()
                        else:
                            model(ids, mask, tt)
                    torch.cuda.synchronize()
                    ts[name].append((time.perf_counter() - t0) / a.iters)
        for name, v in ts.items():
            dt = sorted(v)[len(v) // 2]
            tf = bert.flops_per_sequence(a.seq) * b / dt / 1e12
            print({"batch": b, "variant": name, "fp32": a.fp32, "ms": round(dt * 1e3, 3), "seq_per_s": round(b / dt, 1),
                   "tflops": round(tf, 1)}, flush=True)


if __name__ == "__main__":
    main()
