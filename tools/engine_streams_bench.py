"""Device-side ceiling of the fused DenseNet engine under concurrency: S model
instances (one HIP stream + one captured HIP graph each, like the server's
instances) replay bs-B forwards back to back; prints aggregate img/s.

  python tools/engine_streams_bench.py --batch 128 --streams 1 2 3 4 6 --iters 30
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from triton_client_amd.models import densenet_fused  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--streams", type=int, nargs="+", default=[1, 2, 3, 4, 6])
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    base, _ = densenet_fused.build(a.batch, device=dev)
    res = []
    for S in a.streams:
        engines = [base] + [base.with_workspace() for _ in range(S - 1)]
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        graphs = []
        for e, s in zip(engines, streams):
            x = torch.randn(a.batch, 224, 224, 3, device=dev).bfloat16()
            out = torch.empty(a.batch, 1000, device=dev)
            with torch.cuda.stream(s):
                e(x.permute(0, 3, 1, 2), out=out)
                s.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    e(x.permute(0, 3, 1, 2), out=out)
            graphs.append((g, x, out))
        torch.cuda.synchronize()
        for _ in range(2):
            for (g, _, _), s in zip(graphs, streams):
                with torch.cuda.stream(s):
                    g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            for (g, _, _), s in zip(graphs, streams):
                with torch.cuda.stream(s):
                    g.replay()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        r = {"streams": S, "batch": a.batch, "img_per_s": round(S * a.iters * a.batch / dt, 1),
             "ms_per_forward_per_stream": round(1000 * dt / a.iters, 3)}
        print(r, flush=True)
        res.append(r)
        del graphs
    print(json.dumps(res))


if __name__ == "__main__":
    main()
