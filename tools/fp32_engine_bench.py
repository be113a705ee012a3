#!/usr/bin/env python3
"""Device-side throughput of the fp32-parity DenseNet engine (K8x-K10x) vs the
bf16 engine: one HIP graph per batch size, N replays timed with events, on one
stream and on S concurrent streams (the server's model instances).

    python tools/fp32_engine_bench.py --batches 1,8,64,128 --streams 1,4
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,8,32,128")
    ap.add_argument("--streams", default="1,4")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--engines", default="fp32,bf16")
    ap.add_argument("--json", default="")
    ap.add_argument("--k14x-ab", action="store_true",
                    help="fp32 engine: also capture graphs with K14x off and interleave the two (rounds)")
    ap.add_argument("--ab", default="",
                    help="fp32 engine A/B of one engine attribute, interleaved per round: ATTR=V1,V2 "
                         "(e.g. fuse_v3=0,56; integer values), or of a native knob, captured into each "
                         "variant's graphs (e.g. TCAMD_X3_MAX_SPLITS=2,4; triton_client_amd/utils/knobs.py)")
    ap.add_argument("--rounds", type=int, default=1)
    args = ap.parse_args()
    import torch

    from triton_client_amd.models import densenet_fp32, densenet_fused
    from triton_client_amd.ops import hip

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    batches = [int(b) for b in args.batches.split(",")]
    streams = [int(s) for s in args.streams.split(",")]
    maxb = max(batches)
    rows = []
    for name in args.engines.split(","):
        if name == "fp32":
            eng, _ = densenet_fp32.build(maxb, device=dev)
        else:
            eng, _ = densenet_fused.build(maxb, device=dev)
        eng.concurrent_streams = max(streams)  # routing as a server with that many instances would pick
        engines = [eng] + [eng.with_workspace() for _ in range(max(streams) - 1)]
        imgs = torch.randn(maxb, 3, 224, 224, device=dev)
        for e in engines:
            e.ptrs[:maxb] = torch.arange(maxb, device=dev, dtype=torch.int64) * (3 * 224 * 224 * 4) + imgs.data_ptr()
        outs = [torch.zeros(maxb, 1000, device=dev) for _ in engines]
        sts = [torch.cuda.Stream(device=dev) for _ in engines]
        variants = [("default", None)]
        attr = "smallf_min_blocks"
        if args.k14x_ab and name == "fp32":
            variants = [("k14x", eng.smallf_min_blocks), ("pair", 0)]
        if args.ab and name == "fp32":
            attr, vals = args.ab.split("=")
            variants = [("%s=%s" % (attr, v), int(v)) for v in vals.split(",")]
        for b in batches:
            gv = {}
            for vname, mb in variants:
                graphs = []
                native = attr.startswith("TCAMD_") and attr in hip.knobs()
                prev = hip.knob_set(attr, mb) if native and mb is not None else None
                for e, o, s in zip(engines, outs, sts):
                    if mb is not None and not native:
                        setattr(e, attr, mb)
                    with torch.cuda.stream(s), torch.no_grad():
                        e.forward_ptrs(b, out=o)
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g, stream=s):
                            e.forward_ptrs(b, out=o)
                    graphs.append(g)
                if prev is not None:
                    hip.knob_set(attr, prev)
                gv[vname] = graphs
            torch.cuda.synchronize()
            for ns in streams:
                ts = {v: [] for v, _ in variants}
                for _ in range(args.rounds):
                    for vname, _ in variants:
                        graphs = gv[vname]
                        for _ in range(2):
                            for i in range(ns):
                                with torch.cuda.stream(sts[i]):
                                    graphs[i].replay()
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        for _ in range(args.iters):
                            for i in range(ns):
                                with torch.cuda.stream(sts[i]):
                                    graphs[i].replay()
                        torch.cuda.synchronize()
                        ts[vname].append(time.perf_counter() - t0)
                for vname, _ in variants:
                    dt = sorted(ts[vname])[len(ts[vname]) // 2]
                    ms = 1000 * dt / args.iters
                    r = {"engine": name, "variant": vname, "batch": b, "streams": ns, "ms_per_round": round(ms, 3),
                         "img_per_s": round(ns * b * args.iters / dt, 1)}
                    rows.append(r)
                    print(json.dumps(r), flush=True)
            graphs = None
            gv = None
        del engines, graphs
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
