"""GPU probe: per-variant DenseNet-121 forward timing on one MI355X.

Times (HIP-graph replay, bf16) the full forward per batch bucket for layout
variants, plus the stem conv (7x7/2, Cin=3) alone in each variant — MIOpen
has no MFMA solver for NHWC bf16 with Cin=3 and falls back to its naive
kernel, so the stem is probed with the input zero-padded to 4/8 channels.

  python tools/densenet_probe.py --buckets 1,8,64 --iters 20
"""

import argparse
import json
import time

import torch
import torch.nn.functional as F


def time_graph(fn, iters):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buckets", default="1,8,64")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--full", type=int, default=1)
    ap.add_argument("--stem", type=int, default=1)
    ap.add_argument("--nchw", type=int, default=1)
    ap.add_argument("--torch", type=int, default=1, help="time the torch/MIOpen module too")
    ap.add_argument("--fused", type=int, default=1, help="time the K8-K10 fused engine")
    a = ap.parse_args()
    from triton_client_amd.models import densenet

    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = False
    res = {}
    w = torch.randn(64, 3, 7, 7, device=dev, dtype=torch.bfloat16)
    for b in [int(x) for x in a.buckets.split(",")] if a.stem else []:
        r = {}
        for cpad in (3, 4, 8):
            x = torch.randn(b, cpad, 224, 224, device=dev, dtype=torch.bfloat16)
            wp = torch.zeros(64, cpad, 7, 7, device=dev, dtype=torch.bfloat16)
            wp[:, :3] = w
            xl = x.contiguous(memory_format=torch.channels_last)
            wl = wp.contiguous(memory_format=torch.channels_last)
            r["stem_nhwc_c%d" % cpad] = time_graph(lambda: F.conv2d(xl, wl, stride=2, padding=3), a.iters)
            r["stem_nchw_c%d" % cpad] = time_graph(lambda: F.conv2d(x, wp, stride=2, padding=3), a.iters)
            print(b, cpad, r["stem_nhwc_c%d" % cpad], r["stem_nchw_c%d" % cpad], flush=True)
        res[b] = r
    buckets = [int(x) for x in a.buckets.split(",")]
    if a.fused:
        from triton_client_amd.models import densenet_fused

        eng, _ = densenet_fused.build(max(buckets), device=dev)
        for b in buckets:
            xl = torch.randn(b, 3, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            with torch.no_grad():
                ms = time_graph(lambda: eng(xl), a.iters)
            res.setdefault(b, {})["fused"] = ms
            print("fused", b, "%.3f ms" % ms, "%.0f img/s" % (b * 1000.0 / ms), flush=True)
    if a.full and a.torch:
        m = densenet.build(device=dev)
        mc = densenet.build(device=dev).to(memory_format=torch.contiguous_format)
        for b in [int(x) for x in a.buckets.split(",")]:
            x = torch.randn(b, 3, 224, 224, device=dev, dtype=torch.bfloat16)
            xl = x.contiguous(memory_format=torch.channels_last)
            with torch.no_grad():
                res.setdefault(b, {})
                res[b]["full_nhwc"] = time_graph(lambda: m(xl), a.iters)
                if a.nchw:
                    res[b]["full_nchw"] = time_graph(lambda: mc(x), a.iters)
            print(b, res[b], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    t = time.time()
    main()
    print("elapsed", time.time() - t)
