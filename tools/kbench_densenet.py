"""Per-layer timing of the fused DenseNet kernels (K8/K9) over tile variants.

For each distinct layer shape of DenseNet-121 at a batch size, times every
variant of conv1x1 (TM x BK) and conv3x3 (TM x tap group) with a HIP-graph
captured loop and prints a table (us per launch, effective TFLOP/s and GB/s).

  python tools/kbench_densenet.py --batch 128 --iters 50
"""

import argparse
import json

import torch

from triton_client_amd.ops import hip

V1 = (11, 12, 21, 22, 41, 211, 212, 221, 222, 300)
V3 = (0, 60, 70, 80, 90, 91, 92, 93)


def cs():
    return torch.cuda.current_stream().cuda_stream


def timed(fn, iters):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default="", help="'1x1' or '3x3'")
    a = ap.parse_args()
    dev = "cuda"
    b = a.batch
    res = {"batch": b, "conv1x1": [], "conv3x3": []}
    blocks = [(56, 64, 6), (28, 128, 12), (14, 256, 24), (7, 512, 16)]
    for hw, c0, n in blocks:
        ctot = c0 + 32 * n
        M = b * hw * hw
        x = torch.randn(M, ctot, device=dev).bfloat16()
        z = torch.randn(M, 128, device=dev).bfloat16()
        for K in sorted({c0, c0 + 32 * (n // 2), c0 + 32 * (n - 1)}) if a.only != "3x3" else []:
            s1 = torch.rand(K, device=dev) + 0.5
            t1 = torch.randn(K, device=dev)
            w = torch.randn(128, K, device=dev).bfloat16()
            bias = torch.randn(128, device=dev)
            row = {"hw": hw, "M": M, "K": K}
            for v in V1:
                try:
                    us = timed(lambda: hip.dn_conv1x1(x.data_ptr(), ctot, M, K, s1.data_ptr(), t1.data_ptr(),
                                                      w.data_ptr(), 128, bias.data_ptr(), 1, z.data_ptr(), 128,
                                                      variant=v, stream=cs()), a.iters)
                except RuntimeError:  # variant does not cover this shape (e.g. K8w: K <= 256)
                    continue
                row[v] = round(us, 2)
            best = min((v for v in V1 if v in row), key=lambda v: row[v])
            row["tflops"] = round(2.0 * M * K * 128 / (row[best] * 1e-6) / 1e12, 1)
            row["best"] = best
            res["conv1x1"].append(row)
            print("1x1", row, flush=True)
        if a.only == "1x1":
            continue
        w2 = torch.randn(32, 3, 3, 128, device=dev).bfloat16()
        row = {"hw": hw, "M": M}
        for v in V3:
            us = timed(lambda: hip.dn_conv3x3(z.data_ptr(), b, hw, hw, w2.data_ptr(), x.data_ptr() + 2 * c0, ctot,
                                              variant=v, stream=cs()), a.iters)
            row[v] = round(us, 2)
        best = min(V3, key=lambda v: row[v])
        row["tflops"] = round(2.0 * M * 1152 * 32 / (row[best] * 1e-6) / 1e12, 1)
        row["best"] = best
        res["conv3x3"].append(row)
        print("3x3", row, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
