#!/usr/bin/env python3
"""Microbenchmark of single fp32-parity DenseNet kernels (K8x 1x1 / K9x 3x3)
at the bs=128 layer shapes, for rocprofv3 counter passes and A/B timing:

    python tools/x3_kbench.py --op conv3x3 --hw 56 --imgs 128 --iters 20
    python tools/x3_kbench.py --op conv1x1 --hw 56 --imgs 128 --k 224
"""

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="conv3x3", choices=["conv3x3", "conv1x1", "pool"])
    ap.add_argument("--hw", type=int, default=56)
    ap.add_argument("--imgs", type=int, default=128)
    ap.add_argument("--k", type=int, default=224, help="1x1: input channels")
    ap.add_argument("--ldx", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch

    from triton_client_amd.ops import hip

    dev = "cuda"
    st = torch.cuda.current_stream().cuda_stream
    M = args.imgs * args.hw * args.hw

    def split(t):
        h = t.to(torch.bfloat16)
        return h.contiguous(), (t - h.float()).to(torch.bfloat16).contiguous()

    if args.op == "conv3x3":
        z = torch.relu(torch.randn(M, 128, device=dev))
        zh, zl = split(z)
        wh, wl = split(torch.randn(32, 9 * 128, device=dev) * 0.03)
        ldy = 256
        y = torch.zeros(M, ldy, device=dev)

        def run():
            hip.x3_conv3x3(zh.data_ptr(), zl.data_ptr(), args.imgs, args.hw, args.hw, wh.data_ptr(), wl.data_ptr(),
                           y.data_ptr(), ldy, stream=st)
        flop = 2.0 * M * 1152 * 32
        hbm = 4.0 * M * (128 + 32)
    else:
        pool = args.op == "pool"
        K = args.k
        ldx = args.ldx or K
        x = torch.randn(M, ldx, device=dev)
        s = torch.rand(K, device=dev) + 0.5
        t = torch.randn(K, device=dev) * 0.1
        N = K // 2 if pool else 128
        wh, wl = split(torch.randn(N, K, device=dev) / K ** 0.5)
        b = torch.randn(128, device=dev)
        Mo = M // 4 if pool else M
        zh = torch.empty(Mo, 128, device=dev, dtype=torch.bfloat16)
        zl = torch.empty_like(zh)
        y = torch.empty(Mo, N, device=dev)
        wsb = hip.x3_conv1x1_ws_bytes(Mo, K, N)
        ws = torch.empty(max(wsb, 16), device=dev, dtype=torch.uint8)

        def run():
            if pool:
                hip.x3_conv1x1(x.data_ptr(), ldx, Mo, K, s.data_ptr(), t.data_ptr(), wh.data_ptr(), wl.data_ptr(),
                               y=y.data_ptr(), ldy=N, pool=1, H=args.hw, W=args.hw, ws=ws.data_ptr(), ws_bytes=wsb,
                               stream=st, N=N)
            else:
                hip.x3_conv1x1(x.data_ptr(), ldx, M, K, s.data_ptr(), t.data_ptr(), wh.data_ptr(), wl.data_ptr(),
                               out_bias=b.data_ptr(), z_hi=zh.data_ptr(), z_lo=zl.data_ptr(), ws=ws.data_ptr(),
                               ws_bytes=wsb, stream=st)
        flop = 2.0 * Mo * K * N
        hbm = 4.0 * (M * K + Mo * N)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        run()
    torch.cuda.synchronize()
    us = 1e6 * (time.perf_counter() - t0) / args.iters
    print("%s hw=%d imgs=%d k=%d: %.1f us/launch, %.0f TFLOP/s fp32-equivalent (x3 on MFMA: %.0f), %.2f TB/s" % (
        args.op, args.hw, args.imgs, args.k, us, flop / us / 1e6, 3 * flop / us / 1e6, hbm / us / 1e6), flush=True)


if __name__ == "__main__":
    main()
