#!/usr/bin/env python3
"""Dense-layer pair (K8x 1x1 -> K9x 3x3) over a bs128 56x56 (or 28x28) feature
map, run whole or in image chunks so the 1x1's z (hi|lo, 512 B per pixel) is
re-read by the 3x3 while it is still in the 256 MB Infinity Cache (MALL).

    python tools/x3_pair_bench.py --hw 56 --k 64 --chunks 128,64,32,16
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", type=int, default=56)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--ldx", type=int, default=256)
    ap.add_argument("--imgs", type=int, default=128)
    ap.add_argument("--chunks", default="128,64,32,16")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--ks", default="", help="comma list of K: loop over them (overrides --k)")
    ap.add_argument("--both", action="store_true", help="also time K11x v1 in a child (default v3)")
    a = ap.parse_args()
    for K in ([int(v) for v in a.ks.split(",")] if a.ks else [a.k]):
        a.k = K
        bench(a)


def bench(a):
    import torch

    from triton_client_amd.ops import hip

    dev = "cuda"
    st = torch.cuda.current_stream().cuda_stream
    HW = a.hw * a.hw
    M = a.imgs * HW
    K = a.k

    def split(t):
        h = t.to(torch.bfloat16)
        return h.contiguous(), (t - h.float()).to(torch.bfloat16).contiguous()

    x = torch.randn(M, a.ldx, device=dev)
    s = torch.rand(K, device=dev) + 0.5
    t = torch.randn(K, device=dev) * 0.1
    w1h, w1l = split(torch.randn(128, K, device=dev) / K ** 0.5)
    b1 = torch.randn(128, device=dev)
    w3h, w3l = split(torch.randn(32, 9 * 128, device=dev) * 0.03)
    zh = torch.empty(M, 128, device=dev, dtype=torch.bfloat16)
    zl = torch.empty_like(zh)
    ws = torch.empty(64 << 20, device=dev, dtype=torch.uint8)
    for c in [int(v) for v in a.chunks.split(",") if v]:
        def run():
            for i0 in range(0, a.imgs, c):
                n = min(c, a.imgs - i0)
                r0 = i0 * HW
                m = n * HW
                wsb = hip.x3_conv1x1_ws_bytes(m, K)
                hip.x3_conv1x1(x.data_ptr() + r0 * a.ldx * 4, a.ldx, m, K, s.data_ptr(), t.data_ptr(), w1h.data_ptr(),
                               w1l.data_ptr(), out_bias=b1.data_ptr(), z_hi=zh.data_ptr() + r0 * 256,
                               z_lo=zl.data_ptr() + r0 * 256, ws=ws.data_ptr(), ws_bytes=min(wsb, ws.numel()),
                               stream=st)
                hip.x3_conv3x3(zh.data_ptr() + r0 * 256, zl.data_ptr() + r0 * 256, n, a.hw, a.hw, w3h.data_ptr(),
                               w3l.data_ptr(), x.data_ptr() + (r0 * a.ldx + K) * 4, a.ldx, stream=st)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            run()
        torch.cuda.synchronize()
        us = 1e6 * (time.perf_counter() - t0) / a.iters
        print("hw=%d k=%d chunk=%d: %.1f us per %d images" % (a.hw, K, c, us, a.imgs), flush=True)
    # K11x: the same layer in one kernel, z kept in LDS
    f1h, f1l = hip.x3_w1_fragments(w1h), hip.x3_w1_fragments(w1l)
    v = int(os.environ.get("X3_PAIR_BENCH_V", "3"))
    frag = hip.x3_w3f_fragments
    fn = hip.x3_dense_fused if v == 1 else hip.x3_dense_fused3
    f3h, f3l = frag(w3h), frag(w3l)

    def fused():
        fn(x.data_ptr(), a.ldx, a.imgs, a.hw, a.hw, K, s.data_ptr(), t.data_ptr(), f1h.data_ptr(), f1l.data_ptr(),
           b1.data_ptr(), f3h.data_ptr(), f3l.data_ptr(), x.data_ptr() + K * 4, a.ldx, stream=st)
    for _ in range(3):
        fused()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        fused()
    torch.cuda.synchronize()
    us = 1e6 * (time.perf_counter() - t0) / a.iters
    print("hw=%d k=%d fused v%d: %.1f us per %d images" % (a.hw, K, v, us, a.imgs), flush=True)
    runs = []
    if a.both and os.environ.get("X3_PAIR_BENCH_V", "3") == "3":
        runs.append(("X3_PAIR_BENCH_V", "1", {}))
    if runs:
        import subprocess
        for var, d, extra in runs:
            # the knobs are read once per process: one child per setting
            env = dict(os.environ, **{var: d}, **extra)
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--hw", str(a.hw), "--k", str(K),
                                  "--imgs", str(a.imgs), "--ldx", str(a.ldx), "--chunks", "", "--iters",
                                  str(a.iters)], env=env, capture_output=True, text=True, timeout=300)
            line = [ln for ln in out.stdout.splitlines() if "fused" in ln]
            print("  %s=%s: %s" % (var, d, " / ".join(line) if line else out.stderr[-300:]), flush=True)


if __name__ == "__main__":
    main()
