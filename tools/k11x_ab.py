#!/usr/bin/env python3
"""K11x A/B: time the fused dense-layer kernel versions on the same inputs,
interleaved (v1, v3, v1, v3, ...) so box drift hits both arms alike, and
check every version against v1's output.

    python tools/k11x_ab.py --shapes 56:64,56:224,28:128,28:480 --imgs 128 --versions 1,3
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="56:64,56:128,56:224,28:128,28:224,28:480")
    ap.add_argument("--imgs", default="128")
    ap.add_argument("--versions", default="1,3")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--json", default="")
    a = ap.parse_args()

    import torch

    from triton_client_amd.ops import hip

    dev = "cuda"
    st = torch.cuda.current_stream().cuda_stream
    fns = {1: hip.x3_dense_fused, 3: hip.x3_dense_fused3, 5: hip.x3_dense_fused_ws}
    vers = [int(v) for v in a.versions.split(",")]
    rows = []
    for imgs in [int(v) for v in a.imgs.split(",")]:
        for sh in a.shapes.split(","):
            hw, K = (int(v) for v in sh.split(":"))
            M = imgs * hw * hw
            ldx = max(256, K + 32)
            g = torch.Generator(device=dev).manual_seed(hw * 1000 + K)
            x = torch.randn(M, ldx, device=dev, generator=g)

            def split(t):
                h = t.to(torch.bfloat16)
                return h.contiguous(), (t - h.float()).to(torch.bfloat16).contiguous()
            s = torch.rand(K, device=dev, generator=g) + 0.5
            t = torch.randn(K, device=dev, generator=g) * 0.1
            w1h, w1l = split(torch.randn(128, K, device=dev, generator=g) / K ** 0.5)
            b1 = torch.randn(128, device=dev, generator=g) * 0.1
            w3h, w3l = split(torch.randn(32, 9 * 128, device=dev, generator=g) * 0.03)
            f1h, f1l = hip.x3_w1_fragments(w1h), hip.x3_w1_fragments(w1l)
            frag = {v: (hip.x3_w3f_fragments(w3h), hip.x3_w3f_fragments(w3l)) for v in vers}
            outs = {}

            def run(v):
                fh, fl = frag[v]
                fns[v](x.data_ptr(), ldx, imgs, hw, hw, K, s.data_ptr(), t.data_ptr(), f1h.data_ptr(), f1l.data_ptr(),
                       b1.data_ptr(), fh.data_ptr(), fl.data_ptr(), x.data_ptr() + K * 4, ldx, stream=st)
            for v in vers:
                run(v)
                torch.cuda.synchronize()
                outs[v] = x[:, K:K + 32].clone()
            times = {v: [] for v in vers}
            for _ in range(a.rounds):
                for v in vers:
                    for _ in range(2):
                        run(v)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(a.iters):
                        run(v)
                    torch.cuda.synchronize()
                    times[v].append(1e6 * (time.perf_counter() - t0) / a.iters)
            ref = outs[vers[0]].double()
            row = {"imgs": imgs, "hw": hw, "K": K}
            for v in vers:
                row["v%d_us" % v] = round(min(times[v]), 1)
                row["v%d_us_all" % v] = [round(u, 1) for u in times[v]]
                row["v%d_rel_vs_v%d" % (v, vers[0])] = float((outs[v].double() - ref).norm() / ref.norm())
            rows.append(row)
            print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
