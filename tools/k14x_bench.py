#!/usr/bin/env python3
"""K14x (one-kernel dense layer at 14x14 / 7x7) against the K8x + K9x pair it
replaces, per K, plus the whole fp32 forward with and without it.  Variants
are interleaved round by round in one process (median of the rounds).

    python tools/k14x_bench.py --hw 14 --imgs 128 --ks 256,512,992
    python tools/k14x_bench.py --forward 128,64,32 --rounds 10
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(torch, fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters  # us


def layers(a, torch, hip):
    dev = "cuda"
    st = torch.cuda.current_stream().cuda_stream
    out = []
    for hw in [int(v) for v in a.hw.split(",")]:
        M = a.imgs * hw * hw
        for K in [int(v) for v in a.ks.split(",")]:
            ldx = max(K + 32, a.ldx)

            def split(t):
                h = t.to(torch.bfloat16)
                return h.contiguous(), (t - h.float()).to(torch.bfloat16).contiguous()

            x = torch.randn(M, ldx, device=dev)
            s = torch.rand(K, device=dev) + 0.5
            t = torch.randn(K, device=dev) * 0.1
            w1h, w1l = split(torch.randn(128, K, device=dev) / K ** 0.5)
            b1 = torch.randn(128, device=dev) * 0.1
            w2 = split(torch.randn(32, 9 * 128, device=dev) * 0.03)
            f2 = [hip.x3_w3f_fragments(u) for u in w2]
            w3 = [hip.x3_w3_fragments(u) for u in w2]
            zh = torch.empty(M, 128, device=dev, dtype=torch.bfloat16)
            zl = torch.empty_like(zh)
            ws = torch.empty(256 << 20, device=dev, dtype=torch.uint8)
            y = x.data_ptr() + 4 * K

            def pair():
                hip.x3_dense_layer(x.data_ptr(), ldx, a.imgs, hw, hw, K, s.data_ptr(), t.data_ptr(), w1h.data_ptr(),
                                   w1l.data_ptr(), b1.data_ptr(), zh.data_ptr(), zl.data_ptr(), w3[0].data_ptr(),
                                   w3[1].data_ptr(), y, ldx, ws=ws.data_ptr(), ws_bytes=ws.numel(), stream=st)

            f1 = [hip.x3_w1_fragments(u) for u in (w1h, w1l)]

            def k14():
                hip.x3_dense_small(x.data_ptr(), ldx, a.imgs, hw, hw, K, s.data_ptr(), t.data_ptr(), w1h.data_ptr(),
                                   w1l.data_ptr(), b1.data_ptr(), f2[0].data_ptr(), f2[1].data_ptr(), y, ldx,
                                   stream=st, w1f_hi=f1[0].data_ptr(), w1f_lo=f1[1].data_ptr())

            for f in (pair, k14):
                f()
            torch.cuda.synchronize()
            tp, tk = [], []
            for _ in range(a.rounds):
                tp.append(timeit(torch, pair, a.iters))
                tk.append(timeit(torch, k14, a.iters))
            tp.sort()
            tk.sort()
            gb = M * K * 4 / 1e9
            row = {"hw": hw, "imgs": a.imgs, "K": K, "pair_us": round(tp[len(tp) // 2], 2),
                   "k14x_us": round(tk[len(tk) // 2], 2), "k14x_min_us": round(tk[0], 2),
                   "x_TBps_k14x": round(gb / (tk[len(tk) // 2] * 1e-6) / 1e3, 2)}
            if a.stamp:
                k14()
                torch.cuda.synchronize()
                sm = hip.x3_small_stamps()
                sm = sm[sm[:, 0] > 0]
                t0 = sm[:, 0].min()
                rel = (sm - t0) / 100.0  # us
                ph = {"prologue": (1, 0), "1x1": (2, 1), "z_handover": (3, 2), "z_write": (4, 3), "3x3": (5, 4),
                      "exchange_store": (6, 5)}
                med = {k: round(float(np.median(rel[:, b] - rel[:, e])), 2) for k, (b, e) in ph.items()}
                row["stamps"] = {"blocks": int(len(sm)), "start_spread_us": round(float(rel[:, 0].max()), 2),
                                 "span_us": round(float(rel[:, 7].max()), 2),
                                 "end_spread_us": round(float(rel[:, 7].max() - rel[:, 7].min()), 2),
                                 "median_phase_us": med}
            if a.stamp and a.dbg and int(a.dbg) & 64:
                tlv = hip.x3_small_timeline()
                n = min(int((tlv[:, 2] > 0).sum()), K // 32 - 1)
                d = tlv[:n]
                rel = np.concatenate([[0], np.maximum(d[:-1, 2], d[:-1, 3])])  # previous barrier (approx. release)
                row["timeline_cycles"] = {
                    "x_wait": np.median(d[1:, 0] - rel[1:]).item(), "convert": np.median(d[1:, 1] - d[1:, 0]).item(),
                    "w_issue_and_wait": np.median(d[1:, 2] - d[1:, 1]).item(),
                    "producer_step": np.median(d[1:, 2] - rel[1:]).item(),
                    "consumer_step": np.median(d[1:, 3] - rel[1:]).item(),
                    "producer_last": int((d[1:, 2] > d[1:, 3]).sum()), "steps": n - 1}
            print(json.dumps(row), flush=True)
            out.append(row)
    return out


def forward(a, torch):
    from triton_client_amd.models import densenet_fp32

    dev = torch.device("cuda", 0)
    bmax = max(int(v) for v in a.forward.split(","))
    eng, _ = densenet_fp32.build(max_batch=bmax, device=dev)
    x = torch.randn(bmax, 3, 224, 224, device=dev)
    out = torch.empty(bmax, 1000, device=dev)
    for b in [int(v) for v in a.forward.split(",")]:
        eng.ptrs[:b] = eng._img_off[:b] + x.data_ptr()
        res = {}
        variants = {"pair": 0, "k14x": a.min_blocks}
        for name, mb in variants.items():
            eng.smallf_min_blocks = mb
            with torch.no_grad():
                eng.forward_ptrs(b, out=out)
        torch.cuda.synchronize()
        ts = {n: [] for n in variants}
        for _ in range(a.rounds):
            for name, mb in variants.items():
                eng.smallf_min_blocks = mb
                with torch.no_grad():
                    ts[name].append(timeit(torch, lambda: eng.forward_ptrs(b, out=out), a.fwd_iters))
        for name in variants:
            v = sorted(ts[name])
            res[name + "_us"] = round(v[len(v) // 2], 1)
        res.update({"batch": b, "img_per_s_k14x": round(b / res["k14x_us"] * 1e6, 1)})
        print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", default="14,7")
    ap.add_argument("--imgs", type=int, default=128)
    ap.add_argument("--ks", default="256,512,768,992")
    ap.add_argument("--ldx", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--forward", default="", help="comma list of batch sizes: whole-forward A/B")
    ap.add_argument("--fwd-iters", type=int, default=5)
    ap.add_argument("--min-blocks", type=int, default=1)
    ap.add_argument("--no-layers", action="store_true")
    ap.add_argument("--pf", default="", help="TCAMD_X3_SMALLF_PF for this process (3 or 6)")
    ap.add_argument("--dbg", default="", help="TCAMD_X3_SMALLF_DBG ablation flags (1 no 3x3, 2 X of image 0)")
    ap.add_argument("--wreg", default="", help="TCAMD_X3_SMALLF_WREG for this process (0: W1 by producer "
                                               "LDS copies, 1: consumer fragment loads)")
    ap.add_argument("--stages", default="", help="TCAMD_X3_SMALLF_STAGES for this process (4 or 5)")
    ap.add_argument("--stamp", action="store_true", help="in-kernel timeline marks of one launch per layer")
    a = ap.parse_args()
    if a.pf:
        os.environ["TCAMD_X3_SMALLF_PF"] = a.pf  # read by the library at its first K14x launch
    if a.dbg:
        os.environ["TCAMD_X3_SMALLF_DBG"] = a.dbg
    if a.wreg:
        os.environ["TCAMD_X3_SMALLF_WREG"] = a.wreg
    if a.stages:
        os.environ["TCAMD_X3_SMALLF_STAGES"] = a.stages
    if a.stamp:
        os.environ["TCAMD_X3_SMALLF_STAMP"] = "1"
    import torch

    from triton_client_amd.ops import hip

    hip.lib()
    if not a.no_layers:
        layers(a, torch, hip)
    if a.forward:
        forward(a, torch)


if __name__ == "__main__":
    main()
