#!/usr/bin/env python3
"""K14x (one-kernel dense layer at 14x14 / 7x7) per tiling (tiles per image)
against the K8x + K9x pair, per K and batch, interleaved round by round in
one process (median of the rounds).

    python tools/k14x_bench.py --hw 14,7 --imgs 64,128 --ks 256,512,992 --tiles 1,2,4
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(torch, fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", default="14,7")
    ap.add_argument("--imgs", default="64,128")
    ap.add_argument("--ks", default="256,512,992")
    ap.add_argument("--tiles", default="1,2,4")
    ap.add_argument("--ldx", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    import torch

    from triton_client_amd.ops import hip

    dev = "cuda"
    st = torch.cuda.current_stream().cuda_stream
    rows = []
    for imgs in [int(v) for v in a.imgs.split(",")]:
        for hw in [int(v) for v in a.hw.split(",")]:
            M = imgs * hw * hw
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
                f1 = [hip.x3_w1_fragments(u) for u in (w1h, w1l)]
                zh = torch.empty(M, 128, device=dev, dtype=torch.bfloat16)
                zl = torch.empty_like(zh)
                ws = torch.empty(256 << 20, device=dev, dtype=torch.uint8)
                y = x.data_ptr() + 4 * K

                def pair():
                    hip.x3_dense_layer(x.data_ptr(), ldx, imgs, hw, hw, K, s.data_ptr(), t.data_ptr(),
                                       w1h.data_ptr(), w1l.data_ptr(), b1.data_ptr(), zh.data_ptr(), zl.data_ptr(),
                                       w3[0].data_ptr(), w3[1].data_ptr(), y, ldx, ws=ws.data_ptr(),
                                       ws_bytes=ws.numel(), stream=st)

                def k14(tiles):
                    def run():
                        hip.x3_dense_small(x.data_ptr(), ldx, imgs, hw, hw, K, s.data_ptr(), t.data_ptr(),
                                           f1[0].data_ptr(), f1[1].data_ptr(), b1.data_ptr(), f2[0].data_ptr(),
                                           f2[1].data_ptr(), y, ldx, stream=st, tiles=tiles)
                    return run

                arms = {"pair": pair}
                for tl in [int(v) for v in a.tiles.split(",")]:
                    if not (hw == 14 and tl == 1):
                        arms["t%d" % tl] = k14(tl)
                for f in arms.values():
                    f()
                torch.cuda.synchronize()
                ts = {k: [] for k in arms}
                for _ in range(a.rounds):
                    for k, f in arms.items():
                        ts[k].append(timeit(torch, f, a.iters))
                row = {"hw": hw, "imgs": imgs, "K": K, "default_tiles": hip.x3_small_tiles(imgs, hw)}
                for k, v in ts.items():
                    row[k + "_us"] = round(sorted(v)[len(v) // 2], 2)
                rows.append(row)
                print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
