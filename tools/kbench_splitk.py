"""Split-K sweep of the K8 1x1 conv on the small-M DenseNet layers.

For each (batch, block, K) shape with few M-tiles, times conv1x1 with
splits 1..8 for the TM=1 variants (plus the heuristic), in a HIP-graph
loop, and reports the best.  Used to set pick_1x1's split rule.

  python tools/kbench_splitk.py --batches 1,8,32,128 --iters 50
"""

import argparse
import json

import torch

from triton_client_amd.ops import hip
from kbench_densenet import cs, timed

SPLITS = (1, 2, 3, 4, 6, 8)
VARS = (11, 12, 21)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,8,32,128")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--max-m", type=int, default=100352)
    a = ap.parse_args()
    dev = "cuda"
    out = []
    blocks = [(56, 64, 6), (28, 128, 12), (14, 256, 24), (7, 512, 16)]
    for b in [int(x) for x in a.batches.split(",")]:
        for hw, c0, n in blocks:
            M = b * hw * hw
            if M > a.max_m:
                continue
            ctot = c0 + 32 * n
            x = torch.randn(M, ctot, device=dev).bfloat16()
            z = torch.empty(M, 128, device=dev).bfloat16()
            ws = torch.empty(max(SPLITS) * M * 128, device=dev, dtype=torch.float32)
            for K in sorted({c0, c0 + 32 * (n // 2), c0 + 32 * (n - 1)}):
                s1 = torch.rand(K, device=dev) + 0.5
                t1 = torch.randn(K, device=dev)
                w = torch.randn(128, K, device=dev).bfloat16()
                bias = torch.randn(128, device=dev)
                row = {"batch": b, "hw": hw, "M": M, "K": K}

                def run(v, s):
                    return timed(lambda: hip.dn_conv1x1(
                        x.data_ptr(), ctot, M, K, s1.data_ptr(), t1.data_ptr(), w.data_ptr(), 128, bias.data_ptr(), 1,
                        z.data_ptr(), 128, variant=v, splits=s, ws=ws.data_ptr(), ws_bytes=ws.numel() * 4,
                        stream=cs()), a.iters)

                row["heuristic"] = round(run(0, 0), 2)
                best = (1e9, None)
                for v in VARS:
                    for s in SPLITS:
                        if s > 1 and s * 32 > K:
                            continue
                        us = run(v, s)
                        row["%d/%d" % (v, s)] = round(us, 2)
                        best = min(best, (us, "%d/%d" % (v, s)))
                row["best"] = best[1]
                row["best_us"] = round(best[0], 2)
                out.append(row)
                print(json.dumps(row), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
