#!/usr/bin/env python3
"""Run-to-run spread of the fp32 engine's logits (float-atomic ordering in the
small-M layers): N eager forwards of the same input per batch size, max abs /
rel-L2 difference against the first, and the error vs the fp32 module.

    python tools/engine_repeat.py --batches 1,2,8 --n 5
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,2,8")
    ap.add_argument("--n", type=int, default=5)
    a = ap.parse_args()
    import torch

    from triton_client_amd.models import densenet_fp32

    bs = [int(b) for b in a.batches.split(",")]
    eng, model = densenet_fp32.build(max(bs), device="cuda")
    model = model.cuda().float()
    for b in bs:
        x = torch.randn(b, 3, 224, 224, device="cuda", generator=torch.Generator(device="cuda").manual_seed(b))
        with torch.no_grad():
            ref = model(x).double()
            outs = [eng(x).double().clone() for _ in range(a.n)]
        d = [((o - outs[0]).abs().max().item(), ((o - outs[0]).norm() / outs[0].norm()).item()) for o in outs[1:]]
        err = ((outs[0] - ref).norm() / ref.norm()).item()
        print("b=%d vs fp32 module %.3g | run-to-run max abs %s rel %s" % (
            b, err, " ".join("%.2g" % v[0] for v in d), " ".join("%.2g" % v[1] for v in d)), flush=True)


if __name__ == "__main__":
    main()
