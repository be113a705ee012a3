#!/usr/bin/env python3
"""Where the bf16 bert_large drifts from fp32: per-layer hidden-state rel-L2
of the bf16 model (our fused kernels, and plain torch bf16 ops) against an fp32
forward of the same weights, plus the final start/end logits and argmaxes.

    python tools/bert_accuracy_probe.py --batch 7
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=7)
    ap.add_argument("--seed", type=int, default=108)
    a = ap.parse_args()
    import numpy as np
    import torch

    from triton_client_amd.models import bert

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    from test_bert_accuracy_gpu import _inputs

    ids, mask, tt = (torch.from_numpy(v).cuda() for v in _inputs(a.batch, a.seed))
    m16 = bert.build(device="cuda", dtype=torch.bfloat16)
    m32 = bert.build(device="cuda", dtype=torch.bfloat16).float()

    def run(m, fused):
        bert.FUSED = fused
        hs = []
        hooks = [L.register_forward_hook(lambda mod, i, o: hs.append(o.float())) for L in m.layers]
        with torch.no_grad():
            s, e = m(ids.long(), mask, tt.long())
        for h in hooks:
            h.remove()
        return s.double(), e.double(), hs

    s32, e32, h32 = run(m32, False)
    out = {}
    for name, fused in (("bf16_fused", True), ("bf16_torch", False)):
        s, e, hs = run(m16, fused)
        lay = [float((x - y).norm() / y.norm()) for x, y in zip(hs, h32)]
        rel_s = ((s - s32).norm(dim=1) / s32.norm(dim=1)).cpu().numpy()
        agree = float(np.mean(np.concatenate([(s.argmax(1) == s32.argmax(1)).cpu().numpy(),
                                              (e.argmax(1) == e32.argmax(1)).cpu().numpy()])))
        out[name] = {"layer_rel": [round(v, 5) for v in lay], "start_row_rel": [round(float(v), 4) for v in rel_s],
                     "argmax_agreement": agree}
        print(json.dumps({name: out[name]}), flush=True)


if __name__ == "__main__":
    main()
