#!/usr/bin/env python3
"""bf16 bert_large: do the serving paths agree bit for bit?  (a) K12 masked
with an all-ones mask vs K12 unmasked on the same qkv; (b) the whole model,
eager masked vs eager dense on all-ones masks; (c) eager vs HIP-graph replay
at batch 1 and 8."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


def main():
    import torch

    from triton_client_amd.models import bert
    from triton_client_amd.ops import hip

    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    out = {}
    for b in (1, 8):
        qkv = (torch.randn(b * 384, 3 * 1024, device=dev) * 0.5).to(torch.bfloat16)
        mask = torch.ones(b, 384, device=dev, dtype=torch.int32)
        o1 = torch.empty(b * 384, 1024, device=dev, dtype=torch.bfloat16)
        o2 = torch.empty_like(o1)
        hip.attention(qkv.data_ptr(), mask.data_ptr(), o1.data_ptr(), b, 384, 16, 0.125, stream=st)
        hip.attention(qkv.data_ptr(), None, o2.data_ptr(), b, 384, 16, 0.125, stream=st)
        q, k, v = qkv.float().view(b, 384, 3, 16, 64).permute(2, 0, 3, 1, 4)
        ref = torch.nn.functional.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(b * 384, 1024)
        torch.cuda.synchronize()
        out["k12_b%d" % b] = {"masked_vs_unmasked": rel(o1, o2), "masked_vs_fp32": rel(o1, ref),
                              "unmasked_vs_fp32": rel(o2, ref)}
    m = bert.build(device=dev)
    for b in (1, 8):
        ids = torch.randint(1000, 30000, (b, 384), device=dev)
        mask = torch.ones(b, 384, device=dev, dtype=torch.int32)
        tt = torch.zeros(b, 384, device=dev, dtype=torch.long)
        with torch.no_grad():
            sm, _ = m(ids, mask, tt)
            sd, _ = m(ids, mask, tt, dense=True)
            s2 = torch.cuda.Stream()
            with torch.cuda.stream(s2):
                m(ids, mask, tt)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s2):
                    sg, _ = m(ids, mask, tt)
            g.replay()
            torch.cuda.synchronize()
        out["model_b%d" % b] = {"masked_vs_dense": rel(sm, sd), "eager_vs_graph": rel(sm, sg)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
