#!/usr/bin/env python3
"""K17 (csrc/kernels/gemm.hip) against torch / hipBLASLt on the bert_large
projection shapes, same random bf16 operands, interleaved rounds in one
process (median), PF/s = 2 M N K / time.

    python tools/k17_bench.py --tokens 3072,24576 [--json out.jsonl]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("qkv", 3072, 1024, "none"), ("out", 1024, 1024, "bias"), ("ffn_up", 4096, 1024, "bias_gelu"),
          ("ffn_down", 1024, 4096, "bias")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="384,3072,24576")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default="")
    ap.add_argument("--proj", default="", help="only these projections (comma-separated names)")
    ap.add_argument("--arms", default="k17,hipblaslt", help="k17, k17_t128, k17_t192, k17_t256, hipblaslt (one arm: PMC passes)")
    a = ap.parse_args()
    import torch

    from triton_client_amd.ops import hip

    dev = "cuda"
    st = torch.cuda.current_stream().cuda_stream
    rows = []

    def timeit(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) * 1e3 / a.iters

    for M in [int(v) for v in a.tokens.split(",")]:
        for name, N, K, epi in SHAPES:
            if a.proj and name not in a.proj.split(","):
                continue
            x = torch.empty(M, K, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
            w = (torch.empty(N, K, device=dev, dtype=torch.bfloat16).uniform_(-1, 1) / K ** 0.5).to(torch.bfloat16)
            bias = torch.randn(N, device=dev)
            bias16 = bias.to(torch.bfloat16)
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

            def k17_tm(tm):
                def run():
                    hip.knob_set("TCAMD_K17_TM", tm)
                    hip.k17_gemm(x.data_ptr(), w.data_ptr(), bias.data_ptr(), c.data_ptr(), M, N, K, K, K, N,
                                 epilogue=epi, stream=st)
                return run
            k17 = k17_tm(0)

            if epi == "none":
                def lib():
                    torch.mm(x, w.t())
            elif epi == "bias":
                def lib():
                    torch.addmm(bias16, x, w.t())
            else:
                def lib():
                    torch._addmm_activation(bias16, x, w.t(), use_gelu=True)
            arms = {k: v for k, v in (("k17", k17), ("k17_t128", k17_tm(128)), ("k17_t192", k17_tm(192)),
                                      ("k17_t256", k17_tm(256)), ("hipblaslt", lib)) if k in a.arms.split(",")}
            for f in arms.values():
                f()
            torch.cuda.synchronize()
            ts = {k: [] for k in arms}
            for _ in range(a.rounds):
                for k, f in arms.items():
                    ts[k].append(timeit(f))
            row = {"tokens": M, "proj": name, "N": N, "K": K, "epilogue": epi}
            for k, v in ts.items():
                us = sorted(v)[len(v) // 2]
                row[k + "_us"] = round(us, 1)
                row[k + "_pfs"] = round(2.0 * M * N * K / us / 1e9, 3)
            hip.knob_set("TCAMD_K17_TM", 0)
            k17()
            row["auto_tm"] = hip.k17_last_tm()
            if "k17" in arms and "hipblaslt" in arms:
                row["k17_vs_lib"] = round(row["hipblaslt_us"] / row["k17_us"], 3)
            rows.append(row)
            print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
