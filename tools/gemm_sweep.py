#!/usr/bin/env python3
"""bert_large projection GEMMs: hipBLASLt vs K17 vs every K18 tile / split,
timed the way the served model runs them.

Each arm is captured in a HIP graph that runs the projection once per "layer"
over ``--layers`` distinct weight copies (so the weights come from HBM as in
the 24-layer model, not from a cache warmed by the previous launch), replayed
``--rounds`` times interleaved with the other arms; the reported time is the
median per projection.  The N = 1024 projections (attention-out, FFN-down)
are timed together with the residual add + LayerNorm that follows them in the
model: K11 after a bf16 GEMM, or K11p summing a split-K GEMM's fp32 slabs.

    python tools/gemm_sweep.py --tokens 384,3072 [--json out.jsonl]
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
    ap.add_argument("--tokens", default="384,1536,3072,12288,24576")
    ap.add_argument("--layers", type=int, default=0,
                    help="weight copies cycled through (0: enough for 320 MB, past the 256 MB Infinity Cache)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--proj", default="", help="only these projections (comma-separated names)")
    ap.add_argument("--cfgs", default="0,1,2,3,4,5,6,7,8,9")
    ap.add_argument("--splits", default="1,2,4,8")
    ap.add_argument("--no-k17", action="store_true")
    ap.add_argument("--x3", action="store_true",
                    help="the fp32-parity projections: bf16x3 operands (K tripled), fp32 output, erf GELU, fp32 "
                         "LayerNorm (K11p) behind the N = 1024 ones; the library arm is torch.mm + bias (+ GELU)")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    import torch

    from triton_client_amd.ops import hip

    hip.lib()
    dev = "cuda"
    rows_out = []
    cfgs = [int(c) for c in a.cfgs.split(",") if c != ""]
    splits_all = [int(s) for s in a.splits.split(",")]
    for M in [int(v) for v in a.tokens.split(",")]:
        for name, N, K0, epi in SHAPES:
            if a.proj and name not in a.proj.split(","):
                continue
            K = 3 * K0 if a.x3 else K0
            if a.x3 and epi == "bias_gelu":
                epi = "bias_gelu_erf"
            odt = torch.float32 if a.x3 else torch.bfloat16
            L = a.layers or max(4, min(64, -(-320 * 2 ** 20 // (N * K * 2))))
            x = torch.empty(M, K, device=dev, dtype=torch.bfloat16).uniform_(-1, 1)
            ws = [(torch.empty(N, K, device=dev).uniform_(-1, 1) / K ** 0.5).to(torch.bfloat16) for _ in range(L)]
            bias = torch.randn(N, device=dev) * 0.1
            bias16 = bias.to(torch.bfloat16)
            c = torch.empty(M, N, device=dev, dtype=odt)
            ln = N == 1024  # followed by residual add + LayerNorm in the model
            resid = torch.randn(M, N, device=dev).to(odt) if ln else None
            gamma = torch.ones(N, device=dev, dtype=odt)
            beta = torch.zeros(N, device=dev, dtype=odt)
            lnout = torch.empty(M, N, device=dev, dtype=odt)
            maxs = max(splits_all)
            part = torch.empty(maxs, M, N, device=dev) if ln else None

            def st():
                return torch.cuda.current_stream().cuda_stream

            def k11(y):
                if a.x3:
                    hip.add_layernorm_parts(resid.data_ptr(), y.data_ptr(), 1, M * N, None, gamma.data_ptr(),
                                            beta.data_ptr(), lnout.data_ptr(), M, N, 1e-12, f32=True, stream=st())
                    return
                hip.add_layernorm(resid.data_ptr(), y.data_ptr(), gamma.data_ptr(), beta.data_ptr(), lnout.data_ptr(),
                                  M, N, 1e-12, stream=st())

            def lib_arm(w):
                if a.x3:
                    y = torch.mm(x, w.t(), out_dtype=torch.float32)
                    if epi != "none":
                        y += bias
                    if epi == "bias_gelu_erf":
                        y = torch.nn.functional.gelu(y)
                    if ln:
                        k11(y)
                    return
                if epi == "none":
                    torch.mm(x, w.t(), out=c)
                elif epi == "bias":
                    torch.addmm(bias16, x, w.t(), out=c)
                else:
                    torch._addmm_activation(bias16, x, w.t(), use_gelu=True)
                if ln:
                    k11(c)

            def k17_static_arm(w):
                with hip.knob(TCAMD_K17_DYN=0):
                    k17_arm(w)

            def k17_arm(w):
                hip.k17_gemm(x.data_ptr(), w.data_ptr(), bias.data_ptr(), c.data_ptr(), M, N, K, K, K, N,
                             epilogue=epi, out_f32=a.x3, stream=st())
                if ln:
                    k11(c)

            def k18_arm(cfg, s):
                def run(w):
                    if s == 1:
                        hip.k18_gemm(x.data_ptr(), w.data_ptr(), bias.data_ptr(), c.data_ptr(), M, N, K, K, K, N,
                                     epilogue=epi, out_f32=a.x3, cfg=cfg, stream=st())
                        if ln:
                            k11(c)
                    else:
                        hip.k18_gemm(x.data_ptr(), w.data_ptr(), None, part.data_ptr(), M, N, K, K, K, N,
                                     out_f32=True, cfg=cfg, splits=s, split_stride=M * N, stream=st())
                        hip.add_layernorm_parts(resid.data_ptr(), part.data_ptr(), s, M * N, bias.data_ptr(),
                                                gamma.data_ptr(), beta.data_ptr(), lnout.data_ptr(), M, N, 1e-12,
                                                f32=a.x3, stream=st())
                return run

            arms = {"hipblaslt": lib_arm}
            if not a.no_k17 and N % 256 == 0:
                arms["k17"] = k17_arm
                arms["k17_static"] = k17_static_arm
            for cfg in cfgs:
                tm, tn, _, _ = hip.k18_cfg(cfg)
                if N % tn:
                    continue
                for s in splits_all:
                    if (s > 1 and not ln) or K % (64 * s):
                        continue
                    arms["k18_c%d_s%d" % (cfg, s)] = k18_arm(cfg, s)
            graphs = {}
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for k, f in arms.items():
                    for w in ws[:2]:
                        f(w)
                    torch.cuda.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=s):
                        for w in ws:
                            f(w)
                    graphs[k] = g
            torch.cuda.synchronize()
            ts = {k: [] for k in arms}
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(a.rounds):
                for k, g in graphs.items():
                    g.replay()  # warm
                    ev0.record()
                    g.replay()
                    ev1.record()
                    ev1.synchronize()
                    ts[k].append(ev0.elapsed_time(ev1) * 1e3 / L)
            row = {"tokens": M, "proj": name, "N": N, "K": K, "epilogue": epi, "with_ln": ln, "x3": a.x3}
            for k, v in ts.items():
                row[k + "_us"] = round(sorted(v)[len(v) // 2], 2)
            best = min((k for k in arms if k != "hipblaslt"), key=lambda k: row[k + "_us"])
            row["best"] = best
            row["best_vs_lib"] = round(row["hipblaslt_us"] / row[best + "_us"], 3)
            rows_out.append(row)
            print(json.dumps(row), flush=True)
            del graphs
            torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            for r in rows_out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
