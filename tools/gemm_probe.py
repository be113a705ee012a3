#!/usr/bin/env python3
"""K15 bf16 GEMM (csrc/kernels/gemm.hip) against torch.mm (hipBLASLt) on the
BERT-large projection shapes, interleaved rounds in one process; PF/s from the
median.  Random operands (zero-filled ones read high: the clock rises).

    python tools/gemm_probe.py --tokens 24576 --rounds 7
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="24576,3072")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variant", default="", help="run this TCAMD_GEMM_V in a child (1, 2) and print its rows")
    a = ap.parse_args()
    if a.variant:
        os.environ["TCAMD_GEMM_V"] = a.variant  # read by the library at its first GEMM
    import torch
    import torch.nn.functional as F

    from triton_client_amd.ops import hip

    st = torch.cuda.current_stream().cuda_stream
    shapes = [("qkv", 3072, 1024, "none"), ("out", 1024, 1024, "bias"), ("ffn_up", 4096, 1024, "bias_gelu"),
              ("ffn_down", 1024, 4096, "bias")]

    def t_us(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) * 1e3 / a.iters

    for M in [int(v) for v in a.tokens.split(",")]:
        for name, N, K, epi in shapes:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
            bias = torch.randn(N, device="cuda").to(torch.bfloat16)
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

            def ours():
                hip.gemm_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), M, N, K, bias=bias.data_ptr(), epilogue=epi,
                              stream=st)

            def lib():
                if epi == "none":
                    torch.mm(x, w.t(), out=y)
                elif epi == "bias_gelu":
                    torch._addmm_activation(bias, x, w.t(), use_gelu=True)
                else:
                    torch.addmm(bias, x, w.t(), out=y)

            to, tl = [], []
            for _ in range(a.rounds):
                to.append(t_us(ours))
                tl.append(t_us(lib))
            to.sort()
            tl.sort()
            fl = 2.0 * M * N * K
            mo, ml = to[len(to) // 2], tl[len(tl) // 2]
            print(json.dumps({"variant": os.environ.get("TCAMD_GEMM_V", "1"), "tokens": M, "gemm": name, "N": N, "K": K, "epilogue": epi, "k15_us": round(mo, 1),
                              "hipblaslt_us": round(ml, 1), "k15_PFps": round(fl / mo / 1e9, 3),
                              "hipblaslt_PFps": round(fl / ml / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
