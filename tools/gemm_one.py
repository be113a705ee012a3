"""Run one K15 GEMM shape a few times (for rocprofv3 --pmc passes):
python tools/gemm_one.py --M 24576 --N 4096 --K 1024 --epi bias_gelu --iters 10
(TCAMD_GEMM_V picks the variant)."""
import argparse

import torch

from triton_client_amd.ops import hip

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=24576)
ap.add_argument("--N", type=int, default=4096)
ap.add_argument("--K", type=int, default=1024)
ap.add_argument("--epi", default="bias_gelu")
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
x = torch.randn(a.M, a.K, device="cuda").to(torch.bfloat16)
w = (torch.randn(a.N, a.K, device="cuda") / a.K ** 0.5).to(torch.bfloat16)
b = torch.randn(a.N, device="cuda").to(torch.bfloat16)
r = torch.randn(a.M, a.N, device="cuda").to(torch.bfloat16)
y = torch.empty(a.M, a.N, device="cuda", dtype=torch.bfloat16)
for _ in range(a.iters):
    hip.gemm_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), a.M, a.N, a.K, bias=b.data_ptr(), residual=r.data_ptr(),
                  epilogue=a.epi)
torch.cuda.synchronize()
print("ok")
