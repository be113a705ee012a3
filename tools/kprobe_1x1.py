"""Launch one K8/K8p 1x1-conv shape repeatedly (for rocprofv3 --pmc passes).

  python tools/kprobe_1x1.py --M 6272 --K 992 --ldx 1024 --variant 12 --iters 200
"""

import argparse

import torch

from triton_client_amd.ops import hip


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=6272)
    ap.add_argument("--K", type=int, default=992)
    ap.add_argument("--ldx", type=int, default=1024)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    dev = "cuda"
    x = torch.randn(a.M, a.ldx, device=dev).bfloat16()
    s1 = torch.rand(a.K, device=dev) + 0.5
    t1 = torch.randn(a.K, device=dev)
    w = torch.randn(128, a.K, device=dev).bfloat16()
    bias = torch.randn(128, device=dev)
    z = torch.empty(a.M, 128, device=dev).bfloat16()
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(a.iters):
        hip.dn_conv1x1(x.data_ptr(), a.ldx, a.M, a.K, s1.data_ptr(), t1.data_ptr(), w.data_ptr(), 128, bias.data_ptr(),
                       1, z.data_ptr(), 128, variant=a.variant, stream=st)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
