"""Stem micro-benchmark on one MI355X: the fused K10s kernel (fp32 NCHW via the
pointer table, and bf16 NHWC) against the path it replaced (K6 layout_pack
fp32 NCHW -> bf16 NHWC, library 7x7/2 conv, K10a bias+ReLU+max-pool).

  python tools/kbench_stem.py --batches 1,8,128 --iters 50
"""

import argparse
import json

import torch
import torch.nn.functional as F


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,8,128")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from triton_client_amd.ops import hip

    dev = torch.device("cuda", 0)
    w = torch.randn(64, 3, 7, 7, device=dev) * 0.1
    wl = w.bfloat16().contiguous(memory_format=torch.channels_last)
    wp = torch.zeros(64, 7, 8, 4, device=dev)
    wp[:, :, :7, :3] = w.permute(0, 2, 3, 1)
    wp = wp.reshape(64, -1).bfloat16().contiguous()
    bias = torch.randn(64, device=dev)
    res = {}
    for b in [int(x) for x in a.batches.split(",")]:
        x = torch.randn(b, 3, 224, 224, device=dev)
        tbl = torch.tensor([x[i].data_ptr() for i in range(b)], device=dev, dtype=torch.int64)
        xn = x.bfloat16().permute(0, 2, 3, 1).contiguous()
        nhwc = torch.empty(b, 224, 224, 3, device=dev, dtype=torch.bfloat16)
        y = torch.empty(b * 56 * 56, 256, device=dev, dtype=torch.bfloat16)
        st = torch.cuda.current_stream().cuda_stream
        srcs = [x[i].data_ptr() for i in range(b)]

        def fused_f32():
            hip.dn_stem_fused(tbl.data_ptr(), None, wp.data_ptr(), bias.data_ptr(), y.data_ptr(), b, 256, stream=st)

        def fused_bf16():
            hip.dn_stem_fused(None, xn.data_ptr(), wp.data_ptr(), bias.data_ptr(), y.data_ptr(), b, 256, stream=st)

        def old_path():
            hip.layout_pack(srcs, "FP32", "NCHW", nhwc.data_ptr(), "BF16", "NHWC", 3, 224, 224, stream=st)
            y0 = F.conv2d(nhwc.permute(0, 3, 1, 2), wl, stride=2, padding=3)
            y0 = y0.contiguous(memory_format=torch.channels_last)
            hip.dn_stem_pool(y0.data_ptr(), bias.data_ptr(), y.data_ptr(), b, 112, 112, 64, 256, stream=st)

        r = {"fused_fp32_ptrs_us": timed(fused_f32, a.iters), "fused_bf16_nhwc_us": timed(fused_bf16, a.iters),
             "pack_conv_pool_us": timed(old_path, a.iters)}
        res[b] = r
        print(b, json.dumps(r), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
