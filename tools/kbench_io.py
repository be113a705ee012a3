#!/usr/bin/env python3
"""Achieved bandwidth of the client-side data kernels
against MI355X HBM3E (8 TB/s spec, ~6.3 TB/s measured copy ceiling), at the
densenet bs=8 request size (4.8 MB) and at 1 GB:

  K1 synth_fill FP32 (uniform)            writes N
  K2 pack_bytes (16-B chunk emitter)      reads payload + lens, writes stream
  K3 index_bytes (parallel block walk)    reads stream, writes offs/lens
  K4 convert FP32 -> BF16 (RNE)           reads N, writes N/2
  K5 convert FP32 -> FP8 e4m3             reads N, writes N/4
  K6 layout_pack NCHW fp32 -> NHWC bf16   reads N, writes N/2 (LDS-tiled transpose)
  K7 batched_copy (8 segments)            reads N, writes N
  ref: torch copy_ (hipMemcpy D2D)        reads N, writes N

One JSON line per (kernel, size); run under rocprofv3 --kernel-trace --stats
for the per-kernel table (LDS_Block_Size shows the LDS staging).

    python tools/kbench_io.py --sizes 4.8e6,1e9 --iters 20
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4.8e6,1e9", help="fp32 source bytes per case")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    import numpy as np
    import torch

    from triton_client_amd.ops import hip

    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    s = st.cuda_stream
    rows = []

    def bench(name, nbytes_moved, fn, size):
        if args.only and args.only not in name:
            return
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000.0 / args.iters
        r = {"kernel": name, "src_bytes": int(size), "bytes_moved": int(nbytes_moved), "us": round(us, 2),
             "GBps": round(nbytes_moved / us / 1e3, 1), "pct_of_8TBps": round(100 * nbytes_moved / us / 8e6, 1)}
        rows.append(r)
        print(json.dumps(r), flush=True)

    for size in [float(x) for x in args.sizes.split(",")]:
        n = int(size) // 4 // 16 * 16  # fp32 elements, 64-B multiple
        nb = n * 4
        src = torch.empty(n, device="cuda", dtype=torch.float32)
        hip.synth_fill(src.data_ptr(), n, "FP32", hip.SYNTH_NORMAL, 0.0, 1.0, seed=1, stream=s)
        dst = torch.empty(nb, device="cuda", dtype=torch.uint8)
        bench("K1 synth_fill FP32", nb, lambda: hip.synth_fill(dst.data_ptr(), n, "FP32", hip.SYNTH_UNIFORM, 0.0, 1.0,
                                                                 seed=3, stream=s), size)
        bench("K4 convert FP32->BF16", nb + nb // 2,
              lambda: hip.convert(src.data_ptr(), "FP32", dst.data_ptr(), "BF16", n, rounding="rne", stream=s), size)
        bench("K5 convert FP32->FP8E4M3", nb + nb // 4,
              lambda: hip.convert(src.data_ptr(), "FP32", dst.data_ptr(), "FP8_E4M3", n, rounding="rne", stream=s),
              size)
        # K6: images of 3x224x224 (the densenet request tensor), as many as fit
        img = 3 * 224 * 224
        nimg = max(1, n // img)
        srcs = [src.data_ptr() + i * img * 4 for i in range(nimg)]
        bench("K6 layout_pack NCHW fp32->NHWC bf16", nimg * img * 6,
              lambda: hip.layout_pack(srcs, "FP32", "NCHW", dst.data_ptr(), "BF16", "NHWC", 3, 224, 224, stream=s),
              size)
        seg = nb // 8 // 256 * 256
        bench("K7 batched_copy x8", 2 * 8 * seg,
              lambda: hip.batched_copy([src.data_ptr() + i * seg for i in range(8)],
                                       [dst.data_ptr() + i * seg for i in range(8)], [seg] * 8, stream=s), size)
        bench("ref torch D2D copy_", 2 * nb, lambda: dst.view(torch.float32)[:n].copy_(src), size)
        # K2 / K3: strings of 0..40 bytes (mean 20) totalling ~size bytes
        ne = max(1024, int(size) // 24)
        rng = np.random.default_rng(7)
        lens = rng.integers(0, 41, ne).astype(np.uint32)
        payload_n = int(lens.sum())
        d_payload = torch.randint(0, 256, (max(16, payload_n),), device="cuda", dtype=torch.uint8)
        d_lens = torch.from_numpy(lens.view(np.int32)).cuda()
        total = payload_n + 4 * ne
        packed = torch.empty(total + 16, device="cuda", dtype=torch.uint8)
        ws = torch.empty(hip.pack_bytes_workspace(ne), device="cuda", dtype=torch.uint8)
        bench("K2 pack_bytes (mean 20 B strings)", payload_n + 4 * ne + total,
              lambda: hip.pack_bytes(d_payload.data_ptr(), d_lens.data_ptr(), ne, packed.data_ptr(), ws.data_ptr(), s),
              size)
        offs = torch.empty(ne, device="cuda", dtype=torch.int64)
        lns = torch.empty(ne, device="cuda", dtype=torch.int32)
        status = torch.zeros(4, device="cuda", dtype=torch.int32)
        bench("K3 index_bytes (mean 20 B strings)", total + 12 * ne,
              lambda: hip.index_bytes(packed.data_ptr(), total, ne, offs.data_ptr(), lns.data_ptr(),
                                      status.data_ptr(), s), size)
        assert int(status[0]) == 0
        del src, dst, d_payload, packed, ws, offs, lns
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
