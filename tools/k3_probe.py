#!/usr/bin/env python3
"""K3 index_bytes probe: which path ran (serial / v3 / general), the scan
window, and the wall time per call, for the kbench_io.py data shape (binary
strings of 0..40 bytes) and a few others.  Run under rocprofv3 --kernel-trace
--stats for the per-kernel split.

    python tools/k3_probe.py --sizes 4.8e6,1e9
"""

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4.8e6,1e8")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--maxlen", type=int, default=40)
    args = ap.parse_args()
    import numpy as np
    import torch

    from triton_client_amd.ops import hip

    s = torch.cuda.current_stream().cuda_stream
    for size in [float(x) for x in args.sizes.split(",")]:
        ne = max(1024, int(size) // 24)
        rng = np.random.default_rng(7)
        lens = rng.integers(0, args.maxlen + 1, ne).astype(np.uint32)
        payload_n = int(lens.sum())
        d_payload = torch.randint(0, 256, (max(16, payload_n),), device="cuda", dtype=torch.uint8)
        d_lens = torch.from_numpy(lens.view(np.int32)).cuda()
        total = payload_n + 4 * ne
        packed = torch.empty(total + 16, device="cuda", dtype=torch.uint8)
        ws = torch.empty(hip.pack_bytes_workspace(ne), device="cuda", dtype=torch.uint8)
        hip.pack_bytes(d_payload.data_ptr(), d_lens.data_ptr(), ne, packed.data_ptr(), ws.data_ptr(), s)
        offs = torch.empty(ne, device="cuda", dtype=torch.int64)
        lns = torch.empty(ne, device="cuda", dtype=torch.int32)
        status = torch.zeros(4, device="cuda", dtype=torch.int32)
        torch.cuda.synchronize()
        for it in range(args.iters):
            t0 = time.perf_counter()
            hip.index_bytes(packed.data_ptr(), total, ne, offs.data_ptr(), lns.data_ptr(), status.data_ptr(), s)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            path, window = hip.index_bytes_last_path()
            print("size %.3g n %d: status %d path %d window %d  %.1f us  %.1f GB/s" % (
                size, ne, int(status[0]), path, window, dt * 1e6, total / dt / 1e9), flush=True)
        ok = np.array_equal(lns.cpu().numpy().view(np.uint32), lens)
        exp_offs = np.concatenate([[0], np.cumsum(lens.astype(np.int64) + 4)[:-1]]) + 4
        ok_o = np.array_equal(offs.cpu().numpy(), exp_offs)
        print("lens match:", ok, "offsets match:", ok_o, flush=True)


if __name__ == "__main__":
    main()
