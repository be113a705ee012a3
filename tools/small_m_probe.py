#!/usr/bin/env python3
"""Small-batch (bs1) fp32-engine kernel cases, one after another with an idle gap between
cases, for `rocprofv3 --kernel-trace`; tools/trace_groups.py splits the trace at the gaps.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/smallm -o t -- python3 tools/small_m_probe.py
    python3 tools/trace_groups.py gpurun_out/smallm/**/t_kernel_trace.csv
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from triton_client_amd.ops import hip  # noqa: E402


def split(t):
    h = t.to(torch.bfloat16)
    return h.contiguous(), (t - h.float()).to(torch.bfloat16).contiguous()


def main():
    dev = "cuda"
    st = torch.cuda.current_stream().cuda_stream
    imgs = int(os.environ.get("PROBE_IMGS", "1"))
    iters = 30
    cases = []
    for hw in (56, 28, 14, 7):
        M = imgs * hw * hw
        z = torch.relu(torch.randn(M, 128, device=dev))
        zh, zl = split(z)
        wh, wl = split(torch.randn(32, 9 * 128, device=dev) * 0.03)
        y = torch.zeros(M, 256, device=dev)
        cases.append(("conv3x3 hw=%d" % hw, lambda zh=zh, zl=zl, wh=wh, wl=wl, y=y, hw=hw: hip.x3_conv3x3(
            zh.data_ptr(), zl.data_ptr(), imgs, hw, hw, wh.data_ptr(), wl.data_ptr(), y.data_ptr(), 256, stream=st)))
    for hw, K in ((56, 64), (56, 256), (28, 128), (28, 512), (14, 256), (14, 1024), (7, 512), (7, 992)):
        M = imgs * hw * hw
        x = torch.randn(M, K, device=dev)
        s = torch.rand(K, device=dev) + 0.5
        t = torch.randn(K, device=dev) * 0.1
        wh, wl = split(torch.randn(128, K, device=dev) / K ** 0.5)
        b = torch.randn(128, device=dev)
        zh = torch.empty(M, 128, device=dev, dtype=torch.bfloat16)
        zl = torch.empty_like(zh)
        wsb = hip.x3_conv1x1_ws_bytes(M, K, 128)
        ws = torch.empty(max(wsb, 16), device=dev, dtype=torch.uint8)
        cases.append(("conv1x1 hw=%d K=%d" % (hw, K), lambda x=x, K=K, M=M, s=s, t=t, wh=wh, wl=wl, b=b, zh=zh, zl=zl,
                      ws=ws, wsb=wsb: hip.x3_conv1x1(
                          x.data_ptr(), K, M, K, s.data_ptr(), t.data_ptr(), wh.data_ptr(), wl.data_ptr(),
                          out_bias=b.data_ptr(), z_hi=zh.data_ptr(), z_lo=zl.data_ptr(), ws=ws.data_ptr(),
                          ws_bytes=wsb, stream=st)))
    for name, run in cases:
        for _ in range(iters):
            run()
        torch.cuda.synchronize()
        print("case", name, flush=True)
        time.sleep(0.02)


if __name__ == "__main__":
    main()
