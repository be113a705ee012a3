"""K15 (csrc/kernels/gemm.hip): the hand-written bf16 projection GEMM with
fused epilogues, against a plain PyTorch fp32 matmul of the same bf16
operands.  Shapes: the four BERT-large projections at several token counts
(ragged M included: M is tokens = batch x 384), every epilogue, and leading
dimensions wider than the operands (views into bigger buffers)."""

import pytest

torch = pytest.importorskip("torch")
F = torch.nn.functional

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _ref(x, w, bias, r, epi):
    y = x.float() @ w.float().t()
    if epi != "none":
        y = y + bias.float()
    if epi == "bias_gelu":
        y = F.gelu(y)  # erf form, as BERT (and torch's addmm GELU epilogue)
    if epi == "bias_residual":
        y = y + r.float()
    return y


@pytest.mark.parametrize("M,N,K", [(384, 3072, 1024), (1000, 1024, 1024), (3072, 4096, 1024), (768, 1024, 4096),
                                   (24576, 1024, 1024), (256, 256, 64), (130, 512, 128),
                                   (8200, 2048, 128)])
@pytest.mark.parametrize("epi", ["none", "bias", "bias_gelu", "bias_residual"])
def test_gemm_bf16_matches_fp32_reference(M, N, K, epi):
    _need_gpu()
    from triton_client_amd.ops import hip

    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + K)
    x = (torch.randn(M, K, device=DEV, generator=g)).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, generator=g) / K ** 0.5).to(torch.bfloat16)
    bias = (torch.randn(N, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
    r = torch.randn(M, N, device=DEV, generator=g).to(torch.bfloat16)
    y = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    hip.gemm_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), M, N, K, bias=bias.data_ptr(), residual=r.data_ptr(),
                  epilogue=epi, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = _ref(x, w, bias, r, epi)
    assert torch.isfinite(y).all()
    err = ((y.float() - ref).norm() / ref.norm()).item()
    # bf16 output: ~2^-9 relative per element
    assert err < 4e-3, err
    worst = ((y.float() - ref).abs() / (ref.abs() + 0.05)).max().item()
    assert worst < 3e-2, worst


def test_gemm_bf16_strided_views_and_torch_parity():
    """ld > K / N: operands are column slices of wider buffers (the QKV output
    is consumed by K12 in place); and the result equals torch's bf16 matmul to
    bf16 rounding."""
    _need_gpu()
    from triton_client_amd.ops import hip

    M, N, K = 1536, 1024, 1024
    g = torch.Generator(device=DEV).manual_seed(3)
    xb = torch.randn(M, K + 64, device=DEV, generator=g).to(torch.bfloat16)
    wb = (torch.randn(N, K + 128, device=DEV, generator=g) / 32).to(torch.bfloat16)
    yb = torch.zeros(M, N + 256, device=DEV, dtype=torch.bfloat16)
    x, w = xb[:, :K], wb[:, :K]
    hip.gemm_bf16(x.data_ptr(), w.data_ptr(), yb.data_ptr(), M, N, K, ldx=K + 64, ldw=K + 128, ldy=N + 256,
                  stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = x.float() @ w.float().t()
    assert ((yb[:, :N].float() - ref).norm() / ref.norm()).item() < 4e-3
    assert (yb[:, N:] == 0).all()
    tb = torch.mm(x, w.t())
    assert ((yb[:, :N].float() - tb.float()).norm() / tb.float().norm()).item() < 4e-3


def test_gemm_bf16_rejects_bad_shapes():
    _need_gpu()
    from triton_client_amd.ops import hip

    t = torch.zeros(4096, device=DEV, dtype=torch.bfloat16)
    for M, N, K in [(16, 100, 64), (16, 256, 60)]:
        with pytest.raises(Exception):
            hip.gemm_bf16(t.data_ptr(), t.data_ptr(), t.data_ptr(), M, N, K)
    with pytest.raises(Exception):  # bias epilogue without a bias
        hip.gemm_bf16(t.data_ptr(), t.data_ptr(), t.data_ptr(), 16, 256, 64, epilogue="bias")


@pytest.mark.parametrize("variant", ["1", "2", "3", "4", "5", "7", "8", "9", "10", "11"])
def test_gemm_bf16_phased_variant_matches(tmp_path, variant):
    """TCAMD_GEMM_V=2 (4 phases per K step, counted vmcnt across barriers) and 3
    (the same with the two wave groups one phase apart) in a child process (the variant is chosen once per process): same results as
    the fp32 reference on every epilogue, including K = 64 (one step: the last
    step's wait counts) and K = 4096."""
    _need_gpu()
    import os
    import subprocess
    import sys

    code = r'''
import torch, torch.nn.functional as F
from triton_client_amd.ops import hip
for (M, N, K) in [(512, 256, 64), (1000, 1024, 1024), (768, 1024, 4096), (384, 3072, 1024)]:
    for epi in ["none", "bias", "bias_gelu", "bias_residual"]:
        g = torch.Generator(device="cuda").manual_seed(M + N + K)
        x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
        r = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        hip.gemm_bf16(x.data_ptr(), w.data_ptr(), y.data_ptr(), M, N, K, bias=b.data_ptr(), residual=r.data_ptr(),
                      epilogue=epi)
        torch.cuda.synchronize()
        ref = x.float() @ w.float().t()
        if epi != "none":
            ref = ref + b.float()
        if epi == "bias_gelu":
            ref = F.gelu(ref)
        if epi == "bias_residual":
            ref = ref + r.float()
        err = ((y.float() - ref).norm() / ref.norm()).item()
        assert err < 4e-3, (M, N, K, epi, err)
print("PHASED_OK")
'''
    env = dict(os.environ, TCAMD_GEMM_V=variant)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "PHASED_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
