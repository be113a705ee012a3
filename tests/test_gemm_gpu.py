"""K17 (csrc/kernels/gemm.hip): bf16 GEMM C = A . B^T (+ bias) (GELU) for the
bert_large projections, against an fp32 torch matmul of the same bf16
operands.  Shapes: the four bert projections at 384 and 3,072 tokens, ragged
M (row tails inside a 256-row tile), a single K slab, K not a multiple of
the 3-slab prefetch, strided A / B / C (the ldc padding and the rows past M
must stay untouched), and the fp32-output form the fp32-parity bert uses."""

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _hip():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from triton_client_amd.ops import hip

    hip.lib()
    return hip


def _gelu(x):
    """The tanh form K17 computes (as hipBLASLt's GELU epilogue does); the erf
    form differs by up to 5e-4, which is 3e-2 of a -0.004 output at x = -3."""
    return torch.nn.functional.gelu(x, approximate="tanh")


def _case(M, N, K, lda=None, ldb=None, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed + M + N + K)
    lda, ldb = lda or K, ldb or K
    a = (torch.randn(M, lda, device=DEV, generator=g)).to(torch.bfloat16)
    b = (torch.randn(N, ldb, device=DEV, generator=g) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV, generator=g) * 0.5
    return a, b, bias


@pytest.mark.parametrize("M,N,K", [(384, 3072, 1024), (384, 1024, 1024), (384, 4096, 1024), (384, 1024, 4096),
                                   (3072, 1024, 1024), (300, 256, 64), (1, 256, 32), (517, 512, 96),
                                   (256, 768, 160), (1000, 1280, 2048)])
@pytest.mark.parametrize("epi", ["none", "bias", "bias_gelu"])
@pytest.mark.parametrize("tm", [128, 192, 256])
def test_k17_gemm_bf16_out(M, N, K, epi, tm):
    """Both tile heights (TCAMD_K17_TM; by default picked from how evenly the
    tiles fill the CUs)."""
    hip = _hip()
    a, b, bias = _case(M, N, K)
    ldc = N + 64
    c = torch.full((M + 3, ldc), 7.0, device=DEV, dtype=torch.bfloat16)
    with hip.knob(TCAMD_K17_TM=tm):
        hip.k17_gemm(a.data_ptr(), b.data_ptr(), bias.data_ptr(), c.data_ptr(), M, N, K, K, K, ldc, epilogue=epi,
                     stream=torch.cuda.current_stream().cuda_stream)
        assert hip.k17_last_tm() == tm
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t()
    if epi != "none":
        ref = ref + bias
    if epi == "bias_gelu":
        ref = _gelu(ref)
    got = c[:M, :N].float()
    err = ((got - ref).norm() / ref.norm()).item()
    worst = ((got - ref).abs() / (ref.abs() + 1e-2)).max().item()
    print("K17 M %d N %d K %d %s tm %d: rel-L2 %.3g, worst elementwise %.3g" % (M, N, K, epi, tm, err, worst))
    assert err < 6e-3 and worst < 3e-2  # bf16 output rounding (2^-9 relative)
    assert (c[:M, N:] == 7.0).all() and (c[M:] == 7.0).all(), "wrote outside C[:M, :N]"


@pytest.mark.parametrize("M,N,K,lda,ldb", [(384, 1024, 3072, 3072, 3072), (777, 512, 192, 256, 200)])
@pytest.mark.parametrize("epi", ["none", "bias"])
@pytest.mark.parametrize("tm", [128, 192, 256])
def test_k17_gemm_fp32_out_strided(M, N, K, lda, ldb, epi, tm):
    """fp32 output (the fp32-parity bert's [x_hi|x_hi|x_lo] . [W_hi|W_lo|W_hi]
    GEMM, K = 3 x hidden) and row strides larger than K."""
    hip = _hip()
    a, b, bias = _case(M, N, K, lda, ldb, seed=1)
    c = torch.full((M + 1, N + 8), 7.0, device=DEV)
    with hip.knob(TCAMD_K17_TM=tm):
        hip.k17_gemm(a.data_ptr(), b.data_ptr(), bias.data_ptr(), c.data_ptr(), M, N, K, lda, ldb, N + 8,
                     epilogue=epi, out_f32=True, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = a[:, :K].double() @ b[:, :K].double().t()
    if epi == "bias":
        ref = ref + bias.double()
    err = ((c[:M, :N].double() - ref).norm() / ref.norm()).item()
    assert err < 1e-5, err  # fp32 accumulation of exact bf16 products
    assert (c[:M, N:] == 7.0).all() and (c[M:] == 7.0).all()


def test_k17_gemm_rejects_bad_shapes():
    hip = _hip()
    x = torch.zeros(4096, device=DEV, dtype=torch.bfloat16)
    for M, N, K, lda, ldb, ldc in [(8, 100, 64, 64, 64, 100), (8, 256, 48, 48, 48, 256), (8, 256, 64, 32, 64, 256),
                                   (8, 256, 64, 64, 64, 128), (8, 256, 64, 66, 64, 256)]:
        with pytest.raises(Exception):
            hip.k17_gemm(x.data_ptr(), x.data_ptr(), None, x.data_ptr(), M, N, K, lda, ldb, ldc)
    with pytest.raises(Exception):  # bias epilogue without a bias
        hip.k17_gemm(x.data_ptr(), x.data_ptr(), None, x.data_ptr(), 8, 256, 64, 64, 64, 256, epilogue="bias")


def test_bert_projections_k17_vs_library(monkeypatch):
    """bert's _proj routes the QKV (no epilogue) and FFN-up + GELU projections
    from TC_BERT_K17_MIN_TOKENS tokens and the attention-out projection (bias,
    <= 3,072 tokens) through K17 (TC_BERT_K17=1), the rest through hipBLASLt;
    each routed projection agrees with the library path to bf16 rounding
    (both compute the tanh form of GELU)."""
    hip = _hip()
    from triton_client_amd.models import bert

    g = torch.Generator(device=DEV).manual_seed(5)
    big = bert.K17_MIN_TOKENS
    for tokens in (384, 3072, big):
        x = torch.randn(tokens, 1024, device=DEV, generator=g).to(torch.bfloat16)
        for N, K, epi in ((3072, 1024, "none"), (1024, 1024, "bias"), (4096, 1024, "bias_gelu"),
                          (1024, 4096, "bias")):
            routed = tokens >= big if epi in ("none", "bias_gelu") else (K == 1024 and tokens <= 3072)
            lin = torch.nn.Linear(K, N).to(DEV, torch.bfloat16)
            xin = x if K == 1024 else torch.randn(tokens, K, device=DEV, generator=g).to(torch.bfloat16)
            assert bert._k17_takes(tokens, N, K, epi) == routed, (tokens, N, K, epi)
            monkeypatch.setattr(bert, "K17", True)
            before = hip.k17_calls()
            got = bert._proj(xin, lin, epi).float()
            assert hip.k17_calls() - before == (1 if routed else 0)
            monkeypatch.setattr(bert, "K17", False)
            ref = bert._proj(xin, lin, epi).float()
            torch.cuda.synchronize()
            err = ((got - ref).norm() / ref.norm()).item()
            assert err < 8e-3, (tokens, N, epi, err)
