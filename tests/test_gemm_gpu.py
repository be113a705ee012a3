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


@pytest.mark.parametrize("tokens", [384, 768, 1536, 3072, 12288])
def test_bert_projection_routes(monkeypatch, tokens):
    """Every bert projection through every routing mode (TC_BERT_GEMM): the
    routed kernel is the one gemm_route names (launch counters), and each
    agrees with the hipBLASLt path to bf16 rounding -- the N = 1024
    projections together with the residual add + LayerNorm they feed, so the
    split-K slabs summed by K11p are covered."""
    hip = _hip()
    from triton_client_amd.models import bert

    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(tokens, 1024, device=DEV, generator=g).to(torch.bfloat16)
    resid = torch.randn(tokens, 1024, device=DEV, generator=g).to(torch.bfloat16)
    ln = torch.nn.LayerNorm(1024, eps=1e-12).to(DEV, torch.bfloat16)
    for name, N, K, epi in (("qkv", 3072, 1024, "none"), ("out", 1024, 1024, "bias"),
                            ("ffn_up", 4096, 1024, "bias_gelu"), ("ffn_down", 1024, 4096, "bias")):
        lin = torch.nn.Linear(K, N).to(DEV, torch.bfloat16)
        with torch.no_grad():
            lin.bias.normal_(0, 0.5)
        xin = x if K == 1024 else torch.randn(tokens, K, device=DEV, generator=g).to(torch.bfloat16)

        def run(mode):
            monkeypatch.setattr(bert, "GEMM", mode)
            with torch.no_grad():
                if N == 1024:
                    return bert._proj_add_ln(resid, xin, lin, ln, name).float()
                return bert._proj(xin, lin, epi, name=name).float()

        ref = run("lib")
        for mode in ("auto", "ours"):
            route = bert.gemm_route(name, tokens, mode)
            c17, c18 = hip.k17_calls(), hip.k18_calls()
            got = run(mode)
            assert hip.k17_calls() - c17 == (route[0] == "k17"), (name, mode, route)
            assert hip.k18_calls() - c18 == (route[0] == "k18"), (name, mode, route)
            torch.cuda.synchronize()
            err = ((got - ref).norm() / ref.norm()).item()
            assert err < 8e-3, (tokens, name, mode, route, err)


def test_k17_dynamic_schedule_every_tile_once():
    """K17's claimed-tile scheduler (TCAMD_K17_DYN=1): the output buffers start
    as NaN, so a tile nobody computed shows up.  Back-to-back launches with
    different tile counts on one stream (each must find its counter reset by
    the previous launch's last workgroup), launches alternating between two
    streams (one counter per stream), ragged M, and a captured HIP graph
    replayed several times; every result against the fp32 matmul, and the
    dynamic and static (TCAMD_K17_DYN=0) outputs bitwise equal."""
    hip = _hip()
    shapes = [(24576, 3072, 1024), (6000, 1024, 4096), (12288, 4096, 1024), (777 * 8, 1024, 1024)]
    cases = [_case(M, N, K, seed=7) for M, N, K in shapes]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def run(i, out, stream):
        a, b, bias = cases[i]
        M, N, K = shapes[i]
        hip.k17_gemm(a.data_ptr(), b.data_ptr(), bias.data_ptr(), out.data_ptr(), M, N, K, K, K, N, epilogue="bias",
                     stream=stream.cuda_stream)

    refs = []
    for (a, b, bias), (M, N, K) in zip(cases, shapes):
        refs.append((a.float() @ b.float().t()) + bias)
    outs = [[torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16) for _ in range(3)]
            for M, N, K in shapes]
    torch.cuda.synchronize()  # the NaN fills ran on the current stream; the launches below use two others
    with hip.knob(TCAMD_K17_DYN=1):
        for rep in range(3):
            for i in range(len(shapes)):
                run(i, outs[i][rep], streams[(i + rep) % 2])
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        gout = [torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16) for M, N, K in shapes]
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for i in range(len(shapes)):  # warm-up on the capture stream
                run(i, gout[i], s)
        torch.cuda.synchronize()
        for o in gout:
            o.fill_(float("nan"))
        with torch.cuda.graph(g, stream=s):
            for i in range(len(shapes)):
                run(i, gout[i], s)
        for _ in range(4):
            g.replay()
        torch.cuda.synchronize()
    with hip.knob(TCAMD_K17_DYN=0):
        static = []
        for i, (M, N, K) in enumerate(shapes):
            o = torch.empty((M, N), device=DEV, dtype=torch.bfloat16)
            run(i, o, streams[0])
            static.append(o)
        torch.cuda.synchronize()
    for i, ref in enumerate(refs):
        for got in outs[i] + [gout[i]]:
            assert not got.isnan().any(), "a tile was never computed (shape %s)" % (shapes[i],)
            err = ((got.float() - ref).norm() / ref.norm()).item()
            assert err < 6e-3, (shapes[i], err)
            assert torch.equal(got, static[i]), "dynamic != static schedule (shape %s)" % (shapes[i],)


# ---------------------------------------------------------------------------
# K18 (csrc/kernels/gemm_tiles.hip): small / mid-M tiles, split-K partials
# ---------------------------------------------------------------------------
K18_SHAPES = [(384, 3072, 1024), (384, 1024, 4096), (3072, 4096, 1024), (300, 256, 128), (1, 128, 64),
              (517, 512, 192), (1000, 1280, 2048)]


@pytest.mark.parametrize("M,N,K", K18_SHAPES)
@pytest.mark.parametrize("epi", ["none", "bias", "bias_gelu"])
@pytest.mark.parametrize("cfg", list(range(13)))
def test_k18_gemm_bf16_out(M, N, K, epi, cfg):
    """Every tile configuration against the fp32 matmul of the same bf16
    operands; the ldc padding and the rows past M stay untouched."""
    hip = _hip()
    tm, tn, _, _ = hip.k18_cfg(cfg)
    if N % tn:
        pytest.skip("N not a multiple of the tile width")
    a, b, bias = _case(M, N, K, seed=3)
    ldc = N + 64
    c = torch.full((M + 3, ldc), 7.0, device=DEV, dtype=torch.bfloat16)
    hip.k18_gemm(a.data_ptr(), b.data_ptr(), bias.data_ptr(), c.data_ptr(), M, N, K, K, K, ldc, epilogue=epi, cfg=cfg,
                 stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t()
    if epi != "none":
        ref = ref + bias
    if epi == "bias_gelu":
        ref = _gelu(ref)
    got = c[:M, :N].float()
    err = ((got - ref).norm() / ref.norm()).item()
    worst = ((got - ref).abs() / (ref.abs() + 1e-2)).max().item()
    assert err < 6e-3 and worst < 3e-2, (err, worst)
    assert (c[:M, N:] == 7.0).all() and (c[M:] == 7.0).all(), "wrote outside C[:M, :N]"


@pytest.mark.parametrize("M,N,K,splits", [(384, 1024, 4096, 8), (384, 1024, 1024, 4), (3072, 1024, 4096, 2),
                                          (77, 256, 512, 8), (1000, 512, 3072, 3)])
@pytest.mark.parametrize("cfg", [0, 1, 4, 5, 7, 9, 10, 11, 12])
def test_k18_split_k_partials(M, N, K, splits, cfg):
    """split-K: slab z holds A[:, Kz] . B[:, Kz]^T in fp32 (against fp64), and
    the slabs sum to the whole product."""
    hip = _hip()
    a, b, _ = _case(M, N, K, seed=4)
    stride = (M + 1) * N
    ws = torch.full((splits, M + 1, N), 7.0, device=DEV)
    hip.k18_gemm(a.data_ptr(), b.data_ptr(), None, ws.data_ptr(), M, N, K, K, K, N, out_f32=True, cfg=cfg,
                 splits=splits, split_stride=stride, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    kc = K // splits
    for z in range(splits):
        ref = a[:, z * kc:(z + 1) * kc].double() @ b[:, z * kc:(z + 1) * kc].double().t()
        err = ((ws[z, :M].double() - ref).norm() / ref.norm()).item()
        assert err < 1e-5, (z, err)
        assert (ws[z, M:] == 7.0).all()
    full = a.double() @ b.double().t()
    assert ((ws[:, :M].double().sum(0) - full).norm() / full.norm()).item() < 1e-5


@pytest.mark.parametrize("cfg", [0, 3, 4, 6, 8])
def test_k18_fp32_out_strided(cfg):
    """fp32 output with bias (the fp32-parity bert's bf16x3 GEMM, K = 3 x
    hidden) and row strides larger than K."""
    hip = _hip()
    M, N, K, lda, ldb = 777, 1024, 3072, 3136, 3200
    a, b, bias = _case(M, N, K, lda, ldb, seed=6)
    c = torch.full((M + 1, N + 8), 7.0, device=DEV)
    hip.k18_gemm(a.data_ptr(), b.data_ptr(), bias.data_ptr(), c.data_ptr(), M, N, K, lda, ldb, N + 8,
                 epilogue="bias", out_f32=True, cfg=cfg, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = a[:, :K].double() @ b[:, :K].double().t() + bias.double()
    assert ((c[:M, :N].double() - ref).norm() / ref.norm()).item() < 1e-5
    assert (c[:M, N:] == 7.0).all() and (c[M:] == 7.0).all()


def test_k18_rejects_bad_shapes():
    hip = _hip()
    x = torch.zeros(1 << 16, device=DEV, dtype=torch.bfloat16)
    p = x.data_ptr()
    for args in [(8, 100, 64, 64, 64, 128, 0, 0, 0, 1, 0),   # N not a tile multiple
                 (8, 128, 96, 96, 96, 128, 0, 0, 0, 1, 0),   # K not a multiple of 64
                 (8, 128, 128, 128, 128, 128, 0, 0, 0, 3, 0),  # K not a multiple of 64 x splits
                 (8, 128, 128, 128, 128, 128, 0, 0, 0, 2, 8 * 128),  # split without fp32 out
                 (8, 128, 128, 128, 128, 128, 1, 1, 0, 2, 8 * 128),  # split with an epilogue
                 (8, 128, 128, 128, 128, 128, 0, 1, 0, 2, 100),  # slabs overlap
                 (8, 128, 128, 128, 128, 128, 0, 0, 99, 1, 0)]:  # no such cfg
        M, N, K, lda, ldb, ldc, epi, f32, cfg, splits, stride = args
        with pytest.raises(Exception):
            hip.k18_gemm(p, p, p if epi else None, p, M, N, K, lda, ldb, ldc,
                         epilogue=["none", "bias"][epi], out_f32=bool(f32), cfg=cfg, splits=splits,
                         split_stride=stride)


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("nparts,with_bias", [(0, False), (1, True), (4, True), (8, False)])
def test_add_layernorm_parts(f32, nparts, with_bias):
    """K11p: LayerNorm(x + bias + sum of fp32 partial slabs) against fp64."""
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(11 + nparts)
    rows, H = 777, 1024
    dt = torch.float32 if f32 else torch.bfloat16
    x = torch.randn(rows, H, device=DEV, generator=g).to(dt)
    parts = torch.randn(max(nparts, 1), rows + 2, H, device=DEV, generator=g) * 0.3
    bias = torch.randn(H, device=DEV, generator=g) * 0.1
    gamma = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).to(dt)
    beta = (0.1 * torch.randn(H, device=DEV, generator=g)).to(dt)
    out = torch.empty(rows, H, device=DEV, dtype=dt)
    hip.add_layernorm_parts(x.data_ptr(), parts.data_ptr(), nparts, (rows + 2) * H,
                            bias.data_ptr() if with_bias else None, gamma.data_ptr(), beta.data_ptr(), out.data_ptr(),
                            rows, H, 1e-12, f32=f32, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    v = x.double() + (parts[:nparts, :rows].double().sum(0) if nparts else 0)
    if with_bias:
        v = v + bias.double()
    ref = torch.nn.functional.layer_norm(v, (H,), gamma.double(), beta.double(), eps=1e-12)
    err = ((out.double() - ref).norm() / ref.norm()).item()
    assert err < (1e-6 if f32 else 4e-3), err


@pytest.mark.parametrize("H", [1024, 4096])
def test_add_layernorm_parts_x3_operand(H):
    """K11p's fp32 form with out3: the LayerNorm output also as the next
    bf16x3 GEMM's operand, bitwise what x3_cat makes of the fp32 output."""
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(H)
    rows = 333
    x = torch.randn(rows, H, device=DEV, generator=g)
    y = torch.randn(rows, H, device=DEV, generator=g) * 0.3
    gamma = 1 + 0.1 * torch.randn(H, device=DEV, generator=g)
    beta = 0.1 * torch.randn(H, device=DEV, generator=g)
    out = torch.empty(rows, H, device=DEV)
    out3 = torch.full((rows, 3 * H), 7.0, device=DEV, dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    hip.add_layernorm_parts(x.data_ptr(), y.data_ptr(), 1, rows * H, None, gamma.data_ptr(), beta.data_ptr(),
                            out.data_ptr(), rows, H, 1e-12, f32=True, stream=st, out3=out3.data_ptr())
    ref3 = torch.empty_like(out3)
    hip.x3_cat(out.data_ptr(), ref3.data_ptr(), rows, H, stream=st)
    plain = torch.empty_like(out)
    hip.add_layernorm_parts(x.data_ptr(), y.data_ptr(), 1, rows * H, None, gamma.data_ptr(), beta.data_ptr(),
                            plain.data_ptr(), rows, H, 1e-12, f32=True, stream=st)
    torch.cuda.synchronize()
    assert torch.equal(out3, ref3) and torch.equal(out, plain)
    with pytest.raises(hip.HipError):  # bf16 model: no x3 operand
        hip.add_layernorm_parts(x.data_ptr(), y.data_ptr(), 1, rows * H, None, gamma.data_ptr(), beta.data_ptr(),
                                out.data_ptr(), rows, H, 1e-12, f32=False, stream=st, out3=out3.data_ptr())


@pytest.mark.parametrize("M", [300, 4100])
def test_k17_gelu_erf_x3_operand(M):
    """K17's bias_gelu_erf_x3 epilogue (the fp32-parity FFN-up writing the
    FFN-down's bf16x3 operand) is bitwise x3_cat of its fp32-output form;
    fp32 output and a short ldc are refused."""
    hip = _hip()
    N, K = 1024, 3072
    a, b, bias = _case(M, N, K, seed=M)
    st = torch.cuda.current_stream().cuda_stream
    c = torch.empty(M, N, device=DEV)
    hip.k17_gemm(a.data_ptr(), b.data_ptr(), bias.data_ptr(), c.data_ptr(), M, N, K, K, K, N,
                 epilogue="bias_gelu_erf", out_f32=True, stream=st)
    c3 = torch.full((M, 3 * N), 7.0, device=DEV, dtype=torch.bfloat16)
    hip.k17_gemm(a.data_ptr(), b.data_ptr(), bias.data_ptr(), c3.data_ptr(), M, N, K, K, K, 3 * N,
                 epilogue="bias_gelu_erf_x3", stream=st)
    ref3 = torch.empty_like(c3)
    hip.x3_cat(c.data_ptr(), ref3.data_ptr(), M, N, stream=st)
    torch.cuda.synchronize()
    assert torch.equal(c3, ref3)
    for kw in ({"out_f32": True, "ldc": 3 * N}, {"out_f32": False, "ldc": 2 * N}):
        with pytest.raises(hip.HipError):
            hip.k17_gemm(a.data_ptr(), b.data_ptr(), bias.data_ptr(), c3.data_ptr(), M, N, K, K, K, kw["ldc"],
                         epilogue="bias_gelu_erf_x3", out_f32=kw["out_f32"], stream=st)


@pytest.mark.parametrize("kern", ["k17", "k18_c3", "k18_c6"])
def test_gelu_erf_epilogue_fp32(kern):
    """bias + erf-form GELU with fp32 output (the fp32-parity bert's FFN-up on
    its bf16x3 operands) against fp64 of the same bf16 operands; the bf16
    output form is refused."""
    hip = _hip()
    M, N, K = 300, 512, 3072
    a, b, bias = _case(M, N, K, seed=9)
    c = torch.full((M, N), 7.0, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    if kern == "k17":
        hip.k17_gemm(a.data_ptr(), b.data_ptr(), bias.data_ptr(), c.data_ptr(), M, N, K, K, K, N,
                     epilogue="bias_gelu_erf", out_f32=True, stream=st)
    else:
        hip.k18_gemm(a.data_ptr(), b.data_ptr(), bias.data_ptr(), c.data_ptr(), M, N, K, K, K, N,
                     epilogue="bias_gelu_erf", out_f32=True, cfg=int(kern[-1]), stream=st)
    torch.cuda.synchronize()
    ref = torch.nn.functional.gelu(a.double() @ b.double().t() + bias.double())
    assert ((c.double() - ref).norm() / ref.norm()).item() < 1e-5
    with pytest.raises(Exception):
        hip.k18_gemm(a.data_ptr(), b.data_ptr(), bias.data_ptr(), c.data_ptr(), M, N, K, K, K, N,
                     epilogue="bias_gelu_erf", out_f32=False, cfg=3, stream=st)
