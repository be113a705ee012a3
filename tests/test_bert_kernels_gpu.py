"""K11 fused residual add + LayerNorm, and the fused BERT-large layer path,
against plain PyTorch fp32 references."""

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("rows,H", [(1, 1024), (37, 1024), (1000, 1024), (13, 512), (5, 4096)])
@pytest.mark.parametrize("alias", [False, True])
def test_add_layernorm(rows, H, alias):
    _need_gpu()
    from triton_client_amd.ops import hip

    g = torch.Generator(device=DEV).manual_seed(rows * 7 + H)
    x = (torch.randn(rows, H, device=DEV, generator=g) * 3 + 1).bfloat16()
    y = torch.randn(rows, H, device=DEV, generator=g).bfloat16()
    gamma = (torch.rand(H, device=DEV, generator=g) + 0.5).bfloat16()
    beta = torch.randn(H, device=DEV, generator=g).bfloat16()
    ref = torch.nn.functional.layer_norm(x.float() + y.float(), (H,), gamma.float(), beta.float(), 1e-12)
    out = x if alias else torch.empty_like(x)
    hip.add_layernorm(x.data_ptr(), y.data_ptr(), gamma.data_ptr(), beta.data_ptr(), out.data_ptr(), rows, H, 1e-12)
    torch.cuda.synchronize()
    err = (out.float() - ref).norm() / ref.norm()
    assert err.item() < 1e-2, err.item()
    assert (out.float() - ref).abs().max().item() < 0.1


@pytest.mark.parametrize("b,s", [(1, 384), (3, 128), (2, 7)])
def test_embed_layernorm_matches_torch(b, s):
    """Embedding sum + LayerNorm in one launch vs the torch ops in fp32."""
    _need_gpu()
    from triton_client_amd.models import bert

    m = bert.build(device=DEV, layers=1)
    with torch.no_grad():
        m.ln.weight.copy_(torch.rand_like(m.ln.weight.float()) + 0.5)
        m.ln.bias.copy_(torch.randn_like(m.ln.bias.float()) * 0.1)
        ids = torch.randint(0, bert.VOCAB, (b, s), device=DEV)
        tt = torch.randint(0, bert.TYPES, (b, s), device=DEV)
        got = m._embed(ids, tt).float()
        pos = torch.arange(s, device=DEV)
        e = m.word.weight.float()[ids] + m.pos.weight.float()[pos][None] + m.tok_type.weight.float()[tt]
        ref = torch.nn.functional.layer_norm(e, (bert.HIDDEN,), m.ln.weight.float(), m.ln.bias.float(), m.ln.eps)
    err = (got - ref).norm() / ref.norm()
    assert err.item() < 1e-2, err.item()


def test_add_layernorm_rejects_bad_width():
    _need_gpu()
    from triton_client_amd.ops import hip

    x = torch.zeros(4, 768, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(hip.HipError):
        hip.add_layernorm(x.data_ptr(), x.data_ptr(), x.data_ptr(), x.data_ptr(), x.data_ptr(), 4, 768, 1e-12)


def test_bert_fused_layers_match_torch_ops():
    """The served bf16 model with K11 + GELU-epilogue GEMMs vs the same weights through plain torch ops in fp32."""
    _need_gpu()
    from triton_client_amd.models import bert

    m = bert.build(device=DEV, layers=2)
    with torch.no_grad():  # non-zero biases: the QKV bias is applied inside K12
        for p in m.parameters():
            if p.dim() == 1 and not torch.all(p == 1):
                p.copy_(torch.randn_like(p.float()) * 0.05)
    ids = torch.randint(0, bert.VOCAB, (3, 128), device=DEV)
    mask = torch.ones(3, 128, device=DEV, dtype=torch.int64)
    mask[1, 100:] = 0
    tt = torch.zeros(3, 128, device=DEV, dtype=torch.int64)
    with torch.no_grad():
        s_fused, e_fused = m(ids, mask, tt)
        ref = bert.build(device=DEV, dtype=torch.float32, layers=2)
        ref.load_state_dict({k: v.float() for k, v in m.state_dict().items()})
        try:
            bert.FUSED = False
            s_ref, e_ref = ref(ids, mask, tt)
        finally:
            bert.FUSED = True
    for got, want in ((s_fused, s_ref), (e_fused, e_ref)):
        err = (got.float() - want).norm() / want.norm()
        assert err.item() < 5e-2, err.item()


def test_bert_dense_path_matches_masked_when_no_padding():
    """dense=True (attention without the key-padding bias) is what the server
    replays for batches with no padding: same logits as the masked graph."""
    _need_gpu()
    from triton_client_amd.models import bert

    m = bert.build(device=DEV, layers=2)
    ids = torch.randint(0, bert.VOCAB, (4, 384), device=DEV)
    mask = torch.ones(4, 384, device=DEV, dtype=torch.int64)
    tt = torch.zeros(4, 384, device=DEV, dtype=torch.int64)
    with torch.no_grad():
        a = m(ids, mask, tt)
        b = m(ids, mask, tt, dense=True)
    for x, y in zip(a, b):
        assert ((x - y).norm() / x.norm()).item() < 2e-2


def _attn_ref(qkv, mask, seqs, S, heads=16, D=64):
    x = qkv.float().view(seqs, S, 3, heads, D).permute(2, 0, 3, 1, 4)
    q, k, v = x[0], x[1], x[2]
    s = q @ k.transpose(-1, -2) / D ** 0.5
    if mask is not None:
        s = s + ((1.0 - mask.float()) * -10000.0)[:, None, None, :]
    a = torch.softmax(s, dim=-1) @ v
    return a.transpose(1, 2).reshape(seqs, S, heads * D)


@pytest.mark.parametrize("seqs,S,masked", [(1, 64, False), (3, 128, True), (2, 384, True), (5, 192, False),
                                           (4, 384, False)])
def test_attention_kernel_matches_fp32(seqs, S, masked):
    """K12 vs softmax(QK^T/8 + key-padding bias) V in fp32, reading the fused QKV layout."""
    _need_gpu()
    from triton_client_amd.ops import hip

    g = torch.Generator(device=DEV).manual_seed(seqs * 1000 + S)
    qkv = (torch.randn(seqs * S, 3 * 1024, device=DEV, generator=g) * 1.5).bfloat16()
    mask = None
    if masked:
        mask = torch.ones(seqs, S, device=DEV, dtype=torch.int32)
        for i in range(seqs):
            mask[i, S - 7 * (i + 1) * (S // 64):] = 0  # padded tails of different lengths
        mask[0, 5] = 0  # and one hole inside a sequence
    out = torch.empty(seqs * S, 1024, device=DEV, dtype=torch.bfloat16)
    hip.attention(qkv.data_ptr(), None if mask is None else mask.data_ptr(), out.data_ptr(), seqs, S, 16, 0.125)
    torch.cuda.synchronize()
    ref = _attn_ref(qkv, mask, seqs, S).reshape(seqs * S, 1024)
    err = (out.float() - ref).norm() / ref.norm()
    assert err.item() < 1e-2, err.item()
    assert torch.isfinite(out.float()).all()


@pytest.mark.parametrize("masked", [False, True])
def test_attention_kernel_applies_qkv_bias(masked):
    """K12 with the projection bias passed separately (q + b_q, b_k dropped:
    softmax-invariant, b_v added to the output) vs the reference on qkv + b."""
    _need_gpu()
    from triton_client_amd.ops import hip

    seqs, S = 2, 256
    g = torch.Generator(device=DEV).manual_seed(11 + masked)
    qkv = (torch.randn(seqs * S, 3 * 1024, device=DEV, generator=g) * 1.5).bfloat16()
    bias = (torch.randn(3 * 1024, device=DEV, generator=g) * 0.5).bfloat16()
    mask = None
    if masked:
        mask = torch.ones(seqs, S, device=DEV, dtype=torch.int32)
        mask[1, S - 40:] = 0
    out = torch.empty(seqs * S, 1024, device=DEV, dtype=torch.bfloat16)
    hip.attention(qkv.data_ptr(), None if mask is None else mask.data_ptr(), out.data_ptr(), seqs, S, 16, 0.125,
                  bias=bias.data_ptr())
    torch.cuda.synchronize()
    ref = _attn_ref((qkv.float() + bias.float()).bfloat16(), mask, seqs, S).reshape(seqs * S, 1024)
    err = (out.float() - ref).norm() / ref.norm()
    assert err.item() < 1e-2, err.item()


@pytest.mark.parametrize("seqs,S,masked", [(1, 64, False), (3, 128, True), (2, 384, True), (4, 384, False),
                                           (1, 512, True)])
def test_attention_f32_matches_fp64(seqs, S, masked):
    """K12x (fp32-parity attention: bf16x3 QK^T and PV, fp32 softmax) against
    fp64 softmax(QK^T/8 + key-padding bias) V on fp32 inputs; one sequence
    fully masked (the reference's additive -10000 makes it a plain average)."""
    _need_gpu()
    from triton_client_amd.ops import hip

    g = torch.Generator(device=DEV).manual_seed(seqs * 977 + S)
    qkv = torch.randn(seqs * S, 3 * 1024, device=DEV, generator=g) * 1.5
    mask = None
    if masked:
        mask = torch.ones(seqs, S, device=DEV, dtype=torch.int32)
        for i in range(seqs):
            mask[i, S - 7 * (i + 1) * (S // 64):] = 0
        mask[0, 5] = 0
        if seqs > 2:
            mask[2] = 0
    out = torch.full((seqs * S, 1024), float("nan"), device=DEV)
    hip.attention_f32(qkv.data_ptr(), None if mask is None else mask.data_ptr(), out.data_ptr(), seqs, S, 16, 0.125)
    torch.cuda.synchronize()
    x = qkv.double().view(seqs, S, 3, 16, 64).permute(2, 0, 3, 1, 4)
    sc = x[0] @ x[1].transpose(-1, -2) / 8.0
    if mask is not None:
        sc = sc + ((1.0 - mask.double()) * -10000.0)[:, None, None, :]
    ref = (torch.softmax(sc, dim=-1) @ x[2]).transpose(1, 2).reshape(seqs, S, 1024)
    got = out.double().view(seqs, S, 1024)
    for i in range(seqs):
        err = ((got[i] - ref[i]).norm() / ref[i].norm()).item()
        # a fully masked sequence: every fp32 score carries the -10000 offset,
        # which leaves ~10 fewer bits of it (as in the reference's fp32 path)
        assert err < (2e-3 if mask is not None and not mask[i].any() else 2e-5), (i, err)


def test_attention_f32_x3_operand():
    """K12x with x3: the output written as the out projection's bf16x3 operand
    is bitwise x3_cat of its fp32 output."""
    _need_gpu()
    from triton_client_amd.ops import hip

    seqs, S = 2, 384
    g = torch.Generator(device=DEV).manual_seed(5)
    qkv = torch.randn(seqs * S, 3 * 1024, device=DEV, generator=g)
    mask = torch.ones(seqs, S, device=DEV, dtype=torch.int32)
    mask[1, 300:] = 0
    out = torch.empty(seqs * S, 1024, device=DEV)
    out3 = torch.empty(seqs * S, 3 * 1024, device=DEV, dtype=torch.bfloat16)
    hip.attention_f32(qkv.data_ptr(), mask.data_ptr(), out.data_ptr(), seqs, S, 16, 0.125)
    hip.attention_f32(qkv.data_ptr(), mask.data_ptr(), out3.data_ptr(), seqs, S, 16, 0.125, x3=True)
    ref3 = torch.empty_like(out3)
    hip.x3_cat(out.data_ptr(), ref3.data_ptr(), seqs * S, 1024)
    torch.cuda.synchronize()
    assert torch.equal(out3, ref3)


def test_attention_rejects_unsupported_shapes():
    _need_gpu()
    from triton_client_amd.ops import hip

    x = torch.zeros(448, 3 * 1024, device=DEV, dtype=torch.bfloat16)
    o = torch.zeros(448, 1024, device=DEV, dtype=torch.bfloat16)
    for S in (100, 448):
        with pytest.raises(hip.HipError):
            hip.attention(x.data_ptr(), None, o.data_ptr(), 1, S, 16, 0.125)


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("rows,H", [(1, 1024), (777, 1024), (5, 512)])
def test_qa_head(f32, rows, H):
    """The span head kernel (one launch: both logits planes in fp32) against
    fp64 of the same operands."""
    _need_gpu()
    from triton_client_amd.ops import hip

    g = torch.Generator(device=DEV).manual_seed(rows + H)
    dt = torch.float32 if f32 else torch.bfloat16
    x = torch.randn(rows, H, device=DEV, generator=g).to(dt)
    w = (torch.randn(2, H, device=DEV, generator=g) * 0.05).to(dt)
    b = torch.randn(2, device=DEV, generator=g)
    out = torch.full((2, rows), float("nan"), device=DEV)
    hip.qa_head(x.data_ptr(), w.data_ptr(), b.data_ptr(), out[0].data_ptr(), out[1].data_ptr(), rows, H, f32=f32)
    torch.cuda.synchronize()
    ref = (x.double() @ w.double().t() + b.double()).t()
    err = ((out.double() - ref).norm() / ref.norm()).item()
    assert err < 1e-5, err
