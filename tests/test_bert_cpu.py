"""bert_large module on CPU (1 layer, fp32): shapes, padding-mask semantics,
and agreement with an unfused per-head attention written out by hand."""

import pytest

torch = pytest.importorskip("torch")


def _reference_layer(layer, x, mask):
    import torch.nn.functional as F
    from triton_client_amd.models import bert

    b, s, h = x.shape
    d = h // bert.HEADS
    q, k, v = layer.qkv(x).split(h, dim=-1)
    heads = lambda t: t.view(b, s, bert.HEADS, d).transpose(1, 2)
    q, k, v = heads(q), heads(k), heads(v)
    att = q @ k.transpose(-1, -2) / d ** 0.5 + (1.0 - mask[:, None, None, :].float()) * -10000.0
    a = (att.softmax(-1) @ v).transpose(1, 2).reshape(b, s, h)
    x = layer.ln1(x + layer.out(a))
    return layer.ln2(x + layer.ffn2(F.gelu(layer.ffn1(x))))


def test_bert_cpu_forward_matches_reference():
    from triton_client_amd.models import bert

    torch.manual_seed(0)
    m = bert.build(device="cpu", dtype=torch.float32, layers=1)
    ids = torch.randint(0, bert.VOCAB, (2, 16))
    mask = torch.ones(2, 16, dtype=torch.int32)
    mask[1, 10:] = 0
    tt = torch.zeros(2, 16, dtype=torch.long)
    with torch.no_grad():
        s, e = m(ids, mask, tt)
        x = m.ln(m.word(ids) + m.pos(torch.arange(16))[None] + m.tok_type(tt))
        x = _reference_layer(m.layers[0], x, mask)
        ref = m.qa(x)
    assert s.shape == (2, 16) and e.shape == (2, 16) and s.dtype == torch.float32
    torch.testing.assert_close(s, ref[..., 0], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(e, ref[..., 1], rtol=1e-4, atol=1e-4)


def test_bert_padding_does_not_leak():
    """Changing token ids at masked positions must not change unmasked logits."""
    from triton_client_amd.models import bert

    m = bert.build(device="cpu", dtype=torch.float32, layers=1)
    ids = torch.randint(0, bert.VOCAB, (1, 12))
    mask = torch.ones(1, 12, dtype=torch.int32)
    mask[0, 8:] = 0
    tt = torch.zeros(1, 12, dtype=torch.long)
    ids2 = ids.clone()
    ids2[0, 8:] = (ids2[0, 8:] + 7) % bert.VOCAB
    with torch.no_grad():
        a, _ = m(ids, mask, tt)
        b, _ = m(ids2, mask, tt)
    # -10000 additive bias leaves exp(-1e4) ~ 0 weight on padded keys
    torch.testing.assert_close(a[0, :8], b[0, :8], rtol=1e-5, atol=1e-5)


def test_bert_flops():
    from triton_client_amd.models import bert

    f = bert.flops_per_sequence()
    assert 2.0e11 < f < 3.0e11  # ~0.25 TFLOP per 384-token sequence


def test_gemm_route_table():
    """bert's projection routing (TC_BERT_GEMM): the measured tables (bf16 and
    the fp32-parity bf16x3 ones) in auto mode, no library anywhere in ours
    mode, the library everywhere in lib mode; the last entry covers every
    larger token count."""
    from triton_client_amd.models import bert

    for table, route in ((bert.GEMM_ROUTES, bert.gemm_route), (bert.GEMM_ROUTES_X3, bert.gemm_route_x3)):
        for name, entries in table.items():
            tops = [t for t, _ in entries]
            assert tops == sorted(tops) and tops[-1] == bert.INF, name
            for top, r in entries:
                for M in (top, top - 1 if top > 1 else top):
                    assert route(name, M, "auto") == r
                    ours = route(name, M, "ours")
                    assert ours[0] in ("k17", "k18") and (r[0] == "lib" or ours == r)
                    assert route(name, M, "lib") == ("lib",)
            assert route(name, 10 ** 6, "auto") == entries[-1][1]
        # split-K only where K11p can sum the slabs: the N = 1024 projections
        for name in ("qkv", "ffn_up"):
            assert all(r[0] != "k18" or r[2] == 1 for _, r in table[name])
