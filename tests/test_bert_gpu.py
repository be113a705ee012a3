"""bert_large: module numerics vs fp32, and served through gRPC (host and
HIP-shm tensors) on the GPU server."""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def test_bert_module_bf16_close_to_fp32():
    from triton_client_amd.models import bert

    m32 = bert.build(device="cuda", dtype=torch.float32, layers=4)
    m16 = bert.build(device="cuda", dtype=torch.bfloat16, layers=4)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, bert.VOCAB, (2, 384), generator=g).cuda()
    mask = torch.ones(2, 384, dtype=torch.int32).cuda()
    mask[1, 300:] = 0
    tt = torch.zeros(2, 384, dtype=torch.long).cuda()
    with torch.no_grad():
        s32, e32 = m32(ids, mask, tt)
        s16, e16 = m16(ids, mask, tt)
    rel = ((s16 - s32).norm() / s32.norm()).item()
    assert rel < 0.08, rel
    assert torch.isfinite(s16).all() and torch.isfinite(e16).all()


def test_bert_served(gpu_server):
    import tritonclient.grpc as grpcclient

    c = grpcclient.InferenceServerClient(gpu_server.grpc_url)
    if not c.is_model_ready("bert_large"):
        c.load_model("bert_large")
    rng = np.random.default_rng(0)
    ids = rng.integers(0, 30522, size=(3, 384), dtype=np.int32)
    mask = np.ones((3, 384), dtype=np.int32)
    tt = np.zeros((3, 384), dtype=np.int32)
    ins = []
    for name, a in (("input_ids", ids), ("attention_mask", mask), ("token_type_ids", tt)):
        x = grpcclient.InferInput(name, list(a.shape), "INT32")
        x.set_data_from_numpy(a)
        ins.append(x)
    r1 = c.infer("bert_large", ins)
    st = r1.as_numpy("start_logits")
    assert st.shape == (3, 384) and np.isfinite(st).all()
    # the same request once more: deterministic graph replay
    r2 = c.infer("bert_large", ins)
    np.testing.assert_allclose(r2.as_numpy("start_logits"), st, rtol=0, atol=1e-3)
    # row independence under dynamic batching: row 0 alone equals row 0 of the batch
    ins1 = []
    for name, a in (("input_ids", ids[:1]), ("attention_mask", mask[:1]), ("token_type_ids", tt[:1])):
        x = grpcclient.InferInput(name, list(a.shape), "INT32")
        x.set_data_from_numpy(a)
        ins1.append(x)
    r3 = c.infer("bert_large", ins1)
    np.testing.assert_allclose(r3.as_numpy("start_logits")[0], st[0], rtol=0.05, atol=0.05)
