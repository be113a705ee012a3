"""bert_large (BASELINE config 4) served-level accuracy contract.

Two served precisions of the same BERT-large QA model (seed 0, random init):

* ``bert_large`` (the config-4 serving default): bf16 weights and
  activations, hipBLASLt GEMMs with fp32 accumulation, K11 residual-add +
  LayerNorm, K12 attention (key-padding mask in kernel), one HIP graph per
  batch bucket captured in the server, plus an unmasked ("dense") one for the
  buckets from 32 rows, run when no real row is padded.  Compared with an
  fp32 forward of the SAME weights (the bf16 parameters upcast), so the gap
  is the serving precision, not a weight rounding.
* ``bert_large_fp32``: fp32-parity compute (every projection one bf16x3 GEMM,
  fp32 LayerNorm / GELU / attention), compared with the fp32 module of the
  fp32 weights.

Both are served through the bench server's native gRPC front end at batch 1,
7 (bucket 8: a padded graph) and 64, with padded rows and an
all-full-length batch.  The contract (our own: the reference
holds no bert fixture, parity with it is unpinned), per row of start and end
logits:

  bf16:  rel-L2 <= BF16_REL, answer-span agreement 100 % at BF16_TIE
  fp32:  rel-L2 <= FP32_REL, answer-span agreement 100 % at FP32_TIE

The random-init 24-layer model amplifies perturbations ~1000x into its
logits: K12's masked and unmasked paths differ by 5e-6..2e-5 on the same
inputs and the whole model's logits then differ by 1.1 %
(tools/bert_path_probe.py).  So the logit bounds sit well above per-op
precision (bf16 ~4e-3 per op -> 1.8-4.8 % measured; bf16x3 ~1.5e-5 per op ->
0.04-0.11 % measured), and the answer-span check is tie-aware: the served
argmax must be a position whose REFERENCE logit is within TIE x (reference
range) of the reference maximum (random-init logits are nearly flat, and an
exact argmax flips on near-ties: 93 % exact agreement for bf16, 98 % for the
fp32-parity path).  Measured numbers: profiles/r5_bert_accuracy.md.
"""

import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

BF16_REL = 8e-2
BF16_TIE = 0.05
FP32_REL = 2e-3
FP32_TIE = 0.005
CASES = [(1, False), (7, False), (7, True), (64, False)]


def _inputs(b, seed, full=False):
    rng = np.random.default_rng(seed)
    ids = rng.integers(1000, 30000, size=(b, 384), dtype=np.int32)
    mask = np.ones((b, 384), dtype=np.int32)
    tt = np.zeros((b, 384), dtype=np.int32)
    for i in range(b):
        n = 384 if full or i % 3 == 0 else int(rng.integers(32, 384))
        q = int(rng.integers(8, max(9, n // 3)))
        mask[i, n:] = 0
        ids[i, n:] = 0
        tt[i, q:n] = 1  # question | context segments
    return ids, mask, tt


def _serve(client, model, ids, mask, tt):
    import tritonclient.grpc as grpcclient

    ins = []
    for name, a in (("input_ids", ids), ("attention_mask", mask), ("token_type_ids", tt)):
        x = grpcclient.InferInput(name, list(a.shape), "INT32")
        x.set_data_from_numpy(a)
        ins.append(x)
    r = client.infer(model, ins)
    return r.as_numpy("start_logits").astype(np.float64), r.as_numpy("end_logits").astype(np.float64)


def _fwd(m, ids, mask, tt):
    with torch.no_grad():
        s, e = m(torch.from_numpy(ids).long().cuda(), torch.from_numpy(mask).cuda(), torch.from_numpy(tt).long().cuda())
    return s.double().cpu().numpy(), e.double().cpu().numpy()


def _row_rel(a, b):
    return np.linalg.norm(a - b, axis=1) / np.maximum(np.linalg.norm(b, axis=1), 1e-30)


def _near_best(got, ref, tie):
    """per row: the served argmax is within tie x range of the reference max (in the reference's logits)"""
    pick = ref[np.arange(ref.shape[0]), got.argmax(1)]
    return pick >= ref.max(1) - tie * (ref.max(1) - ref.min(1))


def _compare(got, ref, tie=0.0):
    (s, e), (rs, re_) = got, ref
    rel = np.maximum(_row_rel(s, rs), _row_rel(e, re_))
    exact = np.concatenate([s.argmax(1) == rs.argmax(1), e.argmax(1) == re_.argmax(1)])
    near = np.concatenate([_near_best(s, rs, tie), _near_best(e, re_, tie)])
    return rel, exact, near


@pytest.fixture(scope="module")
def fp32_server():
    """bert_large_fp32 in a server of its own (the shared gpu_server loads the bf16 model only)."""
    from triton_client_amd.perf.harness import ServerProcess

    root = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    log = os.path.join(root, "gpurun_out", "pytest_bert_fp32_server.log")
    os.makedirs(os.path.dirname(log), exist_ok=True)
    srv = ServerProcess(device=0, models="bert_large_fp32", log_path=log, extra_args=["--instance-count", "1"])
    try:
        srv.wait_ready(timeout=900, model="bert_large_fp32")
        yield srv
    finally:
        srv.stop()


@pytest.fixture(scope="module")
def models():
    from triton_client_amd.models import bert

    m16 = bert.build(device="cuda", dtype=torch.bfloat16)
    out = {"bf16_ref": bert.build(device="cuda", dtype=torch.bfloat16).float().eval(),  # served bf16 weights, fp32
           "bf16_inproc": m16,
           "fp32_ref": bert.build(device="cuda", dtype=torch.float32)}
    yield out
    out.clear()
    torch.cuda.empty_cache()


_AGREE = {"bf16": [], "fp32": []}


@pytest.mark.parametrize("b,full", CASES)
def test_bert_bf16_served_vs_fp32(gpu_server, models, b, full):
    import tritonclient.grpc as grpcclient

    c = grpcclient.InferenceServerClient(gpu_server.grpc_url)
    if not c.is_model_ready("bert_large"):
        c.load_model("bert_large")
    ids, mask, tt = _inputs(b, seed=100 + b + int(full), full=full)
    got = _serve(c, "bert_large", ids, mask, tt)
    rel, agree, near = _compare(got, _fwd(models["bf16_ref"], ids, mask, tt), BF16_TIE)
    # the same bf16 model in this process (same kernels, eager, hipBLASLt's
    # eager solution choice): another bf16 rounding path of the same math, so
    # it sits inside the same bf16 band, not bit-equal to the served graphs
    rel_ip = _compare(got, _fwd(models["bf16_inproc"], ids, mask, tt))[0]
    print("bert bf16 served vs fp32: b=%d full=%s row rel max %.3g mean %.3g argmax exact %.3f near %.3f | "
          "vs in-process bf16 %.2g" % (b, full, rel.max(), rel.mean(), agree.mean(), near.mean(), rel_ip.max()))
    assert np.isfinite(got[0]).all() and np.isfinite(got[1]).all()
    assert rel.max() <= BF16_REL, rel
    assert rel_ip.max() <= BF16_REL, rel_ip
    assert near.all(), near
    _AGREE["bf16"].append(agree)


@pytest.mark.parametrize("b,full", CASES)
def test_bert_fp32_parity_served_vs_fp32(fp32_server, models, b, full):
    import tritonclient.grpc as grpcclient

    c = grpcclient.InferenceServerClient(fp32_server.grpc_url)
    ids, mask, tt = _inputs(b, seed=200 + b + int(full), full=full)
    got = _serve(c, "bert_large_fp32", ids, mask, tt)
    rel, agree, near = _compare(got, _fwd(models["fp32_ref"], ids, mask, tt), FP32_TIE)
    print("bert fp32-parity served vs fp32: b=%d full=%s row rel max %.3g mean %.3g argmax exact %.3f near %.3f"
          % (b, full, rel.max(), rel.mean(), agree.mean(), near.mean()))
    assert np.isfinite(got[0]).all() and np.isfinite(got[1]).all()
    assert rel.max() <= FP32_REL, rel
    assert near.all(), near
    _AGREE["fp32"].append(agree)


def test_bert_argmax_agreement_overall():
    """Exact answer-span argmax agreement over every row served above, reported
    (near-ties flip it; the tie-aware check above is the asserted contract),
    with a floor that catches a systematic error (a wrong row, mask or head)."""
    if not _AGREE["bf16"] and not _AGREE["fp32"]:
        pytest.skip("no served rows (run with the cases above)")
    for prec, floor in (("bf16", 0.8), ("fp32", 0.9)):
        if _AGREE[prec]:
            a = np.concatenate(_AGREE[prec])
            print("bert %s exact argmax agreement: %d / %d" % (prec, a.sum(), a.size))
            assert a.mean() >= floor, (prec, a.mean())
