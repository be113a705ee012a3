"""Which models a server loads (server/app.py default_models)."""


def test_fp32_parity_bert_is_opt_in():
    """bert_large_fp32 (~2 GB of bf16x3 weights, 28 HIP graphs per instance)
    is in no default list: --gpu loads the GPU zoo without it, and --models
    must name it (round-5 advisor finding)."""
    from triton_client_amd.server.app import default_models

    names = [m.name for m in default_models(gpu=True)]
    assert "bert_large" in names and "densenet_onnx" in names
    assert "bert_large_fp32" not in names
    sel = [m.name for m in default_models(gpu=True, names=["bert_large_fp32", "simple"])]
    assert sorted(sel) == ["bert_large_fp32", "simple"]
    assert [m.name for m in default_models(gpu=False, names=["bert_large_fp32"])] == []
