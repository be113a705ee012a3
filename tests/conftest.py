import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def cpu_server():
    """In-process KServe-v2 server with the CPU model zoo (HTTP + gRPC)."""
    from triton_client_amd.server import ServerHandle

    h = ServerHandle().start()
    yield h
    h.stop()


@pytest.fixture(scope="session")
def gpu_server():
    """The bench server as a child process on GPU 0 (GPU model zoo + a few CPU models)."""
    from triton_client_amd.perf.harness import ServerProcess

    log = os.path.join(os.environ.get("GRAFT_REPO_ROOT", REPO), "gpurun_out", "pytest_gpu_server.log")
    os.makedirs(os.path.dirname(log), exist_ok=True)
    srv = ServerProcess(device=0, models="simple,simple_identity,densenet_onnx,preprocess_inception,preprocess_inception_ensemble,bert_large",
                        log_path=log, extra_args=["--instance-count", "1"])
    try:
        srv.wait_ready(timeout=900, model="densenet_onnx")
        yield srv
    finally:
        srv.stop()
