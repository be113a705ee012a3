"""Packaging surface: setup.py metadata/extras, deprecated shim packages."""

import importlib
import os
import subprocess
import sys
import warnings

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_setup_metadata():
    out = subprocess.run([sys.executable, "setup.py", "--name", "--version"], cwd=REPO, capture_output=True,
                         text=True, env=dict(os.environ, VERSION="2.41.0"))
    assert out.returncode == 0, out.stderr
    assert out.stdout.split()[-2:] == ["tritonclient", "2.41.0"]


def test_extras_match_reference():
    sys.path.insert(0, REPO)
    import setup as s  # noqa: E402

    assert {"http", "grpc", "cuda", "hip", "all"} <= set(s.extras_require)
    assert set(s.extras_require["all"]) >= set(s.extras_require["grpc"]) | set(s.extras_require["http"])


def test_deprecated_shims_warn_and_reexport():
    for mod, attr in [("tritonhttpclient", "InferenceServerClient"), ("tritongrpcclient", "InferInput"),
                      ("tritonclientutils", "np_to_triton_dtype"), ("tritongrpcclient.grpc_service_pb2",
                                                                    "ModelInferRequest"),
                      ("tritongrpcclient.model_config_pb2", "ModelConfig"),
                      ("tritongrpcclient.grpc_service_pb2_grpc", "GRPCInferenceServiceStub"),
                      ("tritonshmutils.shared_memory", "create_shared_memory_region")]:
        sys.modules.pop(mod, None)
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            m = importlib.import_module(mod)
        assert hasattr(m, attr), (mod, attr)
        assert any(issubclass(x.category, DeprecationWarning) for x in w), mod


def test_protocol_options_trim_packages():
    code = "import setup; print(','.join(setup._packages()))"
    env = dict(os.environ, TRITON_ENABLE_PYTHON_GRPC="OFF")
    out = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True, env=env,
                         check=True).stdout
    pk = out.strip().split(",")
    assert "tritonclient.http" in pk and "tritonclient.grpc" not in pk and "tritongrpcclient" not in pk
    env = dict(os.environ, TRITON_ENABLE_PYTHON_HTTP="OFF")
    pk = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True, env=env,
                        check=True).stdout.strip().split(",")
    assert "tritonclient.grpc" in pk and "tritonclient.http.aio" not in pk
