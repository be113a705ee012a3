"""C++ client library acceptance: cc_client_test and every C++ example
(ports of reference src/c++/examples/*) against the CPU test server.  GPU
examples (HIP shared memory, image classification) run in
tests/test_examples_gpu.py."""

import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "csrc", "cpp", "build", "bin")

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(BIN, "cc_client_test")), reason="csrc/cpp not built")

CPU = [
    ("simple_http_infer_client", "http", []),
    ("simple_http_infer_client", "http", ["-i", "gzip", "-o", "deflate"]),
    ("simple_grpc_infer_client", "grpc", []),
    ("simple_grpc_infer_client", "grpc", ["-C", "gzip", "-t", "5000000"]),
    ("simple_http_async_infer_client", "http", []),
    ("simple_grpc_async_infer_client", "grpc", []),
    ("simple_http_string_infer_client", "http", []),
    ("simple_grpc_string_infer_client", "grpc", []),
    ("simple_http_health_metadata", "http", []),
    ("simple_grpc_health_metadata", "grpc", []),
    ("simple_http_model_control", "http", []),
    ("simple_grpc_model_control", "grpc", []),
    ("simple_http_sequence_sync_infer_client", "http", []),
    ("simple_grpc_sequence_sync_infer_client", "grpc", ["-d"]),
    ("simple_grpc_sequence_stream_infer_client", "grpc", []),
    ("simple_http_shm_client", "http", []),
    ("simple_grpc_shm_client", "grpc", []),
    ("simple_grpc_keepalive_client", "grpc", []),
    ("simple_grpc_custom_args_client", "grpc", []),
    ("simple_grpc_custom_repeat", "grpc", ["-r", "6"]),
    ("reuse_infer_objects_client", "http", ["-i", "http"]),
    ("reuse_infer_objects_client", "grpc", ["-i", "grpc"]),
]


def run_bin(name, url, args, timeout=120):
    return subprocess.run([os.path.join(BIN, name), "-u", url] + list(args), capture_output=True, text=True,
                          timeout=timeout)


@pytest.mark.parametrize("name,proto,args", CPU, ids=["%s%s" % (n, "".join(a)) for n, _, a in CPU])
def test_cpp_example(cpu_server, name, proto, args):
    url = cpu_server.http_url if proto == "http" else cpu_server.grpc_url
    r = run_bin(name, url, args)
    assert r.returncode == 0, "%s failed:\n%s\n%s" % (name, r.stdout[-2000:], r.stderr[-2000:])
    assert "PASS" in r.stdout


def test_cc_client_test(cpu_server):
    r = subprocess.run([os.path.join(BIN, "cc_client_test"), cpu_server.http_url, cpu_server.grpc_url],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_every_reference_cpp_example_is_ported():
    ref = {"ensemble_image_client", "image_client", "reuse_infer_objects_client",
           "simple_grpc_async_infer_client", "simple_grpc_cudashm_client", "simple_grpc_custom_args_client",
           "simple_grpc_custom_repeat", "simple_grpc_health_metadata", "simple_grpc_infer_client",
           "simple_grpc_keepalive_client", "simple_grpc_model_control", "simple_grpc_sequence_stream_infer_client",
           "simple_grpc_sequence_sync_infer_client", "simple_grpc_shm_client", "simple_grpc_string_infer_client",
           "simple_http_async_infer_client", "simple_http_cudashm_client", "simple_http_health_metadata",
           "simple_http_infer_client", "simple_http_model_control", "simple_http_sequence_sync_infer_client",
           "simple_http_shm_client", "simple_http_string_infer_client"}
    assert ref <= set(os.listdir(BIN)), sorted(ref - set(os.listdir(BIN)))
