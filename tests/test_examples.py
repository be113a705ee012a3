"""Every Python example in examples/python (ports of reference
src/python/examples/*) runs against the CPU test server and reports PASS.
GPU-only examples (HIP shared memory, densenet classification) are in
tests/test_examples_gpu.py."""

import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(REPO, "examples", "python")

CPU_EXAMPLES = [
    ("simple_http_infer_client.py", "http", []),
    ("simple_http_infer_client.py", "http", ["-C", "gzip"]),
    ("simple_grpc_infer_client.py", "grpc", []),
    ("simple_grpc_infer_client.py", "grpc", ["-C", "deflate", "-t", "10"]),
    ("simple_http_async_infer_client.py", "http", []),
    ("simple_grpc_async_infer_client.py", "grpc", []),
    ("simple_http_string_infer_client.py", "http", []),
    ("simple_grpc_string_infer_client.py", "grpc", []),
    ("simple_http_health_metadata.py", "http", []),
    ("simple_grpc_health_metadata.py", "grpc", []),
    ("simple_http_model_control.py", "http", []),
    ("simple_grpc_model_control.py", "grpc", []),
    ("simple_http_sequence_sync_infer_client.py", "http", []),
    ("simple_http_sequence_sync_infer_client.py", "http", ["-d"]),
    ("simple_grpc_sequence_sync_infer_client.py", "grpc", []),
    ("simple_grpc_sequence_stream_infer_client.py", "grpc", []),
    ("simple_grpc_sequence_stream_infer_client.py", "grpc", ["-d", "-o", "10"]),
    ("simple_grpc_custom_repeat.py", "grpc", ["-r", "5"]),
    ("simple_http_shm_client.py", "http", []),
    ("simple_grpc_shm_client.py", "grpc", []),
    ("simple_http_shm_string_client.py", "http", []),
    ("simple_grpc_shm_string_client.py", "grpc", []),
    ("simple_grpc_keepalive_client.py", "grpc", []),
    ("simple_grpc_custom_args_client.py", "grpc", []),
    ("simple_http_aio_infer_client.py", "http", []),
    ("simple_grpc_aio_infer_client.py", "grpc", []),
    ("simple_grpc_aio_sequence_stream_infer_client.py", "grpc", []),
    ("reuse_infer_objects_client.py", "http", ["-i", "http"]),
    ("reuse_infer_objects_client.py", "grpc", ["-i", "grpc"]),
    ("grpc_client.py", "grpc", []),
    ("grpc_explicit_int_content_client.py", "grpc", []),
    ("grpc_explicit_int8_content_client.py", "grpc", []),
    ("grpc_explicit_byte_content_client.py", "grpc", []),
    ("memory_growth_test.py", "http", ["-r", "30"]),
    ("memory_growth_test.py", "grpc", ["-i", "grpc", "-r", "30"]),
]


def run_example(script, url, args, timeout=120):
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([REPO, EX, env.get("PYTHONPATH", "")])
    return subprocess.run([sys.executable, os.path.join(EX, script), "-u", url] + list(args), cwd=EX, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("script,proto,args", CPU_EXAMPLES,
                         ids=["%s%s" % (s, "".join(a)) for s, _, a in CPU_EXAMPLES])
def test_example(cpu_server, script, proto, args):
    url = cpu_server.http_url if proto == "http" else cpu_server.grpc_url
    r = run_example(script, url, args)
    assert r.returncode == 0, "%s failed:\n%s\n%s" % (script, r.stdout[-2000:], r.stderr[-2000:])
    assert "PASS" in r.stdout, r.stdout[-2000:]


def test_every_reference_example_is_ported():
    ours = set(os.listdir(EX))
    ref = {
        "ensemble_image_client.py", "grpc_client.py", "grpc_explicit_byte_content_client.py",
        "grpc_explicit_int8_content_client.py", "grpc_explicit_int_content_client.py", "grpc_image_client.py",
        "image_client.py", "memory_growth_test.py", "reuse_infer_objects_client.py",
        "simple_grpc_aio_infer_client.py", "simple_grpc_aio_sequence_stream_infer_client.py",
        "simple_grpc_async_infer_client.py", "simple_grpc_cudashm_client.py", "simple_grpc_custom_args_client.py",
        "simple_grpc_custom_repeat.py", "simple_grpc_health_metadata.py", "simple_grpc_infer_client.py",
        "simple_grpc_keepalive_client.py", "simple_grpc_model_control.py",
        "simple_grpc_sequence_stream_infer_client.py", "simple_grpc_sequence_sync_infer_client.py",
        "simple_grpc_shm_client.py", "simple_grpc_shm_string_client.py", "simple_grpc_string_infer_client.py",
        "simple_http_aio_infer_client.py", "simple_http_async_infer_client.py", "simple_http_cudashm_client.py",
        "simple_http_health_metadata.py", "simple_http_infer_client.py", "simple_http_model_control.py",
        "simple_http_sequence_sync_infer_client.py", "simple_http_shm_client.py",
        "simple_http_shm_string_client.py", "simple_http_string_infer_client.py",
    }
    assert ref <= ours, sorted(ref - ours)
