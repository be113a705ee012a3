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


def _libb64(data):
    """The reference's libb64 framing, written from its documented behaviour
    (src/c++/library/cencode.c:78-81,106): '\\n' after each 72 characters of
    complete 3-byte groups, then the padding, then a terminating '\\n'."""
    import base64

    flat = base64.b64encode(bytes(data)).decode()
    full = len(data) // 3 * 4
    out = []
    for i, ch in enumerate(flat):
        out.append(ch)
        if i < full and (i + 1) % 72 == 0:
            out.append("\n")
    return "".join(out) + "\n"


def _capture_bodies(args, n_requests=2):
    """Run http_body_test against a raw socket that records each request's
    (request line, body) and answers 200 "{}"."""
    import json
    import socket
    import threading

    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(4)
    port = srv.getsockname()[1]
    got = []

    def serve():
        conn, _ = srv.accept()
        buf = b""
        while len(got) < n_requests:
            while b"\r\n\r\n" not in buf:
                d = conn.recv(65536)
                if not d:
                    return
                buf += d
            head, buf = buf.split(b"\r\n\r\n", 1)
            n = [int(h.split(b":")[1]) for h in head.split(b"\r\n") if h.lower().startswith(b"content-length")][0]
            while len(buf) < n:
                buf += conn.recv(65536)
            body, buf = buf[:n], buf[n:]
            got.append((head.split(b"\r\n")[0].decode(), json.loads(body)))
            conn.sendall(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\nContent-Type: application/json\r\n\r\n{}")
        conn.close()

    t = threading.Thread(target=serve, daemon=True)
    t.start()
    r = subprocess.run([os.path.join(BIN, "http_body_test"), "127.0.0.1:%d" % port] + args, capture_output=True,
                       text=True, timeout=60)
    t.join(10)
    srv.close()
    assert r.returncode == 0, r.stderr
    return got


@pytest.mark.parametrize("nbytes", [0, 1, 2, 53, 54, 55, 200])
def test_cpp_http_base64_is_libb64_framed(nbytes):
    """C7: LoadModel file overrides and the CUDA-shm register handle carry
    base64 with the reference's libb64 line framing, byte for byte."""
    got = _capture_bodies([str(nbytes)])
    (load_line, load), (reg_line, reg) = got
    assert load_line.startswith("POST /v2/repository/models/b64_model/load")
    content = bytes(i % 251 for i in range(nbytes))
    assert load["parameters"]["file:1/model.onnx"] == _libb64(content)
    assert reg_line.startswith("POST /v2/cudasharedmemory/region/b64_region/register")
    assert reg["raw_handle"]["b64"] == _libb64(bytes(range(64)))
    # pinned literal for the 64-byte handle: wrapped after 72 characters, trailing newline
    assert reg["raw_handle"]["b64"] == (
        "AAECAwQFBgcICQoLDA0ODxAREhMUFRYXGBkaGxwdHh8gISIjJCUmJygpKissLS4vMDEyMzQ1\n"
        "Njc4OTo7PD0+Pw==\n")
