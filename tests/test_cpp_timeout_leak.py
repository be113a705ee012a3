"""The reference's two CLI test harnesses, ported to our C++ clients and run
against the CPU test server:

* client_timeout_test (reference src/c++/tests/client_timeout_test.cc):
  sync/async/stream inference with a client timeout against the slow
  custom_identity_int32 model (500 ms), and every gRPC control-plane call
  with timeout_ms (the server's ``tc-fault-delay-ms`` header makes them slow);
* memory_leak_test (reference src/c++/tests/memory_leak_test.cc): repeated
  inference with a new or a reused client, with an RSS-growth bound in place
  of the reference's external leak checker.
"""

import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "csrc", "cpp", "build", "bin")

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(BIN, "client_timeout_test")),
                                reason="csrc/cpp not built")


def _run(name, args, timeout=120):
    return subprocess.run([os.path.join(BIN, name)] + list(args), capture_output=True, text=True, timeout=timeout)


MODES = [("http", []), ("http", ["-a"]), ("grpc", []), ("grpc", ["-a"]), ("grpc", ["-s"])]


@pytest.mark.parametrize("proto,flags", MODES, ids=["http", "http-async", "grpc", "grpc-async", "grpc-stream"])
def test_infer_within_timeout(cpu_server, proto, flags):
    url = cpu_server.http_url if proto == "http" else cpu_server.grpc_url
    r = _run("client_timeout_test", ["-i", proto, "-u", url, "-t", "20000000"] + flags)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "PASS: infer" in r.stdout


@pytest.mark.parametrize("proto,flags", MODES, ids=["http", "http-async", "grpc", "grpc-async", "grpc-stream"])
def test_infer_deadline_exceeded(cpu_server, proto, flags):
    """100 ms client timeout against a 500 ms model: every path reports Deadline Exceeded."""
    url = cpu_server.http_url if proto == "http" else cpu_server.grpc_url
    r = _run("client_timeout_test", ["-i", proto, "-u", url, "-t", "100000"] + flags)
    assert r.returncode == 1, r.stdout[-2000:] + r.stderr[-2000:]
    assert "Deadline Exceeded" in r.stdout + r.stderr, r.stdout[-2000:] + r.stderr[-2000:]


def test_control_plane_apis_within_timeout(cpu_server):
    try:
        r = _run("client_timeout_test", ["-i", "grpc", "-u", cpu_server.grpc_url, "-p", "-t", "20000"])
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        assert "PASS: control-plane APIs" in r.stdout
    finally:
        _reload(cpu_server)


def test_control_plane_apis_deadline_exceeded(cpu_server):
    """Each control-plane call delayed 300 ms by the server with a 50 ms timeout."""
    try:
        r = _run("client_timeout_test", ["-i", "grpc", "-u", cpu_server.grpc_url, "-p", "-t", "50",
                                         "-H", "tc-fault-delay-ms:300"])
        assert r.returncode == 1, r.stdout[-3000:] + r.stderr[-3000:]
        failed = [ln for ln in r.stdout.splitlines() if ln.startswith("error: Failed on")]
        assert len(failed) >= 18, r.stdout
        assert all("Deadline Exceeded" in ln for ln in failed), r.stdout
    finally:
        _reload(cpu_server)


def _reload(cpu_server):
    import time

    import tritonclient.grpc as grpcclient

    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    time.sleep(0.5)  # delayed RPCs abandoned by the client may still be running server-side
    c.load_model("custom_identity_int32")
    assert c.is_model_ready("custom_identity_int32")
    c.unregister_system_shared_memory()


@pytest.mark.parametrize("proto", ["http", "grpc"])
@pytest.mark.parametrize("reuse", [False, True], ids=["new-client", "reuse"])
def test_memory_leak_soak(cpu_server, proto, reuse):
    url = cpu_server.http_url if proto == "http" else cpu_server.grpc_url
    args = ["-i", proto, "-u", url, "-r", "300", "-M", "identity_int32", "-w", "1", "-m", "8192"]
    if reuse:
        args.append("-R")
    r = _run("memory_leak_test", args, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "PASS" in r.stdout
    print(r.stdout.strip().splitlines()[-2])
