"""TLS on both protocols, every client flavour (reference surface:
``HttpSslOptions`` src/c++/library/http_client.cc:234-299, ``SslOptions``
src/c++/library/grpc_client.h:43-59, Python ``ssl``/``ssl_options``/``insecure``
tc/http/_client.py and ``ssl``/``root_certificates``/``private_key``/
``certificate_chain`` tc/grpc/_client.py:177-239, and the C++ examples'
``--ssl``/``--ca-certs`` flags).

A throw-away CA and a server certificate (SAN IP:127.0.0.1, DNS:localhost)
are minted with /usr/bin/openssl; an unrelated CA plays the wrong trust
root.  The test server serves HTTPS (aiohttp) and gRPC over TLS (grpc.aio),
optionally requiring client certificates (mutual TLS)."""

import asyncio
import os
import shutil
import ssl
import subprocess

import numpy as np
import pytest

import tritonclient.grpc as grpcclient
import tritonclient.http as httpclient
from tritonclient.utils import InferenceServerException

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "csrc", "cpp", "build", "bin")

pytestmark = pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl not installed")

A = np.arange(16, dtype=np.int32).reshape(1, 16)
B = np.ones((1, 16), dtype=np.int32)


def _openssl(*args, cwd):
    subprocess.run(["openssl", *args], cwd=cwd, check=True, capture_output=True)


@pytest.fixture(scope="module")
def certs(tmp_path_factory):
    d = tmp_path_factory.mktemp("tls")
    for ca in ("ca", "other"):
        _openssl("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", ca + ".key", "-out", ca + ".pem",
                 "-days", "2", "-subj", "/CN=%s-test-ca" % ca, cwd=d)
    (d / "server.ext").write_text("subjectAltName=IP:127.0.0.1,DNS:localhost\nbasicConstraints=CA:FALSE\n")
    (d / "client.ext").write_text("basicConstraints=CA:FALSE\nextendedKeyUsage=clientAuth\n")
    for who in ("server", "client"):
        _openssl("req", "-newkey", "rsa:2048", "-nodes", "-keyout", who + ".key", "-out", who + ".csr", "-subj",
                 "/CN=" + ("localhost" if who == "server" else "test-client"), cwd=d)
        _openssl("x509", "-req", "-in", who + ".csr", "-CA", "ca.pem", "-CAkey", "ca.key", "-CAcreateserial", "-out",
                 who + ".pem", "-days", "2", "-extfile", who + ".ext", cwd=d)
    return {k: str(d / (k + ".pem")) for k in ("ca", "other", "server", "client")} | {
        "server_key": str(d / "server.key"), "client_key": str(d / "client.key")}


def _server(certs, mutual=False):
    from triton_client_amd.server import ServerHandle

    tls = {"cert": certs["server"], "key": certs["server_key"]}
    if mutual:
        tls["client_ca"] = certs["ca"]
    return ServerHandle(tls=tls).start()


@pytest.fixture(scope="module")
def tls_server(certs):
    h = _server(certs)
    yield h
    h.stop()


@pytest.fixture(scope="module")
def mtls_server(certs):
    h = _server(certs, mutual=True)
    yield h
    h.stop()


def _infer(mod, c):
    ins = [mod.InferInput("INPUT0", [1, 16], "INT32"), mod.InferInput("INPUT1", [1, 16], "INT32")]
    ins[0].set_data_from_numpy(A)
    ins[1].set_data_from_numpy(B)
    r = c.infer("simple", ins)
    np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), A + B)


def test_http_sync_verified_wrong_ca_and_insecure(tls_server, certs):
    c = httpclient.InferenceServerClient(tls_server.http_url, ssl=True, ssl_options={"ca_certs": certs["ca"]})
    assert c.is_server_live()
    _infer(httpclient, c)
    c.close()
    bad = httpclient.InferenceServerClient(tls_server.http_url, ssl=True, ssl_options={"ca_certs": certs["other"]})
    with pytest.raises((InferenceServerException, ssl.SSLError, OSError)):
        bad.is_server_live()
    bad.close()
    # insecure: no trust root at all, verification off (reference `insecure=True`)
    ins = httpclient.InferenceServerClient(tls_server.http_url, ssl=True, insecure=True)
    assert ins.is_server_live()
    ins.close()
    # plaintext against the TLS port fails instead of hanging
    plain = httpclient.InferenceServerClient(tls_server.http_url, network_timeout=5.0)
    with pytest.raises(Exception):
        plain.is_server_live()
    plain.close()


def test_grpc_sync_verified_and_wrong_ca(tls_server, certs):
    url = "localhost:%d" % tls_server.grpc_port
    c = grpcclient.InferenceServerClient(url, ssl=True, root_certificates=certs["ca"])
    assert c.is_server_live()
    _infer(grpcclient, c)
    c.close()
    bad = grpcclient.InferenceServerClient(url, ssl=True, root_certificates=certs["other"])
    with pytest.raises(InferenceServerException):
        bad.is_server_live(client_timeout=5)
    bad.close()


def test_aio_clients_over_tls(tls_server, certs):
    import tritonclient.grpc.aio as grpcaio
    import tritonclient.http.aio as httpaio

    async def run():
        ctx = ssl.create_default_context(cafile=certs["ca"])
        h = httpaio.InferenceServerClient(tls_server.http_url, ssl=True, ssl_context=ctx)
        assert await h.is_server_live()
        md = await h.get_server_metadata()
        assert md["name"]
        await h.close()
        g = grpcaio.InferenceServerClient("localhost:%d" % tls_server.grpc_port, ssl=True,
                                          root_certificates=certs["ca"])
        assert await g.is_server_live()
        await g.close()

    asyncio.run(run())


def test_grpc_mutual_tls(mtls_server, certs):
    url = "localhost:%d" % mtls_server.grpc_port
    c = grpcclient.InferenceServerClient(url, ssl=True, root_certificates=certs["ca"], private_key=certs["client_key"],
                                         certificate_chain=certs["client"])
    _infer(grpcclient, c)
    c.close()
    anon = grpcclient.InferenceServerClient(url, ssl=True, root_certificates=certs["ca"])
    with pytest.raises(InferenceServerException):
        anon.is_server_live(client_timeout=5)
    anon.close()
    h = httpclient.InferenceServerClient(mtls_server.http_url, ssl=True,
                                         ssl_options={"ca_certs": certs["ca"], "certfile": certs["client"],
                                                      "keyfile": certs["client_key"]})
    _infer(httpclient, h)
    h.close()


def _cpp(name, *args):
    exe = os.path.join(BIN, name)
    if not os.path.exists(exe):
        pytest.skip("csrc/cpp not built")
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=60)


def test_cpp_http_example_tls_flags(tls_server, certs):
    url = "https://127.0.0.1:%d" % tls_server.http_port
    r = _cpp("simple_http_infer_client", "-u", url, "--ca-certs", certs["ca"])
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr
    r = _cpp("simple_http_infer_client", "-u", url, "--ca-certs", certs["other"])
    assert r.returncode != 0
    r = _cpp("simple_http_infer_client", "-u", url, "--verify-peer", "0", "--verify-host", "0")
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr


def test_cpp_grpc_example_tls_flags(tls_server, mtls_server, certs):
    r = _cpp("simple_grpc_infer_client", "-u", "localhost:%d" % tls_server.grpc_port, "--ssl", "--root-certificates",
             certs["ca"])
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr
    r = _cpp("simple_grpc_infer_client", "-u", "localhost:%d" % tls_server.grpc_port, "--ssl", "--root-certificates",
             certs["other"])
    assert r.returncode != 0
    r = _cpp("simple_grpc_infer_client", "-u", "localhost:%d" % mtls_server.grpc_port, "--ssl", "--root-certificates",
             certs["ca"], "--private-key", certs["client_key"], "--certificate-chain", certs["client"])
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr


def test_perf_analyzer_ssl_flags(tls_server, mtls_server, certs):
    """perf_analyzer's --ssl-grpc-* / --ssl-https-* flags against the TLS server."""
    pa = os.path.join(BIN, "perf_analyzer")
    if not os.path.exists(pa):
        pytest.skip("csrc/cpp not built")

    def run(*args):
        return subprocess.run([pa, "-m", "simple", "--concurrency-range", "2", "-p", "300", "-r", "3", "-s", "80",
                               *args], capture_output=True, text=True, timeout=120)

    r = run("-i", "grpc", "-u", "localhost:%d" % tls_server.grpc_port, "--ssl-grpc-use-ssl",
            "--ssl-grpc-root-certifications-file", certs["ca"])
    assert r.returncode == 0 and "Throughput" in r.stdout, r.stdout[-1500:] + r.stderr[-1500:]
    r = run("-i", "grpc", "-u", "localhost:%d" % mtls_server.grpc_port, "--ssl-grpc-root-certifications-file",
            certs["ca"], "--ssl-grpc-private-key-file", certs["client_key"], "--ssl-grpc-certificate-chain-file",
            certs["client"])
    assert r.returncode == 0 and "Throughput" in r.stdout, r.stdout[-1500:] + r.stderr[-1500:]
    r = run("-i", "http", "-u", "127.0.0.1:%d" % tls_server.http_port, "--ssl-https-ca-certificates-file", certs["ca"])
    assert r.returncode == 0 and "Throughput" in r.stdout, r.stdout[-1500:] + r.stderr[-1500:]
    r = run("-i", "http", "-u", "127.0.0.1:%d" % tls_server.http_port, "--ssl-https-ca-certificates-file",
            certs["other"])
    assert r.returncode != 0
    r = run("-i", "http", "-u", "127.0.0.1:%d" % tls_server.http_port, "--ssl-https-verify-peer", "0",
            "--ssl-https-verify-host", "0")
    assert r.returncode == 0, r.stdout[-1500:] + r.stderr[-1500:]
