"""tcserve, the native gRPC front end (csrc/cpp/server), on CPU.

The fast path (ModelInfer for models with execute_native) must be
indistinguishable on the wire from the Python path; everything else is
proxied to the grpc.aio server behind it.
"""

import json

import numpy as np
import pytest

import tritonclient.grpc as grpcclient
from tritonclient.utils import InferenceServerException
from tritonclient.utils import shared_memory as shm
from triton_client_amd.server import native_frontend

pytestmark = pytest.mark.skipif(not native_frontend.available(), reason="libtcserve.so not built")


def _inputs(a, b):
    i0 = grpcclient.InferInput("INPUT0", list(a.shape), "INT32")
    i0.set_data_from_numpy(a)
    i1 = grpcclient.InferInput("INPUT1", list(b.shape), "INT32")
    i1.set_data_from_numpy(b)
    return [i0, i1]


def test_fast_path_results_and_counters(cpu_server):
    nf = cpu_server.server.native_frontend
    assert nf is not None
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    before = nf.counters()["native_requests"]
    a = np.arange(48, dtype=np.int32).reshape(3, 16)
    b = np.full((3, 16), 5, dtype=np.int32)
    r = c.infer("add_sub_batched", _inputs(a, b), request_id="abc")
    np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), a + b)
    np.testing.assert_array_equal(r.as_numpy("OUTPUT1"), a - b)
    resp = r.get_response()
    assert resp.id == "abc" and resp.model_name == "add_sub_batched" and resp.model_version == "1"
    # a subset of outputs
    r = c.infer("add_sub_batched", _inputs(a, b), outputs=[grpcclient.InferRequestedOutput("OUTPUT1")])
    np.testing.assert_array_equal(r.as_numpy("OUTPUT1"), a - b)
    assert r.as_numpy("OUTPUT0") is None
    assert nf.counters()["native_requests"] == before + 2


def test_fast_path_async_batches(cpu_server):
    cpu_server.server.native_frontend.set_idle_dispatch("add_sub_batched", False)
    try:
        _async_batches(cpu_server)
    finally:
        cpu_server.server.native_frontend.set_idle_dispatch("add_sub_batched", True)


def _async_batches(cpu_server):
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    results = []
    import threading

    done = threading.Event()

    def cb(result, error):
        results.append((result, error))
        if len(results) == 32:
            done.set()

    for k in range(32):
        a = np.full((1, 16), k, dtype=np.int32)
        c.async_infer("add_sub_batched", _inputs(a, a), cb)
    assert done.wait(30)
    assert all(e is None for _, e in results)
    got = sorted(int(r.as_numpy("OUTPUT0")[0, 0]) for r, _ in results)
    assert got == [2 * k for k in range(32)]
    st = c.get_inference_statistics("add_sub_batched", as_json=True)["model_stats"][0]
    assert int(st["inference_count"]) >= 32
    # dynamic batching merged some of them
    assert int(st["execution_count"]) < int(st["inference_stats"]["success"]["count"])


def test_preferred_batch_size_caps_batches(cpu_server):
    """With preferred_batch_size [2] the native batcher dispatches 2-row batches
    as soon as they form instead of filling max_batch_size (8)."""
    import threading

    nf = cpu_server.server.native_frontend
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)

    def sizes():
        st = c.get_inference_statistics("add_sub_batched", as_json=True)["model_stats"][0]
        return {int(b["batch_size"]): int(b["compute_infer"]["count"]) for b in st.get("batch_stats", [])}

    before = sizes()
    nf.set_preferred("add_sub_batched", [2])
    nf.set_idle_dispatch("add_sub_batched", False)  # batch even while the (fast) model is idle
    try:
        done = threading.Event()
        got = []

        def cb(result, error):
            got.append(error)
            if len(got) == 24:
                done.set()

        for k in range(24):
            a = np.full((1, 16), k, dtype=np.int32)
            c.async_infer("add_sub_batched", _inputs(a, a), cb)
        assert done.wait(30)
        assert all(e is None for e in got)
    finally:
        nf.set_preferred("add_sub_batched", [])
        nf.set_idle_dispatch("add_sub_batched", True)
    after = sizes()
    new = {bs: after.get(bs, 0) - before.get(bs, 0) for bs in after}
    assert all(n == 0 for bs, n in new.items() if bs > 2), new
    assert new.get(2, 0) > 0, new
    with pytest.raises(KeyError):
        nf.set_preferred("no_such_model", [2])
    with pytest.raises(KeyError):
        nf.set_idle_dispatch("no_such_model", False)


def test_idle_dispatch_toggle_keeps_results(cpu_server):
    """Idle-aware dispatch on/off only changes when batches go out, never results."""
    nf = cpu_server.server.native_frontend
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    for on in (False, True):
        nf.set_idle_dispatch("add_sub_batched", on)
        a = np.arange(16, dtype=np.int32).reshape(1, 16)
        r = c.infer("add_sub_batched", _inputs(a, a))
        np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), 2 * a)


def test_fast_path_system_shm(cpu_server):
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    nf = cpu_server.server.native_frontend
    a = np.arange(16, dtype=np.int32).reshape(1, 16)
    inp = shm.create_shared_memory_region("nf_in", "/nf_in", 128)
    out = shm.create_shared_memory_region("nf_out", "/nf_out", 128)
    try:
        shm.set_shared_memory_region(inp, [a, a * 3])
        c.register_system_shared_memory("nf_in", "/nf_in", 128)
        c.register_system_shared_memory("nf_out", "/nf_out", 128)
        i0 = grpcclient.InferInput("INPUT0", [1, 16], "INT32")
        i0.set_shared_memory("nf_in", 64)
        i1 = grpcclient.InferInput("INPUT1", [1, 16], "INT32")
        i1.set_shared_memory("nf_in", 64, offset=64)
        o0 = grpcclient.InferRequestedOutput("OUTPUT0")
        o0.set_shared_memory("nf_out", 64)
        o1 = grpcclient.InferRequestedOutput("OUTPUT1")
        o1.set_shared_memory("nf_out", 64, offset=64)
        before = nf.counters()["native_requests"]
        r = c.infer("add_sub_batched", [i0, i1], outputs=[o0, o1])
        assert nf.counters()["native_requests"] == before + 1
        assert r.as_numpy("OUTPUT0") is None
        o = r.get_output("OUTPUT1")
        assert o.parameters["shared_memory_region"].string_param == "nf_out"
        res0 = shm.get_contents_as_numpy(out, np.int32, [1, 16])
        res1 = shm.get_contents_as_numpy(out, np.int32, [1, 16], offset=64)
        np.testing.assert_array_equal(res0, a * 4)
        np.testing.assert_array_equal(res1, -a * 2)
        # output region too small -> the Python server's error text
        small = grpcclient.InferRequestedOutput("OUTPUT0")
        small.set_shared_memory("nf_out", 32)
        with pytest.raises(InferenceServerException, match="should be at least 64 bytes"):
            c.infer("add_sub_batched", [i0, i1], outputs=[small])
        # unknown region
        bad = grpcclient.InferInput("INPUT0", [1, 16], "INT32")
        bad.set_shared_memory("nope", 64)
        with pytest.raises(InferenceServerException, match="Unable to find shared memory region: 'nope'"):
            c.infer("add_sub_batched", [bad, i1])
        # unregister -> mirror forgets it
        c.unregister_system_shared_memory("nf_in")
        with pytest.raises(InferenceServerException, match="nf_in"):
            c.infer("add_sub_batched", [i0, i1])
    finally:
        c.unregister_system_shared_memory()
        shm.destroy_shared_memory_region(inp)
        shm.destroy_shared_memory_region(out)


def test_fallbacks_are_proxied(cpu_server):
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    nf = cpu_server.server.native_frontend
    before = nf.counters()
    a = np.ones((1, 16), dtype=np.int32)
    # wrong input count: the Python server produces the error
    with pytest.raises(InferenceServerException, match="expected 2 inputs"):
        c.infer("add_sub_batched", _inputs(a, a)[:1])
    # classification output is not a fast-path feature
    r = c.infer("add_sub_batched", _inputs(a, a), outputs=[grpcclient.InferRequestedOutput("OUTPUT0", class_count=2)])
    assert r.as_numpy("OUTPUT0").shape == (1, 2)
    # non-native model
    r = c.infer("simple", _inputs(a, a))
    np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), a * 2)
    after = nf.counters()
    assert after["proxied_calls"] >= before["proxied_calls"] + 3
    assert after["native_requests"] == before["native_requests"]
    assert c.is_server_live() and c.is_model_ready("add_sub_batched")


def test_unload_reload_reregisters(cpu_server):
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    nf = cpu_server.server.native_frontend
    c.unload_model("add_sub_batched")
    a = np.ones((1, 16), dtype=np.int32)
    with pytest.raises(InferenceServerException):
        c.infer("add_sub_batched", _inputs(a, a))
    c.load_model("add_sub_batched")
    before = nf.counters()["native_requests"]
    r = c.infer("add_sub_batched", _inputs(a, a))
    np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), a * 2)
    assert nf.counters()["native_requests"] == before + 1


def test_fast_path_large_inband_tensor(cpu_server):
    """frontend_sink: 600 KB/row in-band tensors parsed in place (no copy of
    raw_input_contents) for several batch sizes and compressed requests."""
    nf = cpu_server.server.native_frontend
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    before = nf.counters()["native_requests"]
    rng = np.random.default_rng(0)
    for rows in (1, 3, 8):
        x = rng.standard_normal((rows, 3, 224, 224)).astype(np.float32)
        i = grpcclient.InferInput("data_0", list(x.shape), "FP32")
        i.set_data_from_numpy(x)
        for comp in (None, "gzip"):
            r = c.infer("frontend_sink", [i], compression_algorithm=comp)
            y = r.as_numpy("fc6_1")
            assert y.shape == (rows, 1000)
            np.testing.assert_array_equal(y, np.repeat(x.reshape(rows, -1)[:, :1], 1000, axis=1))
    assert nf.counters()["native_requests"] - before == 6
    # a wrong byte size is rejected by the fast path with the Python server's message
    x = np.zeros((1, 3, 224, 224), np.float32)
    i = grpcclient.InferInput("data_0", [2, 3, 224, 224], "FP32")
    i.set_data_from_numpy(np.zeros((2, 3, 224, 224), np.float32))
    i._raw = x.tobytes()  # bypass the client-side shape check: the server must reject it
    with pytest.raises(InferenceServerException, match="unexpected byte size"):
        c.infer("frontend_sink", [i])


# -- KServe REST through tcserve (csrc/cpp/server: native infer path + relay) ----------------
import socket  # noqa: E402

import tritonclient.http as httpclient  # noqa: E402


def _http_inputs(a, b, binary=True):
    i0 = httpclient.InferInput("INPUT0", list(a.shape), "INT32")
    i0.set_data_from_numpy(a, binary_data=binary)
    i1 = httpclient.InferInput("INPUT1", list(b.shape), "INT32")
    i1.set_data_from_numpy(b, binary_data=binary)
    return [i0, i1]


def test_http_binary_infer_runs_native(cpu_server):
    nf = cpu_server.server.native_frontend
    c = httpclient.InferenceServerClient(cpu_server.http_url)
    a = np.arange(32, dtype=np.int32).reshape(2, 16)
    b = np.full((2, 16), 3, dtype=np.int32)
    before = nf.counters()
    outs = [httpclient.InferRequestedOutput("OUTPUT0", binary_data=True),
            httpclient.InferRequestedOutput("OUTPUT1", binary_data=True)]
    r = c.infer("add_sub_batched", _http_inputs(a, b), outputs=outs, request_id="r1")
    np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), a + b)
    np.testing.assert_array_equal(r.as_numpy("OUTPUT1"), a - b)
    resp = r.get_response()
    assert resp["model_name"] == "add_sub_batched" and resp["id"] == "r1"
    assert resp["outputs"][0]["shape"] == [2, 16] and resp["outputs"][0]["datatype"] == "INT32"
    # no outputs listed: binary_data_output (the client's default) -> native too
    r = c.infer("add_sub_batched", _http_inputs(a, b))
    np.testing.assert_array_equal(r.as_numpy("OUTPUT1"), a - b)
    after = nf.counters()
    assert after["native_requests"] == before["native_requests"] + 2
    assert after["proxied_calls"] == before["proxied_calls"]


def test_http_json_tensors_and_control_plane_are_relayed(cpu_server):
    nf = cpu_server.server.native_frontend
    c = httpclient.InferenceServerClient(cpu_server.http_url)
    a = np.arange(16, dtype=np.int32).reshape(1, 16)
    before = nf.counters()
    # JSON input data and JSON outputs: the Python server answers, same results
    r = c.infer("add_sub_batched", _http_inputs(a, a, binary=False),
                outputs=[httpclient.InferRequestedOutput("OUTPUT0", binary_data=False)])
    np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), 2 * a)
    assert c.is_server_live() and c.is_model_ready("add_sub_batched")
    assert c.get_model_metadata("add_sub_batched")["name"] == "add_sub_batched"
    with pytest.raises(InferenceServerException):
        c.get_model_metadata("no_such_model")
    # gzip'd request body: relayed (the native path takes identity bodies only)
    r = c.infer("add_sub_batched", _http_inputs(a, a), request_compression_algorithm="gzip",
                response_compression_algorithm="gzip")
    np.testing.assert_array_equal(r.as_numpy("OUTPUT1"), 0 * a)
    assert nf.counters()["proxied_calls"] >= before["proxied_calls"] + 5


def test_http_native_errors_and_system_shm(cpu_server):
    c = httpclient.InferenceServerClient(cpu_server.http_url)
    a = np.arange(16, dtype=np.int32).reshape(1, 16)
    i0 = httpclient.InferInput("INPUT0", [1, 16], "INT32")
    i0.set_shared_memory("no_such_region", 64)
    i1 = _http_inputs(a, a)[1]
    with pytest.raises(InferenceServerException, match="Unable to find shared memory region"):
        c.infer("add_sub_batched", [i0, i1])
    h = shm.create_shared_memory_region("http_in0", "/http_in0_native", 64)
    ho = shm.create_shared_memory_region("http_out0", "/http_out0_native", 64)
    try:
        shm.set_shared_memory_region(h, [a])
        c.register_system_shared_memory("http_in0", "/http_in0_native", 64)
        c.register_system_shared_memory("http_out0", "/http_out0_native", 64)
        i0 = httpclient.InferInput("INPUT0", [1, 16], "INT32")
        i0.set_shared_memory("http_in0", 64)
        o0 = httpclient.InferRequestedOutput("OUTPUT0")
        o0.set_shared_memory("http_out0", 64)
        r = c.infer("add_sub_batched", [i0, i1], outputs=[o0])
        assert r.get_output("OUTPUT0")["parameters"]["shared_memory_region"] == "http_out0"
        np.testing.assert_array_equal(shm.get_contents_as_numpy(ho, np.int32, [1, 16]), 2 * a)
    finally:
        c.unregister_system_shared_memory()
        shm.destroy_shared_memory_region(h)
        shm.destroy_shared_memory_region(ho)


def test_http_pipelined_requests_keep_order_and_connection_close(cpu_server):
    """Raw HTTP/1.1: two pipelined requests (native + relayed) answered in
    order on one connection, then Connection: close honoured."""
    host, port = cpu_server.http_url.split(":")
    a = np.arange(16, dtype=np.int32)
    hdr = json.dumps({"inputs": [{"name": n, "shape": [1, 16], "datatype": "INT32",
                                  "parameters": {"binary_data_size": 64}} for n in ("INPUT0", "INPUT1")],
                      "parameters": {"binary_data_output": True}}).encode()
    body = hdr + a.tobytes() + a.tobytes()
    infer = (b"POST /v2/models/add_sub_batched/infer HTTP/1.1\r\nHost: x\r\nInference-Header-Content-Length: %d\r\n"
             b"Content-Length: %d\r\n\r\n" % (len(hdr), len(body))) + body
    live = b"GET /v2/health/live HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n"
    s = socket.create_connection((host, int(port)))
    s.sendall(infer + live)
    data = b""
    while True:
        chunk = s.recv(65536)
        if not chunk:
            break
        data += chunk
    s.close()
    first, rest = data.split(b"\r\n\r\n", 1)
    assert first.startswith(b"HTTP/1.1 200") and b"inference-header-content-length" in first.lower()
    clen = int([ln.split(b":")[1] for ln in first.split(b"\r\n") if ln.lower().startswith(b"content-length")][0])
    second = rest[clen:]
    assert second.startswith(b"HTTP/1.1 200")  # the relayed /live answer, after the infer


def test_http_chunked_upload_is_decoded_and_relayed(cpu_server):
    host, port = cpu_server.http_url.split(":")
    body = json.dumps({"log_verbose_level": 0}).encode()
    req = (b"POST /v2/logging HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\n" +
           b"%x\r\n%s\r\n0\r\n\r\n" % (len(body), body))
    s = socket.create_connection((host, int(port)))
    s.sendall(req)
    data = b""
    while True:
        chunk = s.recv(65536)
        if not chunk:
            break
        data += chunk
    s.close()
    assert data.startswith(b"HTTP/1.1 200"), data[:200]


def test_shm_negative_size_and_huge_offset_rejected(cpu_server):
    """A negative shared_memory_byte_size must not slip past the bounds check
    (offset + size overflow) on either the gRPC or the HTTP fast path."""
    g = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    h = httpclient.InferenceServerClient(cpu_server.http_url)
    region = shm.create_shared_memory_region("neg_in", "/neg_in_native", 128)
    try:
        g.register_system_shared_memory("neg_in", "/neg_in_native", 128)
        a = np.zeros((1, 16), np.int32)
        for off, size in ((128, -1), (2 ** 62, -(2 ** 62)), (-64, 128), (64, 2 ** 63 - 1)):
            for mod, cli in ((grpcclient, g), (httpclient, h)):
                i0 = mod.InferInput("INPUT0", [1, 16], "INT32")
                i0.set_shared_memory("neg_in", size, offset=off)
                i1 = mod.InferInput("INPUT1", [1, 16], "INT32")
                i1.set_data_from_numpy(a)
                with pytest.raises(InferenceServerException, match="(?i)invalid offset|smaller|byte size"):
                    cli.infer("add_sub_batched", [i0, i1])
                o = mod.InferRequestedOutput("OUTPUT0")
                o.set_shared_memory("neg_in", size, offset=off)
                ok = _inputs(a, a) if mod is grpcclient else _http_inputs(a, a)
                with pytest.raises(InferenceServerException, match="(?i)invalid offset|should be at least|byte size"):
                    cli.infer("add_sub_batched", ok, outputs=[o])
        assert g.is_server_live()
    finally:
        g.unregister_system_shared_memory()
        shm.destroy_shared_memory_region(region)


def test_duplicate_input_rejected_on_fast_path(cpu_server):
    g = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    h = httpclient.InferenceServerClient(cpu_server.http_url)
    a = np.ones((1, 16), np.int32)
    dup = _inputs(a, a)
    dup[1] = grpcclient.InferInput("INPUT0", [1, 16], "INT32")
    dup[1].set_data_from_numpy(a)
    with pytest.raises(InferenceServerException, match="more than once"):
        g.infer("add_sub_batched", dup)
    hd = _http_inputs(a, a)
    hd[1] = httpclient.InferInput("INPUT0", [1, 16], "INT32")
    hd[1].set_data_from_numpy(a)
    with pytest.raises(InferenceServerException, match="more than once"):
        h.infer("add_sub_batched", hd)
    assert g.is_server_live()


def test_unregister_defers_unmap_until_inflight_request_done(cpu_server):
    """Unregistering a region while a native request that writes into it is
    executing must neither block the caller (the wait used to run on the
    server's event loop under the registry lock) nor unmap the region under
    the request: the unregister returns at once, the unmap is deferred until
    the request drops its pin, and the output lands."""
    import threading
    import time

    from triton_client_amd.server.cpu_models import AddSubBatched

    g = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    closer = cpu_server.server.shm_closer
    out = shm.create_shared_memory_region("inflight_out", "/inflight_out", 64)
    AddSubBatched.native_delay_s = 0.6
    try:
        g.register_system_shared_memory("inflight_out", "/inflight_out", 64)
        a = np.arange(16, dtype=np.int32).reshape(1, 16)
        o = grpcclient.InferRequestedOutput("OUTPUT0")
        o.set_shared_memory("inflight_out", 64)
        done = threading.Event()
        res = []

        def cb(result, error):
            res.append((result, error))
            done.set()

        g.async_infer("add_sub_batched", _inputs(a, a), cb, outputs=[o])
        time.sleep(0.2)  # the batch is executing (holding the region)
        t0 = time.monotonic()
        g.unregister_system_shared_memory("inflight_out")
        waited = time.monotonic() - t0
        assert waited < 0.3, "unregister blocked on the in-flight request (%.3f s)" % waited
        assert closer.pending() == 1, "the region was unmapped under the executing request"
        assert len(g.get_system_shared_memory_status().regions) == 0
        assert done.wait(10)
        assert res[0][1] is None, res[0][1]
        np.testing.assert_array_equal(shm.get_contents_as_numpy(out, np.int32, [1, 16]), 2 * a)
        deadline = time.monotonic() + 5
        while closer.pending() and time.monotonic() < deadline:
            time.sleep(0.01)
        assert closer.pending() == 0, "the deferred unmap never ran"
    finally:
        AddSubBatched.native_delay_s = 0.0
        g.unregister_system_shared_memory()
        shm.destroy_shared_memory_region(out)


def test_oversized_content_length_gets_413(cpu_server):
    host, port = cpu_server.http_url.split(":")
    for hdr in (b"Content-Length: 99999999999\r\n", b"Transfer-Encoding: chunked\r\n"):
        req = b"POST /v2/models/add_sub_batched/infer HTTP/1.1\r\nHost: x\r\n" + hdr + b"\r\n"
        if b"chunked" in hdr:
            req += b"ffffffffffffffff\r\nabc"
        s = socket.create_connection((host, int(port)))
        s.sendall(req)
        s.settimeout(10)
        data = b""
        while True:
            chunk = s.recv(65536)
            if not chunk:
                break
            data += chunk
        s.close()
        assert data.startswith(b"HTTP/1.1 413"), data[:200]


def _read_http_responses(s, n):
    """n HTTP/1.1 responses (Content-Length framed) from socket s, in arrival order."""
    data, out = b"", []
    while len(out) < n:
        while b"\r\n\r\n" not in data:
            chunk = s.recv(65536)
            assert chunk, "connection closed after %d responses" % len(out)
            data += chunk
        head, rest = data.split(b"\r\n\r\n", 1)
        hdrs = {ln.split(b":", 1)[0].strip().lower(): ln.split(b":", 1)[1].strip()
                for ln in head.split(b"\r\n")[1:] if b":" in ln}
        clen = int(hdrs.get(b"content-length", b"0"))
        while len(rest) < clen:
            chunk = s.recv(65536)
            assert chunk
            rest += chunk
        out.append((head.split(b"\r\n")[0], hdrs, rest[:clen]))
        data = rest[clen:]
    return out


@pytest.mark.parametrize("native", [True, False])
def test_http_large_gzip_infer_on_codec_pool_keeps_pipeline_order(cpu_server, native):
    """A compressed KServe REST infer body >= 64 KiB is inflated on tcserve's
    codec pool (not the loop thread), then served natively (binary tensor) or
    relayed to the Python server as the original compressed request (JSON
    tensor: the relay-fallback path).  A small identity-encoded infer and a
    /live GET pipelined behind it on the same keep-alive connection must come
    back after it, in order, and the inflated / native / proxied counters move
    accordingly."""
    import gzip

    nf = cpu_server.server.native_frontend
    host, port = cpu_server.http_url.split(":")
    rng = np.random.default_rng(7)
    x = rng.standard_normal((1, 3, 224, 224)).astype(np.float32)
    if native:
        hdr = json.dumps({"inputs": [{"name": "data_0", "shape": [1, 3, 224, 224], "datatype": "FP32",
                                      "parameters": {"binary_data_size": x.nbytes}}],
                          "parameters": {"binary_data_output": True}}).encode()
        plain = hdr + x.tobytes()
    else:
        hdr = json.dumps({"inputs": [{"name": "data_0", "shape": [1, 3, 224, 224], "datatype": "FP32",
                                      "data": [round(float(v), 3) for v in x.ravel()]}],
                          "outputs": [{"name": "fc6_1", "parameters": {"binary_data": False}}]}).encode()
        plain = hdr
    z = gzip.compress(plain)
    assert len(z) >= 64 * 1024
    big = (b"POST /v2/models/frontend_sink/infer HTTP/1.1\r\nHost: x\r\nContent-Encoding: gzip\r\n"
           b"Inference-Header-Content-Length: %d\r\nContent-Length: %d\r\n\r\n" % (len(hdr), len(z))) + z
    a = np.arange(16, dtype=np.int32)
    shdr = json.dumps({"inputs": [{"name": n, "shape": [1, 16], "datatype": "INT32",
                                   "parameters": {"binary_data_size": 64}} for n in ("INPUT0", "INPUT1")],
                       "parameters": {"binary_data_output": True}}).encode()
    sbody = shdr + a.tobytes() + (3 * a).tobytes()
    small = (b"POST /v2/models/add_sub_batched/infer HTTP/1.1\r\nHost: x\r\nInference-Header-Content-Length: %d\r\n"
             b"Content-Length: %d\r\n\r\n" % (len(shdr), len(sbody))) + sbody
    live = b"GET /v2/health/live HTTP/1.1\r\nHost: x\r\n\r\n"
    before = nf.counters()
    s = socket.create_connection((host, int(port)))
    try:
        s.sendall(big + small + live)
        (st1, h1, b1), (st2, h2, b2), (st3, _, _) = _read_http_responses(s, 3)
        # the connection stays open for another request (keep-alive)
        s.sendall(live)
        (st4, _, _), = _read_http_responses(s, 1)
    finally:
        s.close()
    assert st1.startswith(b"HTTP/1.1 200") and st2.startswith(b"HTTP/1.1 200"), (st1, b1[:200], st2)
    assert st3.startswith(b"HTTP/1.1 200") and st4.startswith(b"HTTP/1.1 200")
    # response 1: frontend_sink broadcasts the first input value
    if native:
        jl = int(h1[b"inference-header-content-length"])
        out = np.frombuffer(b1[jl:], dtype=np.float32)
        np.testing.assert_array_equal(out, np.full(1000, x.ravel()[0], np.float32))
    else:
        out = json.loads(b1)["outputs"][0]["data"]
        np.testing.assert_allclose(out, np.full(1000, round(float(x.ravel()[0]), 3)), rtol=1e-6)
    # response 2: the pipelined add_sub infer, after the big one
    jl2 = int(h2[b"inference-header-content-length"])
    meta = json.loads(b2[:jl2])
    assert meta["model_name"] == "add_sub_batched"
    np.testing.assert_array_equal(np.frombuffer(b2[jl2:jl2 + 64], dtype=np.int32), 4 * a)
    after = nf.counters()
    assert after["inflated_requests"] == before["inflated_requests"] + 1
    assert after["native_requests"] == before["native_requests"] + (2 if native else 1)
    assert after["proxied_calls"] >= before["proxied_calls"] + (2 if native else 3)
