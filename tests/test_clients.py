"""HTTP + gRPC clients against the in-process KServe-v2 server (CPU models).

Covers the reference's control plane and data plane per protocol:
SURVEY.md §2.7 / Appendix B, plus the cc_client_test scenarios
(InferMulti-style version fan-out, load with config/file override, trace
settings update/clear; reference src/c++/tests/cc_client_test.cc)."""

import base64
import queue
import threading
import time

import numpy as np
import pytest

import tritonclient.grpc as grpcclient
import tritonclient.http as httpclient
from tritonclient.utils import InferenceServerException
from tritonclient.utils import shared_memory as shm

A = np.arange(16, dtype=np.int32).reshape(1, 16)
B = np.full((1, 16), 3, dtype=np.int32)


@pytest.fixture(params=["http", "grpc"])
def proto(request, cpu_server):
    if request.param == "http":
        c = httpclient.InferenceServerClient(cpu_server.http_url, concurrency=4)
        yield "http", httpclient, c
    else:
        c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
        yield "grpc", grpcclient, c
    c.close()


def _inputs(mod, binary=True):
    i0 = mod.InferInput("INPUT0", [1, 16], "INT32")
    i1 = mod.InferInput("INPUT1", [1, 16], "INT32")
    if mod is httpclient:
        i0.set_data_from_numpy(A, binary_data=binary)
        i1.set_data_from_numpy(B, binary_data=binary)
    else:
        i0.set_data_from_numpy(A)
        i1.set_data_from_numpy(B)
    return [i0, i1]


def test_health_and_metadata(proto):
    kind, mod, c = proto
    assert c.is_server_live() and c.is_server_ready()
    assert c.is_model_ready("simple") and not c.is_model_ready("nope")
    md = c.get_server_metadata() if kind == "http" else c.get_server_metadata(as_json=True)
    assert md["name"] == "triton-mi355x" and "binary_tensor_data" in md["extensions"]
    mm = c.get_model_metadata("simple") if kind == "http" else c.get_model_metadata("simple", as_json=True)
    assert [t["name"] for t in mm["inputs"]] == ["INPUT0", "INPUT1"]
    cfg = c.get_model_config("simple") if kind == "http" else c.get_model_config("simple", as_json=True)["config"]
    assert int(cfg["max_batch_size"]) == 8
    with pytest.raises(InferenceServerException):
        c.get_model_metadata("nope")
    with pytest.raises(InferenceServerException):
        c.is_model_ready("simple", model_version=1)  # version must be a string


@pytest.mark.parametrize("binary", [True, False])
def test_infer_add_sub(proto, binary):
    kind, mod, c = proto
    if kind == "http":
        outs = [mod.InferRequestedOutput("OUTPUT0", binary_data=binary), mod.InferRequestedOutput("OUTPUT1", binary_data=not binary)]
    else:
        outs = [mod.InferRequestedOutput("OUTPUT0"), mod.InferRequestedOutput("OUTPUT1")]
    r = c.infer("simple", _inputs(mod, binary), outputs=outs, request_id="r1")
    np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), A + B)
    np.testing.assert_array_equal(r.as_numpy("OUTPUT1"), A - B)
    resp = r.get_response() if kind == "http" else r.get_response(as_json=True)
    assert resp["id"] == "r1" and resp["model_name"] == "simple"
    # no outputs requested -> all outputs, binary
    r = c.infer("simple", _inputs(mod, binary))
    np.testing.assert_array_equal(r.as_numpy("OUTPUT1"), A - B)


def test_infer_errors(proto):
    kind, mod, c = proto
    with pytest.raises(InferenceServerException) as e:
        c.infer("nope", _inputs(mod))
    assert "unknown model" in str(e.value).lower() or "not found" in str(e.value).lower()
    bad = mod.InferInput("INPUT0", [1, 16], "INT32").set_data_from_numpy(A)
    with pytest.raises(InferenceServerException):
        c.infer("simple", [bad])  # missing INPUT1
    with pytest.raises(InferenceServerException):
        mod.InferInput("INPUT0", [1, 16], "FP32").set_data_from_numpy(A)


def test_versions_and_swapped_outputs(proto):
    """cc_client_test InferMulti across versions 1..3 of onnx_int32_int32_int32."""
    kind, mod, c = proto
    for v in ("1", "2", "3"):
        r = c.infer("onnx_int32_int32_int32", _inputs(mod), model_version=v)
        s, d = r.as_numpy("OUTPUT0"), r.as_numpy("OUTPUT1")
        if v == "1":
            np.testing.assert_array_equal(s, A + B)
        else:
            np.testing.assert_array_equal(s, A - B)
            np.testing.assert_array_equal(d, A + B)


def test_strings_and_identity(proto):
    kind, mod, c = proto
    in0 = np.array([str(x).encode() for x in range(16)], dtype=np.object_).reshape(1, 16)
    in1 = np.array([b"1"] * 16, dtype=np.object_).reshape(1, 16)
    i0 = mod.InferInput("INPUT0", [1, 16], "BYTES").set_data_from_numpy(in0)
    i1 = mod.InferInput("INPUT1", [1, 16], "BYTES").set_data_from_numpy(in1)
    r = c.infer("simple_string", [i0, i1])
    assert [int(x) for x in r.as_numpy("OUTPUT0").reshape(-1)] == [x + 1 for x in range(16)]
    data = np.array([[b"\x00\xffbin", b"x"]], dtype=np.object_)
    i = mod.InferInput("INPUT0", [1, 2], "BYTES").set_data_from_numpy(data)
    r = c.infer("simple_identity", [i])
    assert list(r.as_numpy("OUTPUT0").reshape(-1)) == [b"\x00\xffbin", b"x"]


def test_bf16_identity(proto):
    kind, mod, c = proto
    x = np.array([1.0, -2.0, 3.5], dtype=np.float32)
    i = mod.InferInput("INPUT0", [3], "BF16").set_data_from_numpy(x)
    r = c.infer("identity_bf16", [i])
    np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), x)


def test_async_infer(proto):
    kind, mod, c = proto
    if kind == "http":
        reqs = [c.async_infer("simple", _inputs(mod), request_id=str(i)) for i in range(8)]
        for req in reqs:
            np.testing.assert_array_equal(req.get_result().as_numpy("OUTPUT0"), A + B)
    else:
        q = queue.Queue()
        for i in range(8):
            c.async_infer("simple", _inputs(mod), lambda result, error: q.put((result, error)))
        for _ in range(8):
            res, err = q.get(timeout=10)
            assert err is None
            np.testing.assert_array_equal(res.as_numpy("OUTPUT0"), A + B)


def test_statistics(proto):
    kind, mod, c = proto
    c.infer("simple", _inputs(mod))
    st = c.get_inference_statistics("simple") if kind == "http" else c.get_inference_statistics("simple", as_json=True)
    ms = st["model_stats"][0]
    assert ms["name"] == "simple" and int(ms["inference_count"]) >= 1
    assert int(ms["inference_stats"]["success"]["count"]) >= 1
    allst = c.get_inference_statistics() if kind == "http" else c.get_inference_statistics(as_json=True)
    assert len(allst["model_stats"]) > 1


def test_trace_settings_update_and_clear(proto):
    kind, mod, c = proto
    kw = {} if kind == "http" else {"as_json": True}
    glob = c.get_trace_settings(**kw)
    r = c.update_trace_settings(model_name="simple", settings={"trace_rate": "5", "trace_level": ["TIMESTAMPS"]}, **kw)
    s = r if kind == "http" else {k: v["value"] for k, v in r["settings"].items()}
    assert s["trace_level"] == ["TIMESTAMPS"]
    assert s["trace_rate"] in ("5", ["5"])
    r = c.update_trace_settings(model_name="simple", settings={"trace_rate": None}, **kw)
    s = r if kind == "http" else {k: v["value"] for k, v in r["settings"].items()}
    g = glob if kind == "http" else {k: v["value"] for k, v in glob["settings"].items()}
    assert s["trace_rate"] == g["trace_rate"]


def test_log_settings(proto):
    kind, mod, c = proto
    if kind == "http":
        r = c.update_log_settings({"log_verbose_level": 2, "log_info": False})
        assert r["log_verbose_level"] == 2 and r["log_info"] is False
        assert c.get_log_settings()["log_verbose_level"] == 2
    else:
        r = c.update_log_settings({"log_verbose_level": 3, "log_format": "ISO8601"}, as_json=True)
        assert r["settings"]["log_verbose_level"]["uint32_param"] == 3
        assert c.get_log_settings(as_json=True)["settings"]["log_format"]["string_param"] == "ISO8601"
    with pytest.raises(InferenceServerException):
        c.update_log_settings({"no_such": True})


def test_system_shared_memory(proto):
    kind, mod, c = proto
    key_in, key_out = "/tcamd_t_in_%s" % kind, "/tcamd_t_out_%s" % kind
    hin = shm.create_shared_memory_region("in", key_in, 128)
    hout = shm.create_shared_memory_region("out", key_out, 128)
    try:
        shm.set_shared_memory_region(hin, [A, B])
        c.register_system_shared_memory("in_" + kind, key_in, 128)
        c.register_system_shared_memory("out_" + kind, key_out, 128)
        st = c.get_system_shared_memory_status() if kind == "http" else c.get_system_shared_memory_status(as_json=True)["regions"]
        names = [x["name"] for x in st] if kind == "http" else list(st)
        assert "in_" + kind in names
        ins = [mod.InferInput("INPUT0", [1, 16], "INT32"), mod.InferInput("INPUT1", [1, 16], "INT32")]
        ins[0].set_shared_memory("in_" + kind, 64)
        ins[1].set_shared_memory("in_" + kind, 64, offset=64)
        o0 = mod.InferRequestedOutput("OUTPUT0")
        o0.set_shared_memory("out_" + kind, 64)
        o1 = mod.InferRequestedOutput("OUTPUT1")
        o1.set_shared_memory("out_" + kind, 64, offset=64)
        r = c.infer("simple", ins, outputs=[o0, o1])
        assert r.as_numpy("OUTPUT0") is None or r.as_numpy("OUTPUT0").size == 0
        np.testing.assert_array_equal(shm.get_contents_as_numpy(hout, np.int32, [1, 16]), A + B)
        np.testing.assert_array_equal(shm.get_contents_as_numpy(hout, np.int32, [1, 16], offset=64), A - B)
        # too-small output region is an error
        o_small = mod.InferRequestedOutput("OUTPUT0")
        o_small.set_shared_memory("out_" + kind, 8)
        with pytest.raises(InferenceServerException):
            c.infer("simple", ins, outputs=[o_small])
        with pytest.raises(InferenceServerException):
            c.register_system_shared_memory("in_" + kind, key_in, 128)  # duplicate
    finally:
        c.unregister_system_shared_memory("in_" + kind)
        c.unregister_system_shared_memory("out_" + kind)
        shm.destroy_shared_memory_region(hin)
        shm.destroy_shared_memory_region(hout)
    assert key_in not in shm.mapped_shared_memory_regions()


def test_load_unload_and_overrides(proto):
    """cc_client_test LoadWithFileOverride / LoadWithConfigOverride semantics."""
    kind, mod, c = proto
    name = "onnx_int32_int32_int32"
    for v in ("1", "2", "3"):
        assert c.is_model_ready(name, v)
    with pytest.raises(InferenceServerException):
        c.load_model(name, config='{"backend":"onnxruntime", bad json')
    assert c.is_model_ready(name, "3")
    c.load_model(name, config='{"backend":"onnxruntime","version_policy":{"specific":{"versions":[2]}}}')
    assert c.is_model_ready(name, "2") and not c.is_model_ready(name, "3")
    content = b"tcamd-model:onnx_int32_int32_int32"
    with pytest.raises(InferenceServerException):
        c.load_model(name, files={"file:1/model.onnx": content})  # files need a config
    override = "override_model_" + kind
    c.load_model(override, config='{"backend":"onnxruntime"}', files={"file:1/model.onnx": content})
    assert c.is_model_ready(override, "1") and not c.is_model_ready(override, "3")
    r = c.infer(override, _inputs(mod))
    np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), A + B)
    idx = c.get_model_repository_index() if kind == "http" else c.get_model_repository_index(as_json=True)["models"]
    assert any(m["name"] == override for m in idx)
    c.unload_model(override)
    assert not c.is_model_ready(override)
    c.load_model(name, config='{"backend":"onnxruntime","version_policy":{"all":{}}}')
    for v in ("1", "2", "3"):
        assert c.is_model_ready(name, v)
    c.unload_model("simple_identity")
    assert not c.is_model_ready("simple_identity")
    c.load_model("simple_identity")
    assert c.is_model_ready("simple_identity")


def test_config_override_retunes_preferred_batch_size(cpu_server):
    """A repository load with a dynamic_batching override on a loaded model
    (how bench.py's bs=1 point sets its preferred size): no reload, the
    reported config carries the new preferred sizes, requests keep working."""
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    name = "add_sub_pipelined"
    cfg = lambda: c.get_model_config(name, as_json=True)["config"]["dynamic_batching"]  # noqa: E731
    assert [int(x) for x in cfg().get("preferred_batch_size", [])] == [8]
    try:
        c.load_model(name, config='{"dynamic_batching":{"preferred_batch_size":[4]}}')
        assert c.is_model_ready(name)
        assert [int(x) for x in cfg()["preferred_batch_size"]] == [4]
        x = np.arange(16, dtype=np.int32).reshape(1, 16)
        ins = [grpcclient.InferInput("INPUT0", [1, 16], "INT32").set_data_from_numpy(x),
               grpcclient.InferInput("INPUT1", [1, 16], "INT32").set_data_from_numpy(x)]
        r = c.infer(name, ins)
        np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), 2 * x)
    finally:
        c.load_model(name, config='{"dynamic_batching":{"preferred_batch_size":[8]}}')
    assert [int(x) for x in cfg()["preferred_batch_size"]] == [8]


def test_grpc_stream_sequence_and_decoupled(cpu_server):
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    q = queue.Queue()
    c.start_stream(lambda result, error: q.put((result, error)))
    values = [11, 7, 5, 3, 2, 0, 1]
    seqs = {1000: [0] + values, 1001: [100] + [-v for v in values]}
    for step in range(len(values) + 1):
        for sid, vals in seqs.items():
            x = grpcclient.InferInput("INPUT", [1, 1], "INT32").set_data_from_numpy(np.array([[vals[step]]], np.int32))
            c.async_stream_infer("simple_sequence", [x], request_id="%d_%d" % (sid, step), sequence_id=sid,
                                 sequence_start=step == 0, sequence_end=step == len(values))
    got = {1000: [], 1001: []}
    for _ in range(2 * (len(values) + 1)):
        r, e = q.get(timeout=10)
        assert e is None
        sid = int(r.get_response().id.split("_")[0])
        got[sid].append(int(r.as_numpy("OUTPUT")[0][0]))
    assert got[1000] == [1] + values
    assert got[1001] == [101] + [-v for v in values]
    # decoupled: 5 responses + empty final
    ins = [grpcclient.InferInput("IN", [5], "INT32"), grpcclient.InferInput("DELAY", [5], "UINT32"),
           grpcclient.InferInput("WAIT", [1], "UINT32")]
    ins[0].set_data_from_numpy(np.arange(10, 15, dtype=np.int32))
    ins[1].set_data_from_numpy(np.full(5, 2, np.uint32))
    ins[2].set_data_from_numpy(np.zeros(1, np.uint32))
    c.async_stream_infer("repeat_int32", ins, enable_empty_final_response=True)
    outs = []
    while True:
        r, e = q.get(timeout=10)
        assert e is None
        resp = r.get_response()
        if resp.parameters["triton_final_response"].bool_param:
            assert len(resp.outputs) == 0
            break
        outs.append(int(r.as_numpy("OUT")[0]))
    assert outs == list(range(10, 15))
    # errors come back through the callback, stream stays usable
    bad = grpcclient.InferInput("INPUT", [1, 1], "INT32").set_data_from_numpy(np.zeros((1, 1), np.int32))
    c.async_stream_infer("nope", [bad])
    r, e = q.get(timeout=10)
    assert r is None and e is not None
    c.stop_stream()
    with pytest.raises(InferenceServerException):
        c.async_stream_infer("simple", [])
    c.close()


def _repeat_inputs(vals, delay_ms):
    ins = [grpcclient.InferInput("IN", [len(vals)], "INT32"), grpcclient.InferInput("DELAY", [len(vals)], "UINT32"),
           grpcclient.InferInput("WAIT", [1], "UINT32")]
    ins[0].set_data_from_numpy(np.asarray(vals, np.int32))
    ins[1].set_data_from_numpy(np.full(len(vals), delay_ms, np.uint32))
    ins[2].set_data_from_numpy(np.zeros(1, np.uint32))
    return ins


def test_grpc_stream_drain_cancel_and_restart(cpu_server):
    from tritonclient.grpc._infer_stream import StreamState

    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    # stop_stream() without cancel half-closes and waits for every response
    got = []
    c.start_stream(lambda result, error: got.append((result, error)))
    c.async_stream_infer("repeat_int32", _repeat_inputs(list(range(6)), 20))
    s = c._stream
    c.stop_stream()
    assert s.state is StreamState.CLOSED
    assert [int(r.as_numpy("OUT")[0]) for r, e in got if e is None] == list(range(6))
    # cancel while responses are still pending: the rpc ends CANCELLED, the
    # callback sees the cancellation once, and stop returns promptly
    got2 = []
    c.start_stream(lambda result, error: got2.append((result, error)))
    c.async_stream_infer("repeat_int32", _repeat_inputs(list(range(50)), 50))
    time.sleep(0.2)
    s2 = c._stream
    t0 = time.time()
    c.stop_stream(cancel_requests=True)
    assert time.time() - t0 < 2.0
    assert s2.state is StreamState.CANCELLED
    errs = [e for r, e in got2 if e is not None]
    assert len(errs) == 1 and "cancel" in str(errs[0]).lower()
    assert len([r for r, e in got2 if e is None]) < 50
    with pytest.raises(InferenceServerException):
        s2.submit(None)
    # a fresh stream works after a cancelled one; closing from inside the
    # callback does not deadlock
    done = threading.Event()

    def cb(result, error):
        if result is not None and int(result.as_numpy("OUT")[0]) == 2:
            c._stream.close()
            done.set()

    c.start_stream(cb)
    c.async_stream_infer("repeat_int32", _repeat_inputs([0, 1, 2], 1))
    assert done.wait(10)
    c.stop_stream()
    c.close()


def test_decoupled_over_http_rejected(cpu_server):
    c = httpclient.InferenceServerClient(cpu_server.http_url)
    ins = [httpclient.InferInput("IN", [1], "INT32").set_data_from_numpy(np.zeros(1, np.int32)),
           httpclient.InferInput("DELAY", [1], "UINT32").set_data_from_numpy(np.zeros(1, np.uint32)),
           httpclient.InferInput("WAIT", [1], "UINT32").set_data_from_numpy(np.zeros(1, np.uint32))]
    with pytest.raises(InferenceServerException):
        c.infer("repeat_int32", ins)
    c.close()


def test_client_timeouts(cpu_server):
    """client_timeout_test: a slow model + tiny deadline -> Deadline Exceeded."""
    g = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    x = grpcclient.InferInput("INPUT0", [1, 4], "INT32").set_data_from_numpy(np.zeros((1, 4), np.int32))
    with pytest.raises(InferenceServerException) as e:
        g.infer("custom_identity_int32", [x], client_timeout=0.05)
    assert "DEADLINE_EXCEEDED" in str(e.value)
    q = queue.Queue()
    g.async_infer("custom_identity_int32", [x], lambda result, error: q.put(error), client_timeout=0.05)
    err = q.get(timeout=10)
    assert err is not None and "DEADLINE" in str(err)
    assert g.is_server_live(client_timeout=5)
    g.close()
    h = httpclient.InferenceServerClient(cpu_server.http_url, network_timeout=0.1)
    hx = httpclient.InferInput("INPUT0", [1, 4], "INT32").set_data_from_numpy(np.zeros((1, 4), np.int32))
    with pytest.raises(InferenceServerException):
        h.infer("custom_identity_int32", [hx])
    h.close()


def test_cancel_async(cpu_server):
    g = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    x = grpcclient.InferInput("INPUT0", [1, 4], "INT32").set_data_from_numpy(np.zeros((1, 4), np.int32))
    q = queue.Queue()
    ctx = g.async_infer("custom_identity_int32", [x], lambda result, error: q.put(error))
    ctx.cancel()
    err = q.get(timeout=10)
    assert err is not None and "CANCELLED" in str(err)
    g.close()


def test_compression(cpu_server):
    h = httpclient.InferenceServerClient(cpu_server.http_url)
    for alg in ("gzip", "deflate"):
        r = h.infer("simple", _inputs(httpclient), request_compression_algorithm=alg, response_compression_algorithm=alg)
        np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), A + B)
    h.close()
    g = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    for alg in ("gzip", "deflate", None):
        r = g.infer("simple", _inputs(grpcclient), compression_algorithm=alg)
        np.testing.assert_array_equal(r.as_numpy("OUTPUT1"), A - B)
    g.close()


def test_classification(proto):
    kind, mod, c = proto
    if kind == "http":
        out = mod.InferRequestedOutput("OUTPUT0", class_count=3)
    else:
        out = mod.InferRequestedOutput("OUTPUT0", class_count=3)
    r = c.infer("simple", _inputs(mod), outputs=[out])
    top = r.as_numpy("OUTPUT0")
    assert top.shape == (1, 3)
    assert top[0, 0].decode().split(":")[1] == "15"


def test_plugin_basic_auth(cpu_server):
    from tritonclient.http.auth import BasicAuth

    c = httpclient.InferenceServerClient(cpu_server.http_url)
    p = BasicAuth("user", "pass")
    c.register_plugin(p)
    assert c.plugin() is p
    with pytest.raises(InferenceServerException):
        c.register_plugin(p)
    assert c.is_server_live()
    req = httpclient.Request({})
    p(req)
    assert req.headers["authorization"] == "Basic " + base64.b64encode(b"user:pass").decode()
    c.unregister_plugin()
    with pytest.raises(InferenceServerException):
        c.unregister_plugin()
    c.close()


def test_grpc_keepalive_and_channel_args(cpu_server):
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url, keepalive_options=grpcclient.KeepAliveOptions(
        keepalive_time_ms=10000, keepalive_timeout_ms=2000, keepalive_permit_without_calls=True))
    assert c.is_server_live()
    c.close()
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url, channel_args=[("grpc.max_receive_message_length", 1 << 20)])
    assert c.is_server_ready()
    c.close()


def test_http_url_validation():
    with pytest.raises(InferenceServerException):
        httpclient.InferenceServerClient("http://localhost:8000")
    with pytest.raises(InferenceServerException):
        httpclient.InferenceServerClient("localhost:8000").infer("m", [], headers={"Transfer-Encoding": "chunked"})


def test_many_concurrent_http(cpu_server):
    c = httpclient.InferenceServerClient(cpu_server.http_url, concurrency=8)
    t0 = time.time()
    reqs = [c.async_infer("simple", _inputs(httpclient)) for _ in range(200)]
    for r in reqs:
        np.testing.assert_array_equal(r.get_result().as_numpy("OUTPUT0"), A + B)
    assert time.time() - t0 < 30
    c.close()
