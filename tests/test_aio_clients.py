"""asyncio clients (tritonclient.http.aio / tritonclient.grpc.aio) against the
CPU test server — the reference's simple_{http,grpc}_aio_* example flows."""

import asyncio

import numpy as np
import pytest

import tritonclient.grpc.aio as grpcaio
import tritonclient.http.aio as httpaio
from tritonclient.grpc.aio.auth import BasicAuth as GrpcBasicAuth
from tritonclient.http.aio.auth import BasicAuth as HttpBasicAuth
from tritonclient.utils import InferenceServerException
from tritonclient.utils import shared_memory as shm


def run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


def _simple_inputs(mod, a, b):
    i0 = mod.InferInput("INPUT0", list(a.shape), "INT32")
    i0.set_data_from_numpy(a)
    i1 = mod.InferInput("INPUT1", list(b.shape), "INT32")
    i1.set_data_from_numpy(b)
    return [i0, i1]


def test_http_aio_control_and_infer(cpu_server):
    async def body():
        async with httpaio.InferenceServerClient(cpu_server.http_url) as c:
            c.register_plugin(HttpBasicAuth("user", "pass"))
            assert await c.is_server_live()
            assert await c.is_server_ready()
            assert await c.is_model_ready("simple")
            md = await c.get_server_metadata()
            assert "name" in md
            mm = await c.get_model_metadata("simple")
            assert mm["name"] == "simple"
            cfg = await c.get_model_config("simple")
            assert cfg["name"] == "simple"
            idx = await c.get_model_repository_index()
            assert any(m["name"] == "simple" for m in idx)
            a = np.arange(16, dtype=np.int32).reshape(1, 16)
            b = np.ones((1, 16), dtype=np.int32)
            for comp in (None, "gzip", "deflate"):
                r = await c.infer("simple", _simple_inputs(httpaio, a, b),
                                  outputs=[httpaio.InferRequestedOutput("OUTPUT0"),
                                           httpaio.InferRequestedOutput("OUTPUT1", binary_data=False)],
                                  request_compression_algorithm=comp, response_compression_algorithm=comp)
                np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), a + b)
                np.testing.assert_array_equal(r.as_numpy("OUTPUT1"), a - b)
            st = await c.get_inference_statistics("simple")
            assert st["model_stats"][0]["name"] == "simple"
            ts = await c.update_trace_settings("simple", {"trace_rate": "5"})
            assert ts["trace_rate"] in ("5", ["5"])
            await c.get_trace_settings()
            ls = await c.update_log_settings({"log_verbose_level": 1})
            assert ls["log_verbose_level"] == 1
            await c.get_log_settings()
            with pytest.raises(InferenceServerException):
                await c.get_model_metadata("not_a_model")
            await c.unload_model("onnx_int32_int32_int32")
            assert not await c.is_model_ready("onnx_int32_int32_int32")
            await c.load_model("onnx_int32_int32_int32")
            assert await c.is_model_ready("onnx_int32_int32_int32")
            body_, json_size = httpaio.InferenceServerClient.generate_request_body(_simple_inputs(httpaio, a, b))
            assert json_size is not None and len(body_) > json_size

    run(body())


def test_http_aio_system_shm(cpu_server):
    async def body():
        c = httpaio.InferenceServerClient(cpu_server.http_url)
        try:
            a = np.arange(16, dtype=np.int32).reshape(1, 16)
            h = shm.create_shared_memory_region("aio_in", "/aio_in", 128)
            shm.set_shared_memory_region(h, [a, a])
            await c.register_system_shared_memory("aio_in", "/aio_in", 128)
            st = await c.get_system_shared_memory_status()
            assert any(r["name"] == "aio_in" for r in st)
            i0 = httpaio.InferInput("INPUT0", [1, 16], "INT32")
            i0.set_shared_memory("aio_in", 64)
            i1 = httpaio.InferInput("INPUT1", [1, 16], "INT32")
            i1.set_shared_memory("aio_in", 64, offset=64)
            r = await c.infer("simple", [i0, i1])
            np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), a * 2)
            await c.unregister_system_shared_memory("aio_in")
            shm.destroy_shared_memory_region(h)
            await c.get_cuda_shared_memory_status()
        finally:
            await c.close()

    run(body())


def test_grpc_aio_control_and_infer(cpu_server):
    async def body():
        async with grpcaio.InferenceServerClient(cpu_server.grpc_url) as c:
            c.register_plugin(GrpcBasicAuth("user", "pass"))
            assert await c.is_server_live()
            assert await c.is_server_ready()
            assert await c.is_model_ready("simple")
            md = await c.get_server_metadata(as_json=True)
            assert "name" in md
            mm = await c.get_model_metadata("simple")
            assert mm.name == "simple"
            cfg = await c.get_model_config("simple", as_json=True)
            assert cfg["config"]["name"] == "simple"
            await c.get_model_repository_index()
            a = np.arange(16, dtype=np.int32).reshape(1, 16)
            b = np.full((1, 16), 2, dtype=np.int32)
            for comp in (None, "gzip"):
                r = await c.infer("simple", _simple_inputs(grpcaio, a, b), compression_algorithm=comp)
                np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), a + b)
            st = await c.get_inference_statistics("simple", as_json=True)
            assert st["model_stats"][0]["name"] == "simple"
            await c.update_trace_settings(settings={"trace_rate": "7"})
            ts = await c.get_trace_settings(as_json=True)
            assert ts["settings"]["trace_rate"]["value"] == ["7"]
            await c.update_log_settings({"log_info": False})
            await c.get_log_settings()
            with pytest.raises(InferenceServerException):
                await c.infer("not_a_model", _simple_inputs(grpcaio, a, b))
            await c.get_system_shared_memory_status()
            await c.get_cuda_shared_memory_status()

    run(body())


def test_grpc_aio_stream_infer_sequence(cpu_server):
    async def body():
        async with grpcaio.InferenceServerClient(cpu_server.grpc_url) as c:
            values = [11, 7, 5, 3, 2, 0, 1]

            async def requests():
                for i, v in enumerate(values):
                    x = grpcaio.InferInput("INPUT", [1, 1], "INT32")
                    x.set_data_from_numpy(np.array([[v]], dtype=np.int32))
                    yield {"model_name": "simple_sequence", "inputs": [x], "request_id": str(i),
                           "sequence_id": 1001, "sequence_start": i == 0, "sequence_end": i == len(values) - 1}

            got = []
            async for result, error in c.stream_infer(requests()):
                assert error is None, error
                got.append(int(result.as_numpy("OUTPUT")[0][0]))
            assert len(got) == len(values)

    run(body())


def test_http_aio_stays_on_native_path_and_scales(cpu_server):
    """The asyncio REST client used to send aiohttp's default
    ``Accept-Encoding: gzip, deflate`` on every request: the server gzipped
    every response and tcserve relayed them all to the Python front end
    (~2.3 ms per request, 968 infer/s at 64 tasks).  Requests must stay on the
    native path uncompressed unless compression is asked for, compressed
    requests/responses must be served natively too, and 64 tasks in flight
    stay clear of the stall (absolute floors: relative rates are noise on a
    shared CPU)."""
    import time

    nf = cpu_server.server.native_frontend
    if nf is None:
        pytest.skip("native front end not built")
    a = np.arange(16, dtype=np.int32).reshape(1, 16)

    async def body():
        async with httpaio.InferenceServerClient(cpu_server.http_url) as c:
            x = _simple_inputs(httpaio, a, a)
            for _ in range(20):
                await c.infer("add_sub_batched", x)
            before = nf.counters()
            t0 = time.perf_counter()
            for _ in range(100):
                r = await c.infer("add_sub_batched", x)
            one = 100 / (time.perf_counter() - t0)
            np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), 2 * a)
            mid = nf.counters()
            t0 = time.perf_counter()
            for _ in range(5):
                rs = await asyncio.gather(*[c.infer("add_sub_batched", x) for _ in range(64)])
            many = 320 / (time.perf_counter() - t0)
            assert all(np.array_equal(q.as_numpy("OUTPUT1"), 0 * a) for q in rs)
            for comp in ("gzip", "deflate"):
                r = await c.infer("add_sub_batched", x, request_compression_algorithm=comp,
                                  response_compression_algorithm=comp)
                np.testing.assert_array_equal(r.as_numpy("OUTPUT0"), 2 * a)
            after = nf.counters()
            return one, many, before, mid, after

    one, many, before, mid, after = run(body())
    assert mid["native_requests"] - before["native_requests"] == 100
    assert mid["proxied_calls"] == before["proxied_calls"], "plain aio requests were relayed to Python"
    assert mid["compressed_responses"] == before["compressed_responses"], "responses compressed unasked"
    assert after["inflated_requests"] - mid["inflated_requests"] == 2
    assert after["compressed_responses"] - mid["compressed_responses"] == 2
    assert after["proxied_calls"] == before["proxied_calls"]
    assert one > 800, "one aio task: %.0f infer/s (the relayed/gzip path ran ~400)" % one
    assert many > 800, "64 aio tasks: %.0f infer/s (the relayed/gzip path ran ~970-1300)" % many


def test_http_aio_transport_retries_only_idempotent_requests():
    """A keep-alive connection the server drops before answering: GET is retried
    once on a fresh connection, POST is not (it may already have run on the
    server)."""
    from tritonclient.http.aio._transport import HttpTransportError, Pool

    async def body():
        seen = []

        async def handle(reader, writer):
            n = 0
            while True:
                head = await reader.readuntil(b"\r\n\r\n")
                line = head.split(b"\r\n", 1)[0].decode()
                clen = [int(h.split(b":")[1]) for h in head.split(b"\r\n") if h.lower().startswith(b"content-length")]
                if clen:
                    await reader.readexactly(clen[0])
                seen.append(line)
                n += 1
                if n == 2:  # the second request on a connection: drop it unanswered
                    writer.close()
                    return
                writer.write(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\nok")
                await writer.drain()

        srv = await asyncio.start_server(handle, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        pool = Pool("127.0.0.1", port, limit=1)
        try:
            # every second request on a connection is dropped and retried on a new one
            for _ in range(3):
                assert (await pool.request("GET", "/v2", {})).body == b"ok"
        finally:
            pool.close()
        assert sum(s.startswith("GET") for s in seen) == 5
        pool = Pool("127.0.0.1", port, limit=1)
        try:
            assert (await pool.request("POST", "/v2/models/m/infer", {}, b"{}")).status == 200
            with pytest.raises(HttpTransportError):
                await pool.request("POST", "/v2/models/m/infer", {}, b"{}")
        finally:
            pool.close()
            srv.close()
        posts = [s for s in seen if s.startswith("POST")]
        assert len(posts) == 2, seen  # the dropped POST was not re-sent

    run(body())
