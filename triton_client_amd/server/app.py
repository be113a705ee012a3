"""Server process wiring: asyncio loop running the HTTP + gRPC front ends."""

import asyncio
import os
import socket
import threading

import grpc
from aiohttp import web

from tritonclient.grpc import service_pb2_grpc

from .core import InferenceServer
from .grpc_frontend import FaultInjector, GrpcFrontend
from .http_frontend import HttpFrontend


def default_models(gpu=False, names=None):
    """The model classes a server loads: the CPU zoo, plus the GPU zoo with
    ``gpu``; ``names`` (an iterable of model names) selects a subset and may
    also name the opt-in GPU models (OPT_IN_GPU_MODELS), which no default
    list contains."""
    from .cpu_models import CPU_MODELS

    models = list(CPU_MODELS)
    if gpu:
        from .gpu_models import GPU_MODELS, OPT_IN_GPU_MODELS

        models += list(GPU_MODELS)
        if names is not None:
            models += [m for m in OPT_IN_GPU_MODELS if m.name in set(names)]
    if names is not None:
        keep = set(names)
        models = [m for m in models if m.name in keep]
    return models


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


GRPC_OPTIONS = [
    ("grpc.max_send_message_length", 2**31 - 1),
    ("grpc.max_receive_message_length", 2**31 - 1),
    ("grpc.so_reuseport", 0),
]


def native_grpc_available():
    from . import native_frontend

    return native_frontend.available()


async def serve(server, http_port, grpc_port, host="127.0.0.1", ready_evt=None, stop_evt=None, native_grpc=None,
                tls=None):
    """Serve HTTP (aiohttp) and gRPC.  With ``native_grpc`` (default: when
    libtcserve.so is built) the public gRPC port is tcserve, the C++ front
    end, and grpc.aio listens on a loopback port behind it.

    ``tls``: dict(cert=PEM path, key=PEM path[, client_ca=PEM path]) serves
    HTTPS and gRPC over TLS (mutual TLS when ``client_ca`` is given) from the
    Python front ends (tcserve speaks plaintext only)."""
    server.loop = asyncio.get_running_loop()
    if tls:
        native_grpc = False
    if native_grpc is None:
        native_grpc = native_grpc_available()
    runner = None
    native_http = native_grpc and http_port is not None and grpc_port is not None and \
        os.environ.get("TCSERVE_HTTP", "1") != "0"
    inner_http = None
    if http_port is not None:
        runner = web.AppRunner(HttpFrontend(server).app, access_log=None)
        await runner.setup()
        if native_http:
            # the public HTTP port is tcserve's; aiohttp serves what it relays
            site = web.TCPSite(runner, "127.0.0.1", 0, reuse_address=True)
            await site.start()
            inner_http = site._server.sockets[0].getsockname()[1]
        else:
            ctx = None
            if tls:
                import ssl

                ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
                ctx.load_cert_chain(tls["cert"], tls["key"])
                if tls.get("client_ca"):
                    ctx.load_verify_locations(tls["client_ca"])
                    ctx.verify_mode = ssl.CERT_REQUIRED
            site = web.TCPSite(runner, host, http_port, reuse_address=True, ssl_context=ctx)
            await site.start()
    gserver = None
    nf = None
    if grpc_port is not None:
        gserver = grpc.aio.server(options=GRPC_OPTIONS, interceptors=[FaultInjector()])
        service_pb2_grpc.add_GRPCInferenceServiceServicer_to_server(GrpcFrontend(server), gserver)
        if native_grpc:
            inner = gserver.add_insecure_port("127.0.0.1:0")
        elif tls:
            with open(tls["key"], "rb") as f:
                key = f.read()
            with open(tls["cert"], "rb") as f:
                cert = f.read()
            ca = None
            if tls.get("client_ca"):
                with open(tls["client_ca"], "rb") as f:
                    ca = f.read()
            creds = grpc.ssl_server_credentials([(key, cert)], root_certificates=ca, require_client_auth=ca is not None)
            gserver.add_secure_port("%s:%d" % (host, grpc_port), creds)
        else:
            gserver.add_insecure_port("%s:%d" % (host, grpc_port))
        await gserver.start()
        if native_grpc:
            from .native_frontend import NativeFrontend

            nf = NativeFrontend(server, host, grpc_port, inner)
            nf.register_all()
            server.native_frontend = nf
            if native_http:
                nf.listen_http(host, http_port, inner_http)
    if ready_evt is not None:
        ready_evt.set()
    stop = stop_evt or asyncio.Event()
    try:
        await stop.wait()
    finally:
        if nf is not None:
            nf.close()
            server.native_frontend = None
        if gserver is not None:
            await gserver.stop(0.5)
        if runner is not None:
            await runner.cleanup()


class ServerHandle:
    """Runs an InferenceServer on a background thread (tests, benches)."""

    def __init__(self, models=None, http_port=None, grpc_port=None, model_options=None, load=True, native_grpc=None,
                 tls=None):
        self.native_grpc = native_grpc
        self.tls = tls
        self.http_port = http_port or _free_port()
        self.grpc_port = grpc_port or _free_port()
        self.server = InferenceServer(models if models is not None else default_models(), model_options)
        if load:
            self.server.load_all()
        self._ready = threading.Event()
        self._loop = None
        self._stop = None
        self._thread = threading.Thread(target=self._run, daemon=True)

    @property
    def http_url(self):
        return "127.0.0.1:%d" % self.http_port

    @property
    def grpc_url(self):
        return "127.0.0.1:%d" % self.grpc_port

    def _run(self):
        loop = asyncio.new_event_loop()
        self._loop = loop
        asyncio.set_event_loop(loop)

        async def main():
            self._stop = asyncio.Event()
            await serve(self.server, self.http_port, self.grpc_port, ready_evt=self._ready, stop_evt=self._stop,
                        native_grpc=self.native_grpc, tls=self.tls)

        loop.run_until_complete(main())
        # batcher workers (and any other task still parked on a queue) end
        # with the loop, as asyncio.run would do it
        pending = asyncio.all_tasks(loop)
        for t in pending:
            t.cancel()
        if pending:
            loop.run_until_complete(asyncio.gather(*pending, return_exceptions=True))
        loop.run_until_complete(loop.shutdown_asyncgens())
        loop.close()

    def start(self, timeout=30):
        self._thread.start()
        if not self._ready.wait(timeout):
            raise RuntimeError("server failed to start")
        return self

    def stop(self):
        if self._loop is not None and self._stop is not None:
            self._loop.call_soon_threadsafe(self._stop.set)
            self._thread.join(10)
        self.server.sys_shm.unregister()
        try:
            self.server.dev_shm.unregister()
        except Exception:
            pass
        self.server.executor.shutdown(wait=False)

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()


def start_server(**kw):
    return ServerHandle(**kw).start()
