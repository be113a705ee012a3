"""Bench-server lifecycle helpers shared by bench.py, perf tools and GPU tests."""

import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


STRIPE_BASE, STRIPE_WIDTH = 20000, 64


def free_ports(n, stripe):
    """``n`` distinct free ports from stripe ``stripe`` (e.g. the local rank):
    [20000 + 64*stripe, +64), below the kernel's ephemeral range.  Ranks that
    start servers at the same moment get disjoint numbers, and no port a
    server or RCCL later binds to 0 can land on a number handed out here
    between the probe and the server's own bind (a ``free_port()`` race)."""
    lo = STRIPE_BASE + STRIPE_WIDTH * int(stripe)
    out = []
    for p in range(lo, lo + STRIPE_WIDTH):
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
        except OSError:
            continue
        finally:
            s.close()
        out.append(p)
        if len(out) == n:
            return out
    raise RuntimeError("no %d free ports in stripe %d [%d, %d)" % (n, stripe, lo, lo + STRIPE_WIDTH))


class ServerProcess:
    """The KServe-v2 server in a child process (HIP IPC needs a 2nd process)."""

    def __init__(self, device=0, gpu=True, models="", http_port=None, grpc_port=None,
                 extra_args=(), log_path=None, env=None, port_stripe=None):
        if port_stripe is not None and not (http_port or grpc_port):
            http_port, grpc_port = free_ports(2, port_stripe)
        self.http_port = http_port or free_port()
        self.grpc_port = grpc_port or free_port()
        self.device = device
        args = [sys.executable, "-m", "triton_client_amd.server",
                "--http-port", str(self.http_port), "--grpc-port", str(self.grpc_port),
                "--device", str(device)]
        if gpu:
            args.append("--gpu")
        if models:
            args += ["--models", models]
        args += list(extra_args)
        e = dict(os.environ)
        e["PYTHONPATH"] = REPO + os.pathsep + e.get("PYTHONPATH", "")
        if env:
            e.update(env)
        self.log_path = log_path
        self._log = open(log_path, "w") if log_path else subprocess.DEVNULL
        self.proc = subprocess.Popen(args, cwd=REPO, env=e, stdout=self._log, stderr=subprocess.STDOUT,
                                     start_new_session=True)

    @property
    def grpc_url(self):
        return "127.0.0.1:%d" % self.grpc_port

    @property
    def http_url(self):
        return "127.0.0.1:%d" % self.http_port

    def wait_ready(self, timeout=600, model=None):
        import tritonclient.http as httpclient

        t0 = time.time()
        last = None
        said = t0
        while time.time() - t0 < timeout:
            if self.proc.poll() is not None:
                raise RuntimeError("server exited with %s (log: %s)" % (self.proc.returncode, self.log_path))
            if time.time() - said >= 30:  # a long model load (graph captures) must not look hung
                said = time.time()
                print("[harness] waiting for the server (%s): %.0f s" % (model or "ready", said - t0), file=sys.stderr,
                      flush=True)
            try:
                c = httpclient.InferenceServerClient(self.http_url, connection_timeout=2, network_timeout=5)
                ok = c.is_server_ready() and (model is None or c.is_model_ready(model))
                c.close()
                if ok:
                    return self
            except Exception as e:  # noqa: BLE001
                last = e
            time.sleep(0.5)
        raise TimeoutError("server not ready after %ss: %s" % (timeout, last))

    def dump_stacks(self, settle_s=2.0):
        """SIGUSR1: the server writes every thread's Python stack to its log."""
        import signal

        if self.proc.poll() is None:
            self.proc.send_signal(signal.SIGUSR1)
            time.sleep(settle_s)

    def stop(self):
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(30)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait(10)
        if self._log not in (None, subprocess.DEVNULL):
            self._log.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()


class ExternalServer:
    """A server started elsewhere (e.g. under rocprofv3); same interface."""

    def __init__(self, grpc_url, http_url=""):
        self.grpc_url = grpc_url
        if not http_url:
            host, port = grpc_url.rsplit(":", 1)
            http_url = "%s:%d" % (host, int(port) - 1)
        self.http_url = http_url
        self.log_path = None
        self.proc = None

    def wait_ready(self, timeout=600, model=None):
        import tritonclient.http as httpclient

        t0 = time.time()
        last = None
        while time.time() - t0 < timeout:
            try:
                c = httpclient.InferenceServerClient(self.http_url, connection_timeout=2, network_timeout=5)
                ok = c.is_server_ready() and (model is None or c.is_model_ready(model))
                c.close()
                if ok:
                    return self
            except Exception as e:  # noqa: BLE001
                last = e
            time.sleep(0.5)
        raise TimeoutError("external server not ready after %ss: %s" % (timeout, last))

    def stop(self):
        pass
