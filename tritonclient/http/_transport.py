"""Keep-alive HTTP/1.1 connection pool for the synchronous HTTP client.

Replaces the reference's geventhttpclient dependency
(``tritonclient/http/_client.py:182-191``) with a small stdlib transport
designed for tensor payloads:

* request bodies are lists of buffers sent with one ``sendmsg`` (scatter/gather
  ``writev``) — the JSON header and each tensor's bytes go to the kernel
  without first being concatenated (the reference ``b"".join``s them,
  ``http/_utils.py:141-150``);
* responses are read with ``recv_into`` into a single preallocated
  ``bytearray`` sized from ``Content-Length`` so binary outputs can be exposed
  zero-copy via ``np.frombuffer``;
* ``concurrency`` sockets are pooled and handed out under a lock, so one client
  can be shared by the thread pool that backs ``async_infer``.
"""

import socket
import ssl as _ssl
import threading
from collections import deque

_CRLF = b"\r\n"


class HttpError(Exception):
    pass


class Response:
    """Minimal response object: ``status_code``, ``get(header)``, ``read(n)``."""

    __slots__ = ("status_code", "reason", "headers", "_body", "_pos")

    def __init__(self, status_code, reason, headers, body):
        self.status_code = status_code
        self.reason = reason
        self.headers = headers  # lower-cased name -> value
        self._body = body
        self._pos = 0

    def get(self, name, default=None):
        return self.headers.get(name.lower(), default)

    def read(self, length=-1):
        if length is None or length < 0:
            out = self._body[self._pos :] if self._pos else self._body
            self._pos = len(self._body)
            return bytes(out) if isinstance(out, memoryview) else out
        start = self._pos
        self._pos = min(len(self._body), start + length)
        out = self._body[start : self._pos]
        return bytes(out) if isinstance(out, memoryview) else out

    def read_view(self):
        """Zero-copy memoryview of the unread remainder of the body."""
        mv = memoryview(self._body)[self._pos :]
        self._pos = len(self._body)
        return mv

    def __repr__(self):
        return "<Response %d %s %s>" % (self.status_code, self.reason, self.headers)


class _Conn:
    def __init__(self, host, port, connection_timeout, network_timeout, ssl_context):
        sock = socket.create_connection((host, port), timeout=connection_timeout)
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        sock.settimeout(network_timeout)
        if ssl_context is not None:
            sock = ssl_context.wrap_socket(sock, server_hostname=host)
        self.sock = sock
        self.is_ssl = ssl_context is not None
        self.buf = bytearray()
        self.closed = False

    def close(self):
        if not self.closed:
            self.closed = True
            try:
                self.sock.close()
            except OSError:
                pass

    # -- send --------------------------------------------------------------
    def send(self, parts):
        if self.is_ssl:
            self.sock.sendall(b"".join(bytes(p) for p in parts))
            return
        views = [memoryview(p).cast("B") for p in parts if len(p)]
        while views:
            n = self.sock.sendmsg(views[:512])
            while n:
                head = views[0]
                if n >= len(head):
                    n -= len(head)
                    views.pop(0)
                else:
                    views[0] = head[n:]
                    n = 0

    # -- receive -----------------------------------------------------------
    def _fill(self):
        chunk = self.sock.recv(262144)
        if not chunk:
            raise HttpError("connection closed by peer")
        self.buf += chunk

    def _read_line_block(self):
        while True:
            idx = self.buf.find(b"\r\n\r\n")
            if idx >= 0:
                head = bytes(self.buf[:idx])
                del self.buf[: idx + 4]
                return head
            self._fill()

    def _read_exact(self, n):
        out = bytearray(n)
        mv = memoryview(out)
        have = min(len(self.buf), n)
        mv[:have] = self.buf[:have]
        del self.buf[:have]
        while have < n:
            got = self.sock.recv_into(mv[have:], n - have)
            if got == 0:
                raise HttpError("connection closed by peer mid-body")
            have += got
        return out

    def _read_chunked(self):
        out = bytearray()
        while True:
            while b"\r\n" not in self.buf:
                self._fill()
            idx = self.buf.find(b"\r\n")
            size = int(bytes(self.buf[:idx]).split(b";")[0], 16)
            del self.buf[: idx + 2]
            if size == 0:
                # trailers until blank line
                while True:
                    while b"\r\n" not in self.buf:
                        self._fill()
                    idx = self.buf.find(b"\r\n")
                    line = self.buf[:idx]
                    del self.buf[: idx + 2]
                    if not line:
                        return out
            out += self._read_exact(size)
            while len(self.buf) < 2:
                self._fill()
            del self.buf[:2]

    def read_response(self, method):
        head = self._read_line_block()
        lines = head.split(_CRLF)
        status = lines[0].split(b" ", 2)
        if len(status) < 2 or not status[0].startswith(b"HTTP/"):
            raise HttpError("malformed status line %r" % lines[0])
        code = int(status[1])
        reason = status[2].decode("latin-1") if len(status) > 2 else ""
        headers = {}
        for line in lines[1:]:
            k, _, v = line.partition(b":")
            headers[k.strip().lower().decode("latin-1")] = v.strip().decode("latin-1")
        if method == "HEAD" or code in (204, 304) or 100 <= code < 200:
            body = b""
        elif headers.get("transfer-encoding", "").lower() == "chunked":
            body = self._read_chunked()
        elif "content-length" in headers:
            body = self._read_exact(int(headers["content-length"]))
        else:
            # read until close
            chunks = [bytes(self.buf)]
            self.buf.clear()
            while True:
                c = self.sock.recv(262144)
                if not c:
                    break
                chunks.append(c)
            body = b"".join(chunks)
            self.closed = True
        if headers.get("connection", "").lower() == "close":
            self.closed = True
        return Response(code, reason, headers, body)


class ConnectionPool:
    """Pool of up to ``concurrency`` keep-alive connections to one endpoint."""

    def __init__(
        self,
        host,
        port,
        concurrency=1,
        connection_timeout=60.0,
        network_timeout=60.0,
        ssl_context=None,
    ):
        self.host = host
        self.port = port
        self.host_header = host if port in (80, 443) else "%s:%d" % (host, port)
        self.concurrency = max(1, int(concurrency))
        self.connection_timeout = connection_timeout
        self.network_timeout = network_timeout
        self.ssl_context = ssl_context
        self._idle = deque()
        self._sem = threading.BoundedSemaphore(self.concurrency)
        self._lock = threading.Lock()
        self._closed = False

    def _acquire(self):
        self._sem.acquire()
        with self._lock:
            while self._idle:
                c = self._idle.pop()
                if not c.closed:
                    return c, True
        try:
            return (
                _Conn(
                    self.host,
                    self.port,
                    self.connection_timeout,
                    self.network_timeout,
                    self.ssl_context,
                ),
                False,
            )
        except BaseException:
            self._sem.release()
            raise

    def _release(self, conn):
        with self._lock:
            if not conn.closed and not self._closed:
                self._idle.append(conn)
            else:
                conn.close()
        self._sem.release()

    def request(self, method, uri, body_parts=(), headers=None):
        """Send one request; ``body_parts`` is a sequence of buffers."""
        if self._closed:
            raise HttpError("client is closed")
        total = sum(len(p) for p in body_parts)
        head = ["%s %s HTTP/1.1" % (method, uri), "Host: " + self.host_header]
        if headers:
            for k, v in headers.items():
                head.append("%s: %s" % (k, v))
        if method != "GET" or total:
            head.append("Content-Length: %d" % total)
        head.append("")
        head.append("")
        header_bytes = "\r\n".join(head).encode("latin-1")
        for attempt in (0, 1):
            conn, reused = self._acquire()
            try:
                conn.send([header_bytes, *body_parts])
                resp = conn.read_response(method)
            except (HttpError, ConnectionError, BrokenPipeError) as e:
                conn.close()
                self._release(conn)
                # A pooled keep-alive socket may have been closed by the server
                # while idle: retry exactly once on a fresh connection.
                if attempt == 0 and reused:
                    continue
                raise HttpError(str(e)) from None
            except BaseException:
                conn.close()
                self._release(conn)
                raise
            self._release(conn)
            return resp
        raise HttpError("unreachable")

    def close(self):
        with self._lock:
            self._closed = True
            while self._idle:
                self._idle.pop().close()


def make_ssl_context(ssl_options=None, ssl_context_factory=None, insecure=False):
    """Build an ``ssl.SSLContext`` from geventhttpclient-style options."""
    if ssl_context_factory is not None:
        ctx = ssl_context_factory()
    else:
        ctx = _ssl.create_default_context()
    opts = dict(ssl_options or {})
    if "ca_certs" in opts:
        ctx.load_verify_locations(cafile=opts["ca_certs"])
    if "certfile" in opts:
        ctx.load_cert_chain(opts["certfile"], opts.get("keyfile"))
    if insecure or opts.get("cert_reqs") == _ssl.CERT_NONE:
        ctx.check_hostname = False
        ctx.verify_mode = _ssl.CERT_NONE
    return ctx
