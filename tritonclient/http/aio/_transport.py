"""asyncio keep-alive HTTP/1.1 connection pool for the asyncio HTTP client.

The reference's asyncio client sits on aiohttp (``tritonclient/http/aio/
__init__.py:116-121``).  aiohttp costs ~0.35 ms of CPU per request in this
process (request/response objects, header multidicts, stream readers, and by
default an ``Accept-Encoding: gzip, deflate`` header that makes the server
compress every response), which capped the asyncio client below the
synchronous one.  This transport is one ``asyncio.Protocol`` per connection:

* a request is one ``writelines`` of [head, *body buffers] (the tensor buffers
  are not joined in Python first);
* the response head is parsed once; a ``Content-Length`` body is received
  straight into one preallocated ``bytearray``; chunked bodies are decoded;
* connections are pooled (``limit`` at most, like aiohttp's ``conn_limit``),
  reused across requests (HTTP/1.1 keep-alive), and a request that finds its
  reused connection closed by the server before any response byte arrived is
  retried once on a fresh one.
"""

import asyncio
import socket
from collections import deque

_CRLF2 = b"\r\n\r\n"


class HttpTransportError(Exception):
    pass


class Headers(dict):
    """Response headers, case-insensitive (stored lower-cased)."""

    def get(self, key, default=None):
        return dict.get(self, key.lower(), default)

    def __getitem__(self, key):
        return dict.__getitem__(self, key.lower())

    def __contains__(self, key):
        return dict.__contains__(self, key.lower())


class Response:
    __slots__ = ("status", "reason", "headers", "body")

    def __init__(self, status, reason, headers, body):
        self.status = status
        self.reason = reason
        self.headers = headers
        self.body = body


class _Conn(asyncio.Protocol):
    def __init__(self, loop):
        self._loop = loop
        self.transport = None
        self.closed = False
        self.reused = False
        self._waiter = None
        self._reset()

    def _reset(self):
        self._buf = bytearray()
        self._head = None  # (status, reason, headers)
        self._body = None
        self._filled = 0
        self._need = -1  # body bytes expected; -1 unknown (chunked / until close)
        self._chunked = False
        self._got_any = False

    # -- protocol callbacks ------------------------------------------------------------
    def connection_made(self, transport):
        self.transport = transport
        sock = transport.get_extra_info("socket")
        if sock is not None:
            try:
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass

    def connection_lost(self, exc):
        self.closed = True
        w = self._waiter
        if w is not None and not w.done():
            if self._head is not None and self._need < 0 and not self._chunked:
                # body delimited by connection close
                self._finish(bytes(self._buf))
            else:
                err = HttpTransportError("connection closed by the server%s" % (": %s" % exc if exc else ""))
                err.retryable = not self._got_any
                w.set_exception(err)

    def data_received(self, data):
        self._got_any = True
        if self._body is not None:
            n = min(len(data), self._need - self._filled)
            self._body[self._filled:self._filled + n] = data[:n] if n < len(data) else data
            self._filled += n
            if self._filled == self._need:
                self._finish(self._body)
            return
        self._buf += data
        self._advance()

    # -- parsing -----------------------------------------------------------------------
    def _advance(self):
        if self._head is None:
            i = self._buf.find(_CRLF2)
            if i < 0:
                return
            lines = bytes(self._buf[:i]).decode("latin-1").split("\r\n")
            del self._buf[:i + 4]
            parts = lines[0].split(" ", 2)
            try:
                status = int(parts[1])
            except (IndexError, ValueError):
                return self._fail(HttpTransportError("malformed HTTP status line: %r" % lines[0]))
            hdrs = Headers()
            for ln in lines[1:]:
                k, _, v = ln.partition(":")
                hdrs[k.strip().lower()] = v.strip()
            self._head = (status, parts[2] if len(parts) > 2 else "", hdrs)
            te = hdrs.get("transfer-encoding", "")
            if "chunked" in te.lower():
                self._chunked = True
            elif "content-length" in hdrs:
                self._need = int(hdrs["content-length"])
                if len(self._buf) >= self._need:
                    body = bytes(self._buf[:self._need])
                    del self._buf[:self._need]
                    return self._finish(body)
                self._body = bytearray(self._need)
                self._body[:len(self._buf)] = self._buf
                self._filled = len(self._buf)
                self._buf = bytearray()
                return
            else:
                return  # until close
        if self._chunked:
            self._advance_chunked()

    def _advance_chunked(self):
        out = getattr(self, "_chunks", None)
        if out is None:
            out = self._chunks = bytearray()
        while True:
            i = self._buf.find(b"\r\n")
            if i < 0:
                return
            size = int(bytes(self._buf[:i]).split(b";")[0], 16)
            if size == 0:
                rest = self._buf[i + 2:]
                if not rest.startswith(b"\r\n") and rest.find(_CRLF2) < 0:
                    return  # trailers not complete yet
                del self._buf[:]
                self._chunks = None
                return self._finish(bytes(out))
            if len(self._buf) < i + 2 + size + 2:
                return
            out += self._buf[i + 2:i + 2 + size]
            del self._buf[:i + 2 + size + 2]

    def _finish(self, body):
        status, reason, hdrs = self._head
        w = self._waiter
        self._waiter = None
        self._reset()
        if w is not None and not w.done():
            w.set_result(Response(status, reason, hdrs, body))

    def _fail(self, err):
        w = self._waiter
        self._waiter = None
        if w is not None and not w.done():
            w.set_exception(err)
        self.close()

    # -- request -----------------------------------------------------------------------
    def send(self, buffers):
        self._reset()
        self._waiter = self._loop.create_future()
        self.transport.writelines(buffers)
        return self._waiter

    def close(self):
        if self.transport is not None and not self.closed:
            self.transport.close()
        self.closed = True


class Pool:
    """At most ``limit`` keep-alive connections to one host."""

    def __init__(self, host, port, ssl_context=None, limit=100):
        self.host, self.port = host, int(port)
        self.ssl = ssl_context
        self._sem = asyncio.Semaphore(max(1, int(limit)))
        self._idle = deque()
        self._all = set()
        self._host_header = ("%s:%d" % (host, self.port)).encode()

    async def _connect(self):
        loop = asyncio.get_running_loop()
        _, conn = await loop.create_connection(lambda: _Conn(loop), self.host, self.port, ssl=self.ssl,
                                               server_hostname=self.host if self.ssl else None)
        self._all.add(conn)
        return conn

    async def request(self, method, path, headers, body=None):
        """``body``: None, bytes or a list of bytes-like buffers."""
        bufs = [] if body is None else ([body] if isinstance(body, (bytes, bytearray, memoryview)) else list(body))
        n = sum(memoryview(b).nbytes for b in bufs)
        head = [b"%s %s HTTP/1.1\r\nHost: %s\r\n" % (method.encode(), path.encode(), self._host_header)]
        for k, v in headers.items():
            head.append(("%s: %s\r\n" % (k, v)).encode("latin-1"))
        if body is not None or method == "POST":
            head.append(b"Content-Length: %d\r\n" % n)
        head.append(b"\r\n")
        buffers = [b"".join(head)] + [b for b in bufs if memoryview(b).nbytes]
        idempotent = method in ("GET", "HEAD")
        async with self._sem:
            for attempt in (0, 1):
                conn = None
                while self._idle:
                    c = self._idle.pop()
                    if not c.closed:
                        conn = c
                        break
                    self._all.discard(c)
                if conn is None:
                    conn = await self._connect()
                try:
                    resp = await conn.send(buffers)
                except HttpTransportError as e:
                    conn.close()
                    self._all.discard(conn)
                    # a reused keep-alive connection the server closed before
                    # any response byte: retried once, for GET/HEAD only.  A
                    # POST (infer, load, shm register) may already have run on
                    # the server; re-sending it could duplicate a sequence step,
                    # so it surfaces as the reference's aiohttp client does.
                    if attempt == 0 and conn.reused and getattr(e, "retryable", False) and idempotent:
                        continue
                    raise
                except BaseException:
                    conn.close()  # cancelled / timed out mid-request: the connection state is unknown
                    self._all.discard(conn)
                    raise
                if conn.closed or resp.headers.get("connection", "").lower() == "close":
                    conn.close()
                    self._all.discard(conn)
                else:
                    conn.reused = True
                    self._idle.append(conn)
                return resp

    def close(self):
        for c in list(self._all):
            c.close()
        self._all.clear()
        self._idle.clear()
