"""Per-device HIP state for the client's device-side data paths.

One non-blocking HIP stream and one grow-only scratch allocation per device,
shared by ``hip_shared_memory`` (K2/K3/K4/K5 on set/get) and
``InferInput.set_data_from_dlpack`` (K4/K5 before the D2H).  The reference
creates and destroys a CUDA stream per call and keeps no device scratch
(``tritonclient/utils/cuda_shared_memory/_utils.py:103-121``); re-creating
them on every set/get was a measurable share of small-tensor calls.

Use::

    ctx = context(dev)
    with ctx.lock:                 # the stream and scratch are not re-entrant
        tmp = ctx.scratch(nbytes)  # device pointer, >= nbytes, 256-B aligned
        ...launch on ctx.stream.handle...
        ctx.stream.synchronize()
"""

import threading

_LOCK = threading.Lock()
_CTX = {}


def _hip():
    from triton_client_amd.ops import hip

    return hip


class DeviceContext:
    def __init__(self, dev):
        hip = _hip()
        self.dev = int(dev)
        self.lock = threading.RLock()
        self.stream = hip.Stream(self.dev)
        self._scratch = 0
        self._bytes = 0

    def scratch(self, nbytes):
        """Device scratch of at least ``nbytes`` (call with ``lock`` held)."""
        nbytes = int(nbytes)
        if nbytes > self._bytes:
            hip = _hip()
            old = self._bytes  # doubling is against the size being replaced
            if self._scratch:
                self.stream.synchronize()
                hip.free(self.dev, self._scratch)
                self._scratch, self._bytes = 0, 0
            size = max(nbytes, 2 * old, 1 << 20)
            size = (size + (2 << 20) - 1) & ~((2 << 20) - 1)
            self._scratch = hip.malloc(self.dev, size)
            self._bytes = size
        return self._scratch

    def scratch_bytes(self):
        return self._bytes

    def release_scratch(self):
        """Free the scratch allocation (it is re-created on the next use)."""
        with self.lock:
            if self._scratch:
                self.stream.synchronize()
                _hip().free(self.dev, self._scratch)
            self._scratch, self._bytes = 0, 0


def context(dev):
    dev = int(dev)
    with _LOCK:
        c = _CTX.get(dev)
        if c is None:
            c = _CTX[dev] = DeviceContext(dev)
        return c


def release_all_scratch():
    with _LOCK:
        ctxs = list(_CTX.values())
    for c in ctxs:
        c.release_scratch()
