"""K3 (device BYTES index, csrc/kernels/bytes.hip) under the conditions of the
round-4 failure (wrong element counts, "the region holds 163
BYTES elements, 1024 requested", and one illegal address under back-to-back
unserialised calls with the stream-ordered workspace).

* Overrun check: K3's workspace at EXACTLY the size each call asks for, a
  4 KiB canary behind it (tcamd_k3_set_check), and sentinel tails behind the
  caller's offsets / lengths / status buffers; every call's index must equal
  the host walk, with no sentinel or canary byte changed.  Covers the three
  paths (v3 walk with 64 and 256 candidates, the general walk) on the
  failing record's data (n = 1024 / 4096, mean length 20).
* Concurrency: two threads on two streams, each indexing its own region back
  to back (the K3 workspace is one per device, owned by the call holding its
  mutex until its stream drained).
* The recorded sequence through the public API: HIP-shm set (K2) and get
  (K3) round trips, unserialised.
"""

import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

SENT = 0x5A5A5A5A


def _chain(rng, n, lo, hi):
    lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
    buf = bytearray()
    offs = np.empty(n, np.uint64)
    for i, L in enumerate(lens):
        buf += int(L).to_bytes(4, "little")
        offs[i] = len(buf)
        buf += bytes(rng.integers(97, 123, int(L), dtype=np.uint8))
    return bytes(buf), offs, lens


class _Bufs:
    """Device offs / lens / status with sentinel tails."""

    def __init__(self, n):
        self.n = n
        self.offs = torch.full((n + 64,), SENT, dtype=torch.int64, device="cuda")
        self.lens = torch.full((n + 64,), SENT, dtype=torch.int32, device="cuda")
        self.status = torch.full((4 + 64,), SENT, dtype=torch.int32, device="cuda")

    def run(self, hip, data_dev, nbytes, stream):
        self.offs.fill_(SENT)
        self.lens.fill_(SENT)
        self.status.fill_(SENT)
        torch.cuda.synchronize()
        hip.index_bytes(data_dev.data_ptr(), nbytes, self.n, self.offs.data_ptr(), self.lens.data_ptr(),
                        self.status.data_ptr(), stream)
        torch.cuda.synchronize()
        st = self.status.cpu().numpy()
        assert (self.offs[self.n:] == SENT).all() and (self.lens[self.n:] == SENT).all(), "offs/lens overrun"
        assert (st[4:] == SENT).all(), "status overrun"
        return int(st[0]), self.offs[:self.n].cpu().numpy().astype(np.uint64), \
            self.lens[:self.n].cpu().numpy().astype(np.uint32)


@pytest.fixture
def hip_check():
    from triton_client_amd.ops import hip

    prev = hip.k3_set_check(True)
    yield hip
    hip.k3_set_check(prev)


@pytest.mark.parametrize("n,lo,hi,path", [(1024, 0, 40, 1), (4096, 0, 40, 1), (16384, 0, 40, 1), (2048, 40, 250, 3),
                                          (600, 200, 9000, 2)])
def test_k3_exact_workspace_no_overrun(hip_check, n, lo, hi, path):
    hip = hip_check
    rng = np.random.default_rng(n + lo + hi)
    raw, offs, lens = _chain(rng, n, lo, hi)
    data = torch.frombuffer(bytearray(raw + b"\0" * 64), dtype=torch.uint8).cuda()
    b = _Bufs(n)
    s = torch.cuda.Stream()
    for rep in range(30):
        st, o, ln = b.run(hip, data, len(raw), s.cuda_stream)
        assert st == 0, (rep, st)
        np.testing.assert_array_equal(o, offs)
        np.testing.assert_array_equal(ln, lens)
    assert hip.index_bytes_last_path()[0] == path
    # asking for more elements than the chain holds: status 1 with the count, no overrun
    b2 = _Bufs(n + 7)
    st, _, _ = b2.run(hip, data, len(raw), s.cuda_stream)
    assert st == 1
    assert int(b2.status[2:4].cpu().numpy().view(np.uint64)[0]) == n


def test_k3_two_streams_back_to_back():
    from triton_client_amd.ops import hip

    errs = []

    def worker(k):
        try:
            rng = np.random.default_rng(100 + k)
            n = (1024, 4096)[k]
            raw, offs, lens = _chain(rng, n, 0, 40)
            data = torch.frombuffer(bytearray(raw + b"\0" * 64), dtype=torch.uint8).cuda()
            s = torch.cuda.Stream()
            offs_d = torch.empty(n, dtype=torch.int64, device="cuda")
            lens_d = torch.empty(n, dtype=torch.int32, device="cuda")
            st_d = torch.empty(4, dtype=torch.int32, device="cuda")
            for rep in range(150):
                with torch.cuda.stream(s):
                    offs_d.zero_()
                hip.index_bytes(data.data_ptr(), len(raw), n, offs_d.data_ptr(), lens_d.data_ptr(), st_d.data_ptr(),
                                s.cuda_stream)
                s.synchronize()
                st = int(st_d.cpu()[0])
                if st != 0 or not np.array_equal(offs_d.cpu().numpy().astype(np.uint64), offs) or \
                        not np.array_equal(lens_d.cpu().numpy().astype(np.uint32), lens):
                    errs.append((k, rep, st))
                    return
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append((k, repr(e)))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs


def test_k3_recorded_sequence_through_hip_shm():
    """The round-4 failing sequence: device set (K2) then device get (K3) of
    the same region, back to back, at n = 1024 and 4096 (mean length 20)."""
    from tritonclient.utils import hip_shared_memory as hipshm
    from tritonclient.utils import serialize_byte_tensor

    rng = np.random.default_rng(0)
    for n in (1024, 4096):
        lens = rng.integers(0, 41, n)
        pool = rng.integers(97, 123, int(lens.sum()) + 1, dtype=np.uint8).tobytes()
        o = np.concatenate([[0], np.cumsum(lens)])
        data = np.array([pool[o[i]:o[i + 1]] for i in range(n)], dtype=np.object_)
        want = serialize_byte_tensor(data).item()
        h = hipshm.create_shared_memory_region("k3seq_%d" % n, len(want) + 256, 0)
        try:
            for rep in range(60):
                hipshm.set_shared_memory_region(h, [data], serialize_bytes=True, bytes_path="device")
                out = hipshm.get_contents_as_numpy(h, np.object_, [n], bytes_path="device")
                assert list(out) == list(data), (n, rep)
        finally:
            hipshm.destroy_shared_memory_region(h)
