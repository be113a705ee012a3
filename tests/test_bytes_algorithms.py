"""CPU models of the K2 / K3 device algorithms (csrc/kernels/bytes.hip).

The kernels themselves are checked bit-exactly on the GPU
(tests/test_kernels_gpu.py); these tests run the same block decomposition,
candidate walk, resolve and tile arithmetic in numpy/Python on many shapes
(including the edge cases that only a few inputs hit: elements longer than
the candidate window, zero-length runs, data ending on a block boundary,
trailing garbage after the last element, windows smaller than the data) and
compare against the host codec, so a logic error is caught on the CPU before
a kernel ever runs.
"""

import numpy as np
import pytest

from tritonclient.utils import serialize_byte_tensor

XB, XR = 4096, 256
BAD, FAR, END = 0xFFFF, 0xFFFE, 0xFFFD
AMBIG, NONE = 0xFFFFFFFF, 0xFFFFFFFE
MAX_BACK = 64


def _le32(buf, p):
    return int.from_bytes(bytes(buf[p:p + 4]), "little")


def k3_model(buf, nbytes, window, n_expected):
    """Python model of index_v3 (ix_walk/ix_resolve/ix_mask/scan/ix_status/ix_emit).
    Returns (status, offs, lens)."""
    nblk = (window + XB - 1) // XB
    tab = np.zeros((nblk, XR), np.uint32)
    tcnt = np.zeros((nblk, XR), np.uint32)
    sync = np.zeros(nblk, np.uint64)
    for b in range(nblk):
        b0, bend = b * XB, (b + 1) * XB
        live_codes = []
        for c in range(XR):
            p = b0 + c
            cnt = 0
            if p >= nbytes:
                code = END
            else:
                while True:
                    if p + 4 > nbytes:
                        code = BAD
                        break
                    nx = p + 4 + _le32(buf, p)
                    if nx > nbytes:
                        code = BAD
                        break
                    cnt += 1
                    p = nx
                    if nx == nbytes:
                        code = END
                        break
                    if nx >= bend:
                        code = nx - bend if nx - bend < XR else FAR
                        break
            tab[b, c], tcnt[b, c] = code, cnt
            if code < XR:
                live_codes.append(code)
        sync[b] = NONE if not live_codes else (live_codes[0] if min(live_codes) == max(live_codes) else AMBIG)
    end, fail = None, None
    entry = [NONE] * nblk
    count = np.zeros(nblk, np.uint64)
    for b in range(nblk):
        if b == 0:
            e, k = 0, 0
        else:
            j, depth = b - 1, 0
            while j > 0 and sync[j] == AMBIG and depth < MAX_BACK:
                j -= 1
                depth += 1
            if sync[j] == AMBIG and j > 0:
                fail = b if fail is None else min(fail, b)
                continue
            if sync[j] == AMBIG:
                e, k = 0, 0
            else:
                e = NONE if sync[j] == NONE else int(sync[j])
                k = j + 1
            while k < b and e != NONE:
                c = tab[k, e]
                e = int(c) if c < XR else NONE
                k += 1
        entry[b] = e
        if e == NONE:
            continue
        count[b] = tcnt[b, e]
        c = tab[b, e]
        reason = {END: 0, BAD: 1, FAR: 2}.get(int(c), 3 if b == nblk - 1 else None)
        if reason is not None:
            key = (b << 2) | reason
            end = key if end is None else min(end, key)
    if end is None:  # every block from `fail` on unresolved: the kernel's ctl->end stays all-ones
        end = (1 << 64) - 1
    end_blk, reason = end >> 2, end & 3
    count[end_blk + 1:] = 0
    if fail is not None:
        count[fail:] = 0  # the chain may end inside an unresolved block
    total = int(count.sum())
    if total >= n_expected:
        st = 0
    elif fail is not None and fail <= end_blk:
        st = 3
    else:
        st = {0: 1, 1: -1, 2: 3, 3: 2}[reason]
    if st not in (0, 1):
        return st, None, None
    offs, lens = [], []
    for b in range(nblk):
        if entry[b] == NONE or b > end_blk or count[b] == 0:
            continue
        p = b * XB + entry[b]
        for _ in range(int(count[b])):
            if len(offs) >= n_expected:
                break
            L = _le32(buf, p)
            offs.append(p + 4)
            lens.append(L)
            p += 4 + L
    return st, np.array(offs, np.uint64), np.array(lens, np.uint32)


def host_index(buf, nbytes, n):
    offs, lens, p = [], [], 0
    while len(offs) < n:
        if p + 4 > nbytes:
            return (1 if p == nbytes else -1), None, None
        L = _le32(buf, p)
        if p + 4 + L > nbytes:
            return -1, None, None
        offs.append(p + 4)
        lens.append(L)
        p += 4 + L
    return 0, np.array(offs, np.uint64), np.array(lens, np.uint32)


def k3_driver(buf, nbytes, n):
    """The host loop of tcamd_index_bytes: grow the window 8x, fall back."""
    window = min(nbytes, ((max(64 * n, 1 << 20) + XB - 1) // XB) * XB)
    while True:
        st, o, ln = k3_model(buf, nbytes, window, n)
        if st in (0, 1, -1):
            return st, o, ln, "v3"
        if st == 2 and window < nbytes:
            window = min(window * 8, nbytes)
            continue
        return host_index(buf, nbytes, n) + ("general",)


def _serialize(elems):
    return np.frombuffer(serialize_byte_tensor(np.array(elems, dtype=np.object_)).item(), np.uint8)


def _random_elems(rng, n, maxlen, alphabet=None):
    out = []
    for _ in range(n):
        L = int(rng.integers(0, maxlen + 1))
        if alphabet == "zeros":
            out.append(bytes(L))
        elif alphabet == "binary":
            out.append(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        else:
            out.append(bytes(rng.integers(32, 127, L, dtype=np.uint8)))
    return out


@pytest.mark.parametrize("n,maxlen,alphabet,tail", [
    (3000, 40, None, 0),           # typical short strings
    (2000, 200, None, 3000),       # up to the candidate window, trailing region bytes
    (4000, 8, "zeros", 0),         # runs of zero bytes: ambiguous blocks
    (1500, 60, "binary", 777),     # random binary payloads
    (600, 5000, None, 0),          # elements longer than kXR: fallback path
    (5000, 0, None, 0),            # empty strings: 4-byte elements
])
def test_k3_model_matches_host_walk(n, maxlen, alphabet, tail):
    rng = np.random.default_rng(n + maxlen)
    data = _serialize(_random_elems(rng, n, maxlen, alphabet))
    region = np.concatenate([data, rng.integers(0, 256, tail, dtype=np.uint8)])
    st, offs, lens, path = k3_driver(region, region.size, n)
    hs, ho, hl = host_index(region, region.size, n)
    assert st == hs == 0
    np.testing.assert_array_equal(offs, ho)
    np.testing.assert_array_equal(lens, hl)
    if maxlen > XR:
        assert path == "general"


def test_k3_model_window_growth_and_block_boundary():
    # data ends exactly on a 4 KiB block boundary inside a larger region of zeros
    elems = [b"x" * 60] * (8192 // 64)
    data = _serialize(elems)
    assert data.size == 8192
    region = np.concatenate([data, np.zeros(3 * XB, np.uint8)])
    st, offs, lens, path = k3_driver(region, region.size, len(elems))
    assert st == 0 and path == "v3"
    assert list(lens) == [60] * len(elems)
    # asking for more elements than the data holds: zeros after the data parse
    # as empty elements (exactly like the host walk)
    st2, o2, l2 = k3_model(region, region.size, region.size, len(elems) + 5)
    hs, ho, hl = host_index(region, region.size, len(elems) + 5)
    assert st2 == hs == 0
    np.testing.assert_array_equal(o2, ho)


def test_k3_model_small_window_retries():
    rng = np.random.default_rng(7)
    elems = _random_elems(rng, 20000, 120)
    data = _serialize(elems)
    st, offs, lens = k3_model(data, data.size, 4 * XB, len(elems))
    assert st == 2  # the chain leaves the window before n elements
    st, offs, lens, path = k3_driver(data, data.size, len(elems))
    assert st == 0 and path == "v3" and len(offs) == len(elems)


def test_k3_model_malformed_and_short():
    data = _serialize([b"abc"] * 1000)
    bad = data.copy()
    bad[4 * 7 + 3 * 6] = 0xFF  # a length prefix with a huge low byte -> runs past the data? (stays in range)
    bad[-7:-3] = np.frombuffer((10 ** 6).to_bytes(4, "little"), np.uint8)  # last element's length runs past
    st, _, _, _ = k3_driver(bad, bad.size, 1000)
    hs, _, _ = host_index(bad, bad.size, 1000)
    assert st == hs
    st, _, _, _ = k3_driver(data, data.size, 1001)
    assert st == 1


PK_SPAN, PK_PART, PK_TILE = 1024, 65536, 8192


def k2_model(elems, stride=None):
    """Python model of pk_block_sums / scan / pk_emit (tile + chunk arithmetic)."""
    n = len(elems)
    lens = np.array([len(e) for e in elems], np.uint64)
    payload = b"".join(elems)
    nb = (n + PK_SPAN - 1) // PK_SPAN
    S = [int(lens[b * PK_SPAN:(b + 1) * PK_SPAN].sum()) for b in range(nb)]
    P = np.concatenate([[0], np.cumsum(S)]).astype(np.int64)
    total = int(P[-1]) + 4 * n
    out = bytearray(total)
    owner_written = np.zeros(total, np.int64)
    for b in range(nb):
        first = b * PK_SPAN
        cnt = min(PK_SPAN, n - first)
        bl = lens[first:first + cnt]
        os_ = np.concatenate([[0], np.cumsum(bl + 4)]).astype(np.int64)
        Lb = int(os_[cnt])
        Ob = int(P[b]) + 4 * first
        Db = int(P[b])
        parts = (Lb + PK_PART - 1) // PK_PART
        for part in range(parts):
            q0, q1 = part * PK_PART, min((part + 1) * PK_PART, Lb)
            c0, c1 = (Ob + q0) // 16, (Ob + q1 + 15) // 16
            for ct in range(c0, c1, PK_TILE // 16):
                ce = min(ct + PK_TILE // 16, c1)
                t0 = ct * 16 - Ob if ct * 16 > Ob + q0 else q0
                t1 = ce * 16 - Ob if ce * 16 < Ob + q1 else q1

                def owner(pos):
                    return int(np.searchsorted(os_[:cnt], pos, side="right") - 1)

                ea, ez = owner(t0), owner(t1 - 1)
                pa = os_[ea] - 4 * ea + (t0 - os_[ea] - 4 if t0 - os_[ea] > 4 else 0)
                pz = os_[ez] - 4 * ez + (t1 - 1 - os_[ez] - 4 + 1 if t1 - 1 - os_[ez] >= 4 else 0)
                pay_lo = (Db + pa) & ~15
                pay_hi = Db + max(pz, pa)
                assert pay_hi - pay_lo <= PK_TILE + 15
                staged = payload[pay_lo:pay_hi]
                for c in range(ct, ce):
                    l0 = c * 16 - Ob
                    for k in range(16):
                        pos = l0 + k
                        if pos < t0 or pos >= t1:
                            continue
                        e = owner(pos)
                        rel = pos - os_[e]
                        if rel < 4:
                            byte = (int(bl[e]) >> (8 * rel)) & 0xFF
                        elif stride:
                            byte = elems[first + e][rel - 4]
                        else:
                            byte = staged[Db + os_[e] - 4 * e + (rel - 4) - pay_lo]
                        out[c * 16 + k] = byte
                        owner_written[c * 16 + k] += 1
    assert (owner_written == 1).all(), "every output byte written exactly once"
    return bytes(out)


@pytest.mark.parametrize("n,maxlen", [(1, 0), (7, 3), (1500, 30), (2100, 100), (3, 200000), (1030, 1)])
def test_k2_model_matches_serialize(n, maxlen):
    rng = np.random.default_rng(n * 7 + maxlen)
    elems = _random_elems(rng, n, maxlen)
    want = serialize_byte_tensor(np.array(elems, dtype=np.object_)).item()
    assert k2_model(elems) == want


def test_k3_model_small_tensor_before_zero_tail():
    """A small tensor followed by megabytes of zero bytes: every zero block is
    ambiguous (chains of 4-byte hops in 4 phases), so blocks far into the
    zeros cannot be resolved -- which must not matter once the wanted
    elements all lie before them."""
    rng = np.random.default_rng(9)
    elems = _random_elems(rng, 3000, 29)
    data = _serialize(elems)
    region = np.concatenate([data, np.zeros(1 << 20, np.uint8)])
    window = ((max(64 * len(elems), 1 << 20) + XB - 1) // XB) * XB
    st, offs, lens = k3_model(region, region.size, window, len(elems))
    assert st == 0
    _, ho, hl = host_index(region, region.size, len(elems))
    np.testing.assert_array_equal(offs, ho)
    np.testing.assert_array_equal(lens, hl)
