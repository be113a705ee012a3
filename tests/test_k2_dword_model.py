"""CPU model of K2's dword-assembled emit (csrc/kernels/bytes.hip,
pk_emit_packed): the same part / tile / mark / max-scan / per-dword formula,
written with numpy and checked against the wire format.  It pins the
algorithm (owner marks, the two-element dword rule, staging window, edge
masks) independently of the GPU; tests/test_kernels_gpu.py checks the kernel.
"""

import numpy as np
import pytest

SPAN, PART, TILE = 1024, 65536, 8192


def _wire(payload, lens):
    from tests.test_kernels_gpu import _pack_ref

    return _pack_ref(payload, lens)


def _emit_model(payload, lens, ob_global, db_global):
    """Emit into a buffer whose byte 0 is at global address ob_global (the
    16-B chunk grid is global); db_global, the payload pointer's alignment,
    only picks vector vs byte staging loads in the kernel."""
    n = lens.size
    total = int(lens.sum()) + 4 * n
    out = np.zeros(total + 64, dtype=np.uint8)
    pstart = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    for b in range(0, (n + SPAN - 1) // SPAN):
        first = b * SPAN
        cnt = min(SPAN, n - first)
        L = lens[first:first + cnt].astype(np.int64)
        o = np.concatenate([[0], np.cumsum(L + 4)])  # local starts, o[cnt] = Lb
        Lb = int(o[cnt])
        ol = np.concatenate([o, [0xFFFFFFFF]])
        ln = np.concatenate([L, [0, 0]])
        Db = int(pstart[first])  # payload start (relative)
        Ob = Db + 4 * first      # output start (relative)
        for q0 in range(0, Lb, PART):
            q1 = min(q0 + PART, Lb)
            ea = int(np.searchsorted(o[:cnt], q0, side="right") - 1)
            c0 = (ob_global + Ob + q0) // 16
            c1 = (ob_global + Ob + q1 + 15) // 16
            for ct in range(c0, c1, TILE // 16):
                base = ct * 16 - ob_global - Ob
                tb0, tb1 = max(base, q0), min(base + TILE, q1)
                mark = np.zeros(TILE // 4, dtype=np.int64)
                ez = None
                for j in range(ea, cnt):
                    oj = int(o[j])
                    if oj >= tb1:
                        break
                    q = max((oj - base + 3) >> 2, 0)
                    if q < TILE // 4:
                        mark[q] = j + 1
                    if oj <= tb1 - 1 < int(o[j + 1]):
                        ez = j
                assert ez is not None
                # staged payload window (global addresses aligned to 16)
                oa, oz = int(o[ea]), int(o[ez])
                pa = oa - 4 * ea + max(tb0 - oa - 4, 0)
                pz = oz - 4 * ez + (tb1 - oz - 4 if tb1 - 1 - oz >= 4 else 0)
                pay_lo = (Db + pa) & ~15  # relative to the payload pointer, as in the kernel
                pay_hi = Db + max(pz, pa)
                nbytes = pay_hi - pay_lo
                assert nbytes <= TILE + 15
                stage = np.zeros(TILE + 64, dtype=np.uint8)
                if nbytes > 0:
                    stage[16:16 + nbytes] = payload[pay_lo:pay_lo + nbytes]
                own = np.maximum.accumulate(np.maximum(mark, ea + 1)) - 1
                pbase = Db - pay_lo + 16
                for qd in range(TILE // 4):
                    u = base + 4 * qd
                    if u + 4 <= tb0 or u >= tb1:
                        continue
                    j = int(own[qd])
                    rel, s = u - int(ol[j]), int(ol[j + 1]) - u
                    if rel < 0:  # j starts inside this dword (a block's or part's first one)
                        w = (int(ln[j]) << (8 * (-rel & 3))) & 0xFFFFFFFF if rel > -4 else 0
                    else:
                        w = (int(ln[j]) >> (8 * (rel & 3))) if rel < 4 else 0
                    w |= ((int(ln[j + 1]) << (8 * (s & 3))) & 0xFFFFFFFF) if s < 4 else 0
                    pix = min(max(pbase + u - 4 * (j + 1), 0), TILE + 56)
                    pv = int.from_bytes(stage[pix:pix + 4].tobytes(), "little")
                    rc, sc = min(max(rel, 0), 4), min(max(s, 0), 4)
                    lo_m = ((0xFFFFFFFFFFFFFFFF << (32 - 8 * rc)) & 0xFFFFFFFF)
                    hi_m = 0xFFFFFFFF >> (32 - 8 * sc)
                    w |= pv & lo_m & hi_m
                    for k in range(4):
                        if tb0 <= u + k < tb1:
                            out[Ob + u + k] = (w >> (8 * k)) & 0xFF
                ea = ez + 1 if int(ol[ez + 1]) <= tb1 else ez
    return out[:total]


@pytest.mark.parametrize("ob,db", [(0, 0), (3, 5), (14, 1)])
def test_dword_model_matches_wire_format(ob, db):
    rng = np.random.default_rng(ob * 11 + db)
    n = 2300
    lens = rng.integers(0, 40, n).astype(np.uint32)
    lens[5] = 9000       # spans a tile
    lens[1500] = 70000   # spans a part
    lens[1024:1100] = 0  # prefix-only run
    payload = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    got = _emit_model(payload, lens, ob, db)
    assert np.array_equal(got, _wire(payload, lens))
