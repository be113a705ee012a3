"""tcserve's dynamic-batcher dispatch rules (csrc/cpp/server/batch_policy.h)
under scripted arrivals, through tcserve_batch_policy_sim: the same two
functions the threaded batcher runs (Server::Worker), driven by a
discrete-event simulation, so batch composition and start spacing are exact.

Rules covered: preferred-size batches go at once; otherwise the queue delay
from the oldest request; idle-aware dispatch; pipelined dispatch of partial
batches; staggered starts of full batches on several instances; the take
limit (largest preferred size the queue fills, whole requests, FIFO); and, in
the closed-loop simulator, how a loop of one-row clients settles into groups."""

import ctypes
import os

import numpy as np
import pytest

from triton_client_amd.server import native_frontend

pytestmark = pytest.mark.skipif(not os.path.exists(native_frontend.LIB_PATH), reason="libtcserve not built")

US = 1000
IDLE, PIPE, STAGGER = 1, 2, 4


def sim(arrivals, rows, max_batch=128, delay_us=2000, preferred=(), instances=1, flags=IDLE | STAGGER,
        exec_base_us=1000, exec_per_row_us=0):
    lib = ctypes.CDLL(native_frontend.LIB_PATH)
    f = lib.tcserve_batch_policy_sim
    f.restype = ctypes.c_int32
    n = len(arrivals)
    a = np.ascontiguousarray(np.asarray(arrivals, np.uint64) * US)
    r = np.ascontiguousarray(np.asarray(rows, np.int32))
    pref = np.ascontiguousarray(np.asarray(preferred, np.int32))
    cap = n + 1
    st, nr, first, inst = (np.zeros(cap, np.uint64), np.zeros(cap, np.int32), np.zeros(cap, np.int32),
                           np.zeros(cap, np.int32))
    P = ctypes.c_void_p
    nb = f(ctypes.c_int32(max_batch), ctypes.c_uint64(delay_us * US), P(pref.ctypes.data if len(pref) else 0),
           ctypes.c_int32(len(pref)), ctypes.c_int32(instances), ctypes.c_int32(flags), P(a.ctypes.data),
           P(r.ctypes.data), ctypes.c_int32(n), ctypes.c_uint64(exec_base_us * US),
           ctypes.c_uint64(exec_per_row_us * US), P(st.ctypes.data), P(nr.ctypes.data), P(first.ctypes.data),
           P(inst.ctypes.data), ctypes.c_int32(cap))
    assert nb >= 0, nb
    return [dict(start_us=int(st[i]) // US, rows=int(nr[i]), first=int(first[i]), instance=int(inst[i]))
            for i in range(nb)]


def test_lone_request_on_idle_gpu_goes_now_and_without_idle_rule_waits_the_delay():
    b = sim([0], [8])
    assert b == [dict(start_us=0, rows=8, first=0, instance=0)]
    b = sim([0], [8], flags=0)
    assert b[0]["start_us"] == 2000  # the whole queue delay


def test_preferred_batch_dispatches_at_once_while_busy():
    # instance busy from t=0 (first request, 1 ms); 16 x 8 rows arrive at t=100 us:
    # the queue reaches the preferred 128 rows, so no delay; but with one
    # instance it starts when the instance frees (t=1000)
    arr = [0] + [100] * 16
    b = sim(arr, [8] * 17, preferred=(128,))
    assert [x["rows"] for x in b] == [8, 128]
    assert b[1]["start_us"] == 1000 and b[1]["first"] == 1


def test_partial_batch_waits_for_the_delay_from_the_oldest_request():
    # two instances; one is busy (exec 5 ms), 3 requests queue at t=10..30 us:
    # nothing fills 128 rows, no pipelining -> they go at oldest arrival + 2 ms
    arr = [0, 10, 20, 30]
    b = sim(arr, [8] * 4, preferred=(128,), instances=2, exec_base_us=5000)
    assert b[0]["rows"] == 8 and b[0]["start_us"] == 0
    assert b[1]["rows"] == 24 and b[1]["start_us"] == 10 + 2000 and b[1]["instance"] == 1


def test_take_limit_is_the_largest_preferred_size_the_queue_fills():
    # one instance busy 3 ms; 20 x 8-row requests queue; preferred {64, 128}:
    # first batch takes 128 (16 requests), the rest (32 rows) waits
    arr = [0] + [50] * 20
    b = sim(arr, [8] * 21, preferred=(64, 128), exec_base_us=3000)
    assert [x["rows"] for x in b] == [8, 128, 32]
    assert b[1]["first"] == 1 and b[2]["first"] == 17
    # whole requests only, FIFO: 5 + 5 + 5 rows under a cap of 12 -> 10, then 5
    b = sim([0, 1, 2, 3], [4, 5, 5, 5], max_batch=12, exec_base_us=3000)
    assert [x["rows"] for x in b] == [4, 10, 5]


def test_pipelined_dispatch_goes_once_the_queue_holds_the_last_batch_rows():
    # bs1 closed-loop shape: 2 instances, the first batch carried 4 rows; while
    # instance 0 runs, 4 more single-row requests arrive at t=100..400 us
    arr = [0, 0, 0, 0, 100, 200, 300, 400]
    common = dict(preferred=(128,), instances=2, exec_base_us=2000)
    off = sim(arr, [1] * 8, flags=IDLE, **common)
    on = sim(arr, [1] * 8, flags=IDLE | PIPE, **common)
    # without pipelining the partial queue waits (its delay would end at
    # 100 + 2000) until instance 0 frees at 2000 and the idle rule sends it
    assert off[1]["start_us"] == 2000
    # pipelined: as soon as 4 rows are queued (t=400) the free instance takes them
    assert on[1]["start_us"] == 400 and on[1]["rows"] == 4 and on[1]["instance"] == 1


def test_staggered_starts_of_full_batches():
    # a saturated closed loop: a backlog of 12 full batches at t=0 on 2
    # instances (4 ms each).  Without stagger both instances start together
    # every 4 ms (a request that just misses a start waits a whole execution:
    # bimodal latency); with it, once the EMA is known, starts are spaced by
    # ema / instances = 2 ms while the other instance is busy
    n = 16 * 12
    arr = [0] * n
    b_on = sim(arr, [8] * n, preferred=(128,), instances=2, exec_base_us=4000, flags=IDLE | STAGGER)
    b_off = sim(arr, [8] * n, preferred=(128,), instances=2, exec_base_us=4000, flags=IDLE)
    for b in (b_on, b_off):
        assert len(b) == 12 and all(x["rows"] == 128 for x in b)
        assert sum(x["rows"] for x in b) == 8 * n
        firsts = [x["first"] for x in b]
        assert firsts == sorted(firsts) and firsts[0] == 0
    starts_off = [x["start_us"] for x in b_off]
    assert starts_off[:4] == [0, 0, 4000, 4000]
    starts_on = [x["start_us"] for x in b_on]
    assert starts_on[:4] == [0, 0, 4000, 6000]
    assert (np.diff(starts_on[3:]) == 2000).all(), starts_on


def test_stagger_never_delays_a_partial_batch_or_an_idle_gpu():
    # partial batch with another instance busy: the stagger rule does not apply
    b = sim([0, 0, 100], [128, 8, 8], preferred=(128,), instances=2, exec_base_us=4000, delay_us=50)
    assert b[0]["rows"] == 128 and b[1]["start_us"] == 0 + 50 and b[1]["rows"] == 8
    # nothing busy: a full batch goes now whatever the last start
    b = sim([0, 5000], [128, 128], preferred=(128,), instances=2, exec_base_us=1000)
    assert b[1]["start_us"] == 5000


def test_bad_arguments_are_rejected():
    lib = ctypes.CDLL(native_frontend.LIB_PATH)
    f = lib.tcserve_batch_policy_sim
    f.restype = ctypes.c_int32
    a = np.array([0], np.uint64)
    r = np.array([300], np.int32)  # more rows than max_batch
    out = np.zeros(4, np.uint64)
    o32 = np.zeros(4, np.int32)
    P = ctypes.c_void_p
    assert f(128, 0, P(0), 0, 1, 1, P(a.ctypes.data), P(r.ctypes.data), 1, 0, 0, P(out.ctypes.data),
             P(o32.ctypes.data), P(o32.ctypes.data), P(o32.ctypes.data), 4) == -1


def sim_closed(flags, clients=64, instances=2, exec_base_us=1600, exec_per_row_us=3, turnaround_us=150,
               spacing_us=4, spread_us=10, horizon_us=100000, max_batch=128, delay_us=2000):
    """tcserve_batch_policy_sim_closed: a closed loop of ``clients`` one-row
    requests (each client re-sends ``turnaround_us`` after its batch ends, the
    j-th response ``j * spacing_us`` later)."""
    lib = ctypes.CDLL(native_frontend.LIB_PATH)
    f = lib.tcserve_batch_policy_sim_closed
    f.restype = ctypes.c_int32
    cap = 20000
    st, nr, inst = np.zeros(cap, np.uint64), np.zeros(cap, np.int32), np.zeros(cap, np.int32)
    P, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32
    nb = f(i32(max_batch), u64(delay_us * US), P(0), i32(0), i32(instances), i32(flags), i32(clients), i32(1),
           u64(spread_us * US), u64(turnaround_us * US), u64(spacing_us * US), u64(exec_base_us * US),
           u64(exec_per_row_us * US), u64(horizon_us * US), P(st.ctypes.data), P(nr.ctypes.data), P(inst.ctypes.data),
           i32(cap))
    assert nb > 0, nb
    return [dict(start_us=int(st[i]) // US, rows=int(nr[i]), instance=int(inst[i])) for i in range(nb)]


def test_closed_loop_pipelined_settles_into_one_group_per_instance():
    # bs1 at concurrency 64 on 2 instances: with pipelined dispatch the loop
    # splits into two groups of 32 that alternate between the instances (each
    # returning group is taken as soon as it is back); with the idle rule
    # alone, one instance takes almost everything and the other idles
    tail = [b for b in sim_closed(IDLE | PIPE) if b["start_us"] > 50000]
    assert {b["rows"] for b in tail} == {32}
    assert all(x["instance"] != y["instance"] for x, y in zip(tail, tail[1:]))
    idle = [b for b in sim_closed(IDLE) if b["start_us"] > 50000]
    assert {b["instance"] for b in idle} == {0} and max(b["rows"] for b in idle) == 63
    # rows served per ms of the steady state
    rate = lambda bs: sum(b["rows"] for b in bs) / (bs[-1]["start_us"] - bs[0]["start_us"]) * 1000  # noqa: E731
    assert rate(tail) > 1.3 * rate(idle)


def test_closed_loop_rejects_bad_arguments():
    lib = ctypes.CDLL(native_frontend.LIB_PATH)
    f = lib.tcserve_batch_policy_sim_closed
    f.restype = ctypes.c_int32
    buf = np.zeros(4, np.uint64)
    P, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32
    args = [i32(8), u64(0), P(0), i32(0), i32(1), i32(IDLE), i32(4), i32(1), u64(0), u64(0), u64(0), u64(US), u64(0),
            u64(100 * US), P(buf.ctypes.data), P(buf.ctypes.data), P(buf.ctypes.data)]
    assert f(*args, i32(1)) == -2  # more batches than the output holds
    bad = list(args)
    bad[7] = i32(9)  # rows per request above max_batch
    assert f(*bad, i32(4)) == -1
