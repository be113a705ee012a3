"""Per-rank port stripes of the bench-server harness (bench.py with N ranks)."""

import socket

from triton_client_amd.perf import harness


def test_free_ports_distinct_and_striped():
    a = harness.free_ports(2, 0)
    b = harness.free_ports(2, 1)
    assert len(set(a)) == 2 and len(set(b)) == 2
    assert all(harness.STRIPE_BASE <= p < harness.STRIPE_BASE + harness.STRIPE_WIDTH for p in a)
    assert all(harness.STRIPE_BASE + harness.STRIPE_WIDTH <= p < harness.STRIPE_BASE + 2 * harness.STRIPE_WIDTH
               for p in b)


def test_free_ports_skips_taken_port():
    first = harness.free_ports(1, 5)[0]
    s = socket.socket()
    s.bind(("127.0.0.1", first))
    s.listen(1)
    try:
        got = harness.free_ports(2, 5)
        assert first not in got and len(set(got)) == 2
    finally:
        s.close()
