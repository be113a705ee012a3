"""Python concurrency-mode load generator (perf_analyzer ``--concurrency-range``).

Keeps exactly ``concurrency`` requests in flight on one gRPC channel: each
slot re-issues its next request from the completion callback of the previous
one (closed loop), recording per-request latency with a monotonic clock.
Used by bench.py and the pytest GPU tests; the native perf tool
(csrc/perf) is the C++ counterpart.
"""

import threading
import time

import numpy as np


class ConcurrencyRun:
    def __init__(self, client, model_name, inputs, outputs_per_slot, concurrency, model_version=""):
        self.client = client
        self.model_name = model_name
        self.inputs = inputs
        self.outputs_per_slot = outputs_per_slot
        self.concurrency = concurrency
        self.model_version = model_version

    def run(self, requests_per_slot):
        """Issue ``requests_per_slot`` sequential requests on each slot;
        returns (latencies_ns np.array, errors list, wall_seconds)."""
        lat = []
        errors = []
        lock = threading.Lock()
        remaining = [requests_per_slot] * self.concurrency
        done = threading.Event()
        active = [self.concurrency]

        def issue(slot):
            t0 = time.monotonic_ns()

            def cb(result, error, slot=slot, t0=t0):
                t1 = time.monotonic_ns()
                with lock:
                    lat.append(t1 - t0)
                    if error is not None:
                        errors.append(error)
                    remaining[slot] -= 1
                    again = remaining[slot] > 0
                    if not again:
                        active[0] -= 1
                        if active[0] == 0:
                            done.set()
                if again:
                    issue(slot)

            self.client.async_infer(
                self.model_name,
                self.inputs,
                cb,
                model_version=self.model_version,
                outputs=self.outputs_per_slot[slot],
            )

        if requests_per_slot <= 0:
            return np.zeros(0, np.int64), [], 0.0
        w0 = time.monotonic()
        for s in range(self.concurrency):
            issue(s)
        done.wait()
        return np.array(lat, dtype=np.int64), errors, time.monotonic() - w0


def percentile_us(lat_ns, p):
    if len(lat_ns) == 0:
        return 0.0
    return float(np.percentile(lat_ns, p)) / 1000.0
