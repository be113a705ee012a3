#!/usr/bin/env python3
"""HIP-shm BYTES set / get: host codec path against the device kernels (K2
pack, K3 index) from 16 to 1e6 elements, mean string length --mean-len.
Both paths interleaved per round in one process; median of the rounds.

    python tools/bytes_crossover.py --sizes 16,64,256,1024,4096,16384,65536,262144,1000000
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="16,64,256,1024,4096,16384,65536,262144,1000000")
    ap.add_argument("--mean-len", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    from tritonclient.utils import hip_shared_memory as hipshm
    from tritonclient.utils import serialize_byte_tensor

    rng = np.random.default_rng(0)
    for n in [int(v) for v in a.sizes.split(",")]:
        lens = rng.integers(0, 2 * a.mean_len + 1, n)
        pool = rng.integers(97, 123, int(lens.sum()) + 1, dtype=np.uint8).tobytes()
        offs = np.concatenate([[0], np.cumsum(lens)])
        data = np.array([pool[offs[i]:offs[i + 1]] for i in range(n)], dtype=np.object_)
        nbytes = len(serialize_byte_tensor(data).item())
        h = hipshm.create_shared_memory_region("xover_%d" % n, nbytes + 256, 0)
        t = {"set_host": [], "set_device": [], "get_host": [], "get_device": []}
        reps = max(1, min(200, 20000 // max(1, n // 64)))
        errors = []
        for _ in range(a.rounds):
            for path in ("host", "device"):
                try:
                    t0 = time.perf_counter()
                    for _ in range(reps):
                        hipshm.set_shared_memory_region(h, [data], serialize_bytes=True, bytes_path=path)
                    t["set_" + path].append((time.perf_counter() - t0) / reps)
                    t0 = time.perf_counter()
                    for _ in range(reps):
                        out = hipshm.get_contents_as_numpy(h, np.object_, [n], bytes_path=path)
                    t["get_" + path].append((time.perf_counter() - t0) / reps)
                    if list(out) != list(data):
                        errors.append("%s: values differ" % path)
                except hipshm.CudaSharedMemoryException as e:
                    errors.append("%s: %s" % (path, e))
        hipshm.destroy_shared_memory_region(h)
        row = {"n": n, "bytes": nbytes}
        for k, v in t.items():
            row[k + "_us"] = round(sorted(v)[len(v) // 2] * 1e6, 1) if v else None
        if row["set_host_us"] and row["set_device_us"]:
            row["set_faster"] = "host" if row["set_host_us"] < row["set_device_us"] else "device"
        if row["get_host_us"] and row["get_device_us"]:
            row["get_faster"] = "host" if row["get_host_us"] < row["get_device_us"] else "device"
        if errors:
            row["errors"] = errors[:4]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
