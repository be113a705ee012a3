#!/usr/bin/env python3
"""Repeat the HIP-shm BYTES device round trip (K2 pack, K3 index) on one
region many times and count mismatches: K2's output against the host codec's
bytes after every set, K3's element count / offsets against the host walk
after every get.  Reproduces the round-4 bytes_crossover failure (n = 1024,
mean length 20, 200 sets then 200 gets: K3 reported 163 elements).

    python tools/k3_stress.py --n 1024 --reps 300
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="256,1024,4096")
    ap.add_argument("--mean-len", type=int, default=20)
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--crossover-seq", action="store_true",
                    help="replay tools/bytes_crossover.py's exact sequence (sizes 16,64,256,1024, host then device "
                         "paths, same data), printing every step")
    a = ap.parse_args()
    if a.crossover_seq:
        return crossover_seq(a)
    from tritonclient.utils import hip_shared_memory as hipshm
    from tritonclient.utils import serialize_byte_tensor

    rng = np.random.default_rng(0)
    for n in [int(v) for v in a.n.split(",")]:
        lens = rng.integers(0, 2 * a.mean_len + 1, n)
        pool = rng.integers(97, 123, int(lens.sum()) + 1, dtype=np.uint8).tobytes()
        offs = np.concatenate([[0], np.cumsum(lens)])
        data = np.array([pool[offs[i]:offs[i + 1]] for i in range(n)], dtype=np.object_)
        want = serialize_byte_tensor(data).item()
        h = hipshm.create_shared_memory_region("k3s_%d" % n, len(want) + 256, 0)
        bad_set = bad_get = errs = 0
        first = None
        for r in range(a.reps):
            hipshm.set_shared_memory_region(h, [data], serialize_bytes=True, bytes_path="device")
            raw = hipshm.get_contents_as_numpy(h, np.uint8, [len(want)]).tobytes()
            if raw != want:
                bad_set += 1
                if first is None:
                    d = next(i for i in range(len(want)) if raw[i] != want[i])
                    first = {"rep": r, "kind": "k2", "first_diff_byte": d}
            try:
                out = hipshm.get_contents_as_numpy(h, np.object_, [n], bytes_path="device")
                if list(out) != list(data):
                    bad_get += 1
                    first = first or {"rep": r, "kind": "k3 values"}
            except hipshm.CudaSharedMemoryException as e:
                errs += 1
                first = first or {"rep": r, "kind": "k3 error", "msg": str(e)}
        hipshm.destroy_shared_memory_region(h)
        print(json.dumps({"n": n, "bytes": len(want), "reps": a.reps, "k2_mismatch": bad_set, "k3_mismatch": bad_get,
                          "k3_errors": errs, "first": first}), flush=True)


def crossover_seq(a):
    from tritonclient.utils import hip_shared_memory as hipshm
    from tritonclient.utils import serialize_byte_tensor

    rng = np.random.default_rng(0)
    for n in (16, 64, 256, 1024, 4096):
        lens = rng.integers(0, 2 * a.mean_len + 1, n)
        pool = rng.integers(97, 123, int(lens.sum()) + 1, dtype=np.uint8).tobytes()
        offs = np.concatenate([[0], np.cumsum(lens)])
        data = np.array([pool[offs[i]:offs[i + 1]] for i in range(n)], dtype=np.object_)
        want = serialize_byte_tensor(data).item()
        h = hipshm.create_shared_memory_region("xs_%d" % n, len(want) + 256, 0)
        for path in ("host", "device"):
            for r in range(a.reps):
                print("n %d path %s rep %d set" % (n, path, r), flush=True)
                hipshm.set_shared_memory_region(h, [data], serialize_bytes=True, bytes_path=path)
                raw = hipshm.get_contents_as_numpy(h, np.uint8, [len(want)]).tobytes()
                if raw != want:
                    print("SET MISMATCH", n, path, r, flush=True)
                print("n %d path %s rep %d get" % (n, path, r), flush=True)
                out = hipshm.get_contents_as_numpy(h, np.object_, [n], bytes_path=path)
                if list(out) != list(data):
                    print("GET MISMATCH", n, path, r, flush=True)
        hipshm.destroy_shared_memory_region(h)
    print("CROSSOVER_SEQ_DONE", flush=True)


if __name__ == "__main__":
    main()
