#!/usr/bin/env python3
"""Stateful sequences over gRPC with int and string correlation ids
(reference src/python/examples/simple_grpc_sequence_sync_infer_client.py)."""
import argparse
import sys

import numpy as np

import tritonclient.grpc as grpcclient


def step(client, model, value, seq_id, start, end):
    x = grpcclient.InferInput("INPUT", [1, 1], "INT32")
    x.set_data_from_numpy(np.array([[value]], dtype=np.int32))
    r = client.infer(model, [x], sequence_id=seq_id, sequence_start=start, sequence_end=end)
    return int(r.as_numpy("OUTPUT")[0][0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    ap.add_argument("-d", "--dyna", action="store_true", help="use simple_dyna_sequence")
    a = ap.parse_args()
    client = grpcclient.InferenceServerClient(a.url, verbose=a.verbose)
    model = "simple_dyna_sequence" if a.dyna else "simple_sequence"
    values = [11, 7, 5, 3, 2, 0, 1]
    for s0, s1 in ((1000, 1001), ("1000_str", "1001_str")):
        r0 = [step(client, model, 0, s0, True, False)]
        r1 = [step(client, model, 100, s1, True, False)]
        for i, v in enumerate(values):
            end = i == len(values) - 1
            r0.append(step(client, model, v, s0, False, end))
            r1.append(step(client, model, -v, s1, False, end))
        print("sequence %s: %s" % (s0, r0))
        print("sequence %s: %s" % (s1, r1))
        if r0 == r1:
            print("error: sequences interfered")
            sys.exit(1)
    print("PASS: Sequence")


if __name__ == "__main__":
    main()
