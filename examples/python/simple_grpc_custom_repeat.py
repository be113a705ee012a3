#!/usr/bin/env python3
"""Decoupled model `repeat_int32`: one request, many streamed responses
(reference src/python/examples/simple_grpc_custom_repeat.py)."""
import argparse
import queue
import sys
from functools import partial

import numpy as np

import tritonclient.grpc as grpcclient


def callback(user_data, result, error):
    user_data.put(error if error else result)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    ap.add_argument("-r", "--repetitions", type=int, default=4)
    a = ap.parse_args()
    values = np.arange(a.repetitions, dtype=np.int32)
    delays = np.zeros(a.repetitions, dtype=np.uint32)
    q = queue.Queue()
    with grpcclient.InferenceServerClient(a.url, verbose=a.verbose) as client:
        client.start_stream(callback=partial(callback, q))
        inputs = [grpcclient.InferInput("IN", [a.repetitions], "INT32"),
                  grpcclient.InferInput("DELAY", [a.repetitions], "UINT32"),
                  grpcclient.InferInput("WAIT", [1], "UINT32")]
        inputs[0].set_data_from_numpy(values)
        inputs[1].set_data_from_numpy(delays)
        inputs[2].set_data_from_numpy(np.array([0], dtype=np.uint32))
        client.async_stream_infer("repeat_int32", inputs, request_id="0")
        got = []
        for _ in range(a.repetitions):
            r = q.get(timeout=60)
            if isinstance(r, Exception):
                print("error: " + str(r))
                sys.exit(1)
            got.append(int(r.as_numpy("OUT")[0]))
        client.stop_stream()
    if sorted(got) != list(values):
        print("error: expected %s, got %s" % (list(values), got))
        sys.exit(1)
    print("PASS: repeat_int32 (%d responses)" % len(got))


if __name__ == "__main__":
    main()
