#!/usr/bin/env python3
"""gRPC async_infer with a completion callback (reference
src/python/examples/simple_grpc_async_infer_client.py)."""
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
    ap.add_argument("-t", "--client-timeout", type=float, default=None)
    a = ap.parse_args()
    client = grpcclient.InferenceServerClient(a.url, verbose=a.verbose)
    x = np.arange(16, dtype=np.int32).reshape(1, 16)
    y = np.ones((1, 16), dtype=np.int32)
    inputs = [grpcclient.InferInput("INPUT0", [1, 16], "INT32"), grpcclient.InferInput("INPUT1", [1, 16], "INT32")]
    inputs[0].set_data_from_numpy(x)
    inputs[1].set_data_from_numpy(y)
    done = queue.Queue()
    n = 4
    for i in range(n):
        client.async_infer("simple", inputs, partial(callback, done), request_id=str(i),
                           client_timeout=a.client_timeout)
    for _ in range(n):
        r = done.get(timeout=60)
        if isinstance(r, Exception):
            print("inference failed: " + str(r))
            sys.exit(1)
        if not (np.array_equal(r.as_numpy("OUTPUT0"), x + y) and np.array_equal(r.as_numpy("OUTPUT1"), x - y)):
            print("async infer error: incorrect result")
            sys.exit(1)
    print("PASS: Async infer")


if __name__ == "__main__":
    main()
