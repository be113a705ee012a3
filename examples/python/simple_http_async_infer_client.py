#!/usr/bin/env python3
"""HTTP async_infer: several requests in flight, results collected with
get_result() (reference src/python/examples/simple_http_async_infer_client.py)."""
import argparse
import sys

import numpy as np

import tritonclient.http as httpclient


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8000")
    a = ap.parse_args()
    client = httpclient.InferenceServerClient(a.url, verbose=a.verbose, concurrency=4)
    x = np.arange(16, dtype=np.int32).reshape(1, 16)
    y = np.ones((1, 16), dtype=np.int32)
    inputs = [httpclient.InferInput("INPUT0", [1, 16], "INT32"), httpclient.InferInput("INPUT1", [1, 16], "INT32")]
    inputs[0].set_data_from_numpy(x, binary_data=False)
    inputs[1].set_data_from_numpy(y, binary_data=True)
    outputs = [httpclient.InferRequestedOutput("OUTPUT0", binary_data=True),
               httpclient.InferRequestedOutput("OUTPUT1", binary_data=True)]
    pending = [client.async_infer("simple", inputs, outputs=outputs, request_id=str(i)) for i in range(4)]
    for i, req in enumerate(pending):
        r = req.get_result()
        assert r.get_response()["id"] == str(i)
        s, d = r.as_numpy("OUTPUT0"), r.as_numpy("OUTPUT1")
        if not (np.array_equal(s, x + y) and np.array_equal(d, x - y)):
            print("async infer error: incorrect result")
            sys.exit(1)
    print("PASS: Async infer")


if __name__ == "__main__":
    main()
