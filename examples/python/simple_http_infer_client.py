#!/usr/bin/env python3
"""Sync HTTP inference on `simple` (INT32 add/sub), with binary and JSON
outputs and optional gzip/deflate (reference src/python/examples/simple_http_infer_client.py)."""
import argparse
import sys

import numpy as np

import tritonclient.http as httpclient
from tritonclient.utils import InferenceServerException


def run(client, model, compression=None, binary_out=True):
    a = np.arange(16, dtype=np.int32).reshape(1, 16)
    b = np.ones((1, 16), dtype=np.int32)
    inputs = [httpclient.InferInput("INPUT0", [1, 16], "INT32"), httpclient.InferInput("INPUT1", [1, 16], "INT32")]
    inputs[0].set_data_from_numpy(a, binary_data=False)
    inputs[1].set_data_from_numpy(b, binary_data=True)
    outputs = [httpclient.InferRequestedOutput("OUTPUT0", binary_data=binary_out),
               httpclient.InferRequestedOutput("OUTPUT1", binary_data=False)]
    r = client.infer(model, inputs, outputs=outputs, query_params={"test_1": 1, "test_2": 2},
                     request_compression_algorithm=compression, response_compression_algorithm=compression)
    s, d = r.as_numpy("OUTPUT0"), r.as_numpy("OUTPUT1")
    for i in range(16):
        print("%d + %d = %d" % (a[0][i], b[0][i], s[0][i]))
        print("%d - %d = %d" % (a[0][i], b[0][i], d[0][i]))
        if a[0][i] + b[0][i] != s[0][i] or a[0][i] - b[0][i] != d[0][i]:
            print("error: incorrect result")
            sys.exit(1)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8000")
    ap.add_argument("-s", "--ssl", action="store_true")
    ap.add_argument("--key-file", default=None)
    ap.add_argument("--cert-file", default=None)
    ap.add_argument("--ca-certs", default=None)
    ap.add_argument("--insecure", action="store_true")
    ap.add_argument("-C", "--compression-algorithm", choices=["deflate", "gzip"], default=None)
    a = ap.parse_args()
    try:
        client = httpclient.InferenceServerClient(a.url, verbose=a.verbose, ssl=a.ssl,
                                                  ssl_options={"keyfile": a.key_file, "certfile": a.cert_file,
                                                               "ca_certs": a.ca_certs} if a.ssl else None,
                                                  insecure=a.insecure)
    except Exception as e:
        print("channel creation failed: " + str(e))
        sys.exit(1)
    run(client, "simple", a.compression_algorithm)
    run(client, "simple", a.compression_algorithm, binary_out=False)
    try:
        run(client, "not_a_model")
        print("expected an error for an unknown model")
        sys.exit(1)
    except InferenceServerException as e:
        print("expected error: " + e.message())
    print("PASS: infer")


if __name__ == "__main__":
    main()
