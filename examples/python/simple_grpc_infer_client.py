#!/usr/bin/env python3
"""Sync gRPC inference on `simple` with SSL/compression/timeout options
(reference src/python/examples/simple_grpc_infer_client.py)."""
import argparse
import sys

import numpy as np

import tritonclient.grpc as grpcclient
from tritonclient.utils import InferenceServerException


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    ap.add_argument("-s", "--ssl", action="store_true")
    ap.add_argument("-t", "--client-timeout", type=float, default=None)
    ap.add_argument("-r", "--root-certificates", default=None)
    ap.add_argument("-p", "--private-key", default=None)
    ap.add_argument("-x", "--certificate-chain", default=None)
    ap.add_argument("-C", "--grpc-compression-algorithm", choices=["deflate", "gzip"], default=None)
    a = ap.parse_args()
    try:
        client = grpcclient.InferenceServerClient(a.url, verbose=a.verbose, ssl=a.ssl,
                                                  root_certificates=a.root_certificates,
                                                  private_key=a.private_key, certificate_chain=a.certificate_chain)
    except Exception as e:
        print("channel creation failed: " + str(e))
        sys.exit(1)
    x = np.arange(16, dtype=np.int32).reshape(1, 16)
    y = np.ones((1, 16), dtype=np.int32)
    inputs = [grpcclient.InferInput("INPUT0", [1, 16], "INT32"), grpcclient.InferInput("INPUT1", [1, 16], "INT32")]
    inputs[0].set_data_from_numpy(x)
    inputs[1].set_data_from_numpy(y)
    outputs = [grpcclient.InferRequestedOutput("OUTPUT0"), grpcclient.InferRequestedOutput("OUTPUT1")]
    try:
        r = client.infer("simple", inputs, outputs=outputs, client_timeout=a.client_timeout,
                         headers={"test": "1"}, compression_algorithm=a.grpc_compression_algorithm)
    except InferenceServerException as e:
        if "Deadline" in str(e) or "DEADLINE" in str(e):
            print("deadline exceeded: " + str(e))
            sys.exit(1)
        raise
    print(r.get_response())
    s, d = r.as_numpy("OUTPUT0"), r.as_numpy("OUTPUT1")
    for i in range(16):
        print("%d + %d = %d" % (x[0][i], y[0][i], s[0][i]))
        print("%d - %d = %d" % (x[0][i], y[0][i], d[0][i]))
        if x[0][i] + y[0][i] != s[0][i] or x[0][i] - y[0][i] != d[0][i]:
            print("sync infer error: incorrect result")
            sys.exit(1)
    print("PASS: infer")


if __name__ == "__main__":
    main()
