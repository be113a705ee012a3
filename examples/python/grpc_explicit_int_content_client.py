#!/usr/bin/env python3
"""Typed `contents.int_contents` inputs instead of raw bytes, including one
raw and one typed input in the same request (reference
src/python/examples/grpc_explicit_int_content_client.py)."""
import argparse
import sys

import grpc
import numpy as np

from tritonclient.grpc import service_pb2, service_pb2_grpc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    a = ap.parse_args()
    stub = service_pb2_grpc.GRPCInferenceServiceStub(grpc.insecure_channel(a.url))
    x = np.arange(16, dtype=np.int32)
    y = np.ones(16, dtype=np.int32)
    for mixed in (False, True):
        req = service_pb2.ModelInferRequest(model_name="simple")
        t0 = req.inputs.add(name="INPUT0", datatype="INT32", shape=[1, 16])
        t0.contents.int_contents[:] = x.tolist()
        t1 = req.inputs.add(name="INPUT1", datatype="INT32", shape=[1, 16])
        if mixed:
            req.raw_input_contents.append(y.tobytes())
        else:
            t1.contents.int_contents[:] = y.tolist()
        req.outputs.add(name="OUTPUT0")
        req.outputs.add(name="OUTPUT1")
        resp = stub.ModelInfer(req)
        s = np.frombuffer(resp.raw_output_contents[0], dtype=np.int32)
        d = np.frombuffer(resp.raw_output_contents[1], dtype=np.int32)
        if not (np.array_equal(s, x + y) and np.array_equal(d, x - y)):
            print("error: incorrect result (mixed=%s)" % mixed)
            sys.exit(1)
    print("PASS: explicit int content")


if __name__ == "__main__":
    main()
