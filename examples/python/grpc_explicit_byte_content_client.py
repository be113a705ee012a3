#!/usr/bin/env python3
"""Typed `contents.bytes_contents` BYTES inputs on `simple_string` (reference
src/python/examples/grpc_explicit_byte_content_client.py)."""
import argparse
import sys

import grpc
import numpy as np

from tritonclient.grpc import service_pb2, service_pb2_grpc
from tritonclient.utils import deserialize_bytes_tensor


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    a = ap.parse_args()
    stub = service_pb2_grpc.GRPCInferenceServiceStub(grpc.insecure_channel(a.url))
    vals = list(range(16))
    req = service_pb2.ModelInferRequest(model_name="simple_string")
    t0 = req.inputs.add(name="INPUT0", datatype="BYTES", shape=[1, 16])
    t0.contents.bytes_contents[:] = [str(v).encode() for v in vals]
    t1 = req.inputs.add(name="INPUT1", datatype="BYTES", shape=[1, 16])
    t1.contents.bytes_contents[:] = [b"1"] * 16
    req.outputs.add(name="OUTPUT0")
    req.outputs.add(name="OUTPUT1")
    resp = stub.ModelInfer(req)
    s = deserialize_bytes_tensor(resp.raw_output_contents[0])
    d = deserialize_bytes_tensor(resp.raw_output_contents[1])
    for i, v in enumerate(vals):
        if int(s[i]) != v + 1 or int(d[i]) != v - 1:
            print("error: incorrect result at %d" % i)
            sys.exit(1)
    print("PASS: explicit byte content")


if __name__ == "__main__":
    main()
