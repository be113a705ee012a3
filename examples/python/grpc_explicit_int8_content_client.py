#!/usr/bin/env python3
"""Typed `contents.int_contents` for an INT8 identity model (reference
src/python/examples/grpc_explicit_int8_content_client.py)."""
import argparse
import sys

import grpc
import numpy as np

from tritonclient.grpc import service_pb2, service_pb2_grpc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    ap.add_argument("-m", "--model", default="identity_int8")
    a = ap.parse_args()
    stub = service_pb2_grpc.GRPCInferenceServiceStub(grpc.insecure_channel(a.url))
    md = stub.ModelMetadata(service_pb2.ModelMetadataRequest(name=a.model))
    in_name, out_name = md.inputs[0].name, md.outputs[0].name
    x = np.arange(-8, 8, dtype=np.int8)
    req = service_pb2.ModelInferRequest(model_name=a.model)
    t = req.inputs.add(name=in_name, datatype="INT8", shape=[1, 16])
    t.contents.int_contents[:] = x.tolist()
    req.outputs.add(name=out_name)
    resp = stub.ModelInfer(req)
    out = np.frombuffer(resp.raw_output_contents[0], dtype=np.int8)
    if not np.array_equal(out, x):
        print("error: expected %s got %s" % (x, out))
        sys.exit(1)
    print("PASS: explicit int8 content")


if __name__ == "__main__":
    main()
