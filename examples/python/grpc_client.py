#!/usr/bin/env python3
"""Raw gRPC stubs (service_pb2 / service_pb2_grpc) without the client class
(reference src/python/examples/grpc_client.py)."""
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
    channel = grpc.insecure_channel(a.url)
    stub = service_pb2_grpc.GRPCInferenceServiceStub(channel)
    print(stub.ServerLive(service_pb2.ServerLiveRequest()))
    print(stub.ServerReady(service_pb2.ServerReadyRequest()))
    print(stub.ModelReady(service_pb2.ModelReadyRequest(name="simple", version="")))
    print(stub.ServerMetadata(service_pb2.ServerMetadataRequest()))
    print(stub.ModelMetadata(service_pb2.ModelMetadataRequest(name="simple", version="")))
    print(stub.ModelConfig(service_pb2.ModelConfigRequest(name="simple", version="")))
    req = service_pb2.ModelInferRequest(model_name="simple", model_version="", id="my request id")
    x = np.arange(16, dtype=np.int32)
    y = np.ones(16, dtype=np.int32)
    for name, arr in (("INPUT0", x), ("INPUT1", y)):
        t = service_pb2.ModelInferRequest().InferInputTensor(name=name, datatype="INT32", shape=[1, 16])
        req.inputs.extend([t])
        req.raw_input_contents.append(arr.tobytes())
    for name in ("OUTPUT0", "OUTPUT1"):
        req.outputs.extend([service_pb2.ModelInferRequest().InferRequestedOutputTensor(name=name)])
    resp = stub.ModelInfer(req)
    print("model infer:", resp.model_name, resp.id)
    s = np.frombuffer(resp.raw_output_contents[0], dtype=np.int32)
    d = np.frombuffer(resp.raw_output_contents[1], dtype=np.int32)
    if not (np.array_equal(s, x + y) and np.array_equal(d, x - y)):
        print("error: incorrect result")
        sys.exit(1)
    print("PASS: grpc_client")


if __name__ == "__main__":
    main()
