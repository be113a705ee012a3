#!/usr/bin/env python3
"""Image classification over raw gRPC stubs (service_pb2), with the
classification extension (reference src/python/examples/grpc_image_client.py)."""
import argparse
import sys

import grpc
import numpy as np

from tritonclient.grpc import service_pb2, service_pb2_grpc
from tritonclient.utils import deserialize_bytes_tensor


def load(path, h, w):
    from image_client import load_image, preprocess

    return preprocess(load_image(path), "NCHW", "FP32", 3, h, w, "INCEPTION")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-m", "--model-name", required=True)
    ap.add_argument("-x", "--model-version", default="")
    ap.add_argument("-b", "--batch-size", type=int, default=1)
    ap.add_argument("-c", "--classes", type=int, default=1)
    ap.add_argument("-u", "--url", default="localhost:8001")
    ap.add_argument("image_filename")
    a = ap.parse_args()
    stub = service_pb2_grpc.GRPCInferenceServiceStub(grpc.insecure_channel(a.url))
    md = stub.ModelMetadata(service_pb2.ModelMetadataRequest(name=a.model_name, version=a.model_version))
    cfg = stub.ModelConfig(service_pb2.ModelConfigRequest(name=a.model_name, version=a.model_version)).config
    inp, out = md.inputs[0], md.outputs[0]
    c, h, w = list(inp.shape)[-3:]
    img = load(a.image_filename, h, w)
    batch = np.stack([img] * a.batch_size) if cfg.max_batch_size > 0 else img
    req = service_pb2.ModelInferRequest(model_name=a.model_name, model_version=a.model_version)
    t = req.inputs.add(name=inp.name, datatype=inp.datatype, shape=list(batch.shape))
    req.raw_input_contents.append(batch.astype(np.float32).tobytes())
    o = req.outputs.add(name=out.name)
    o.parameters["classification"].int64_param = a.classes
    del t
    resp = stub.ModelInfer(req)
    labels = deserialize_bytes_tensor(resp.raw_output_contents[0])
    if len(labels) != a.batch_size * a.classes:
        print("error: expected %d classes, got %d" % (a.batch_size * a.classes, len(labels)))
        sys.exit(1)
    for s in labels:
        print("    " + s.decode())
    print("PASS")


if __name__ == "__main__":
    main()
