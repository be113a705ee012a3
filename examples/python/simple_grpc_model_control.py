#!/usr/bin/env python3
"""Model repository control over gRPC, including a load with file override
(reference src/python/examples/simple_grpc_model_control.py)."""
import argparse
import json
import sys

import tritonclient.grpc as grpcclient
from tritonclient.utils import InferenceServerException


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    a = ap.parse_args()
    c = grpcclient.InferenceServerClient(a.url, verbose=a.verbose)
    model = "simple"
    print(c.get_model_repository_index())
    c.unload_model(model)
    if c.is_model_ready(model):
        print("FAILED : unload_model")
        sys.exit(1)
    c.load_model(model)
    if not c.is_model_ready(model):
        print("FAILED : load_model")
        sys.exit(1)
    try:
        c.load_model("wrong_model_name")
        print("FAILED : load_model wrong_model_name")
        sys.exit(1)
    except InferenceServerException as e:
        print("expected error: " + e.message())
    # load a new model name from an override config + model file ("tcamd-model:<builtin>"
    # names the builtin implementation, the framework's model-file format)
    cfg = json.dumps({"backend": "onnxruntime", "max_batch_size": 8})
    c.load_model("simple_override", config=cfg, files={"file:1/model.onnx": b"tcamd-model:simple"})
    if not c.is_model_ready("simple_override", "1"):
        print("FAILED : load_model with override files")
        sys.exit(1)
    c.unload_model("simple_override")
    print("PASS: model control")


if __name__ == "__main__":
    main()
