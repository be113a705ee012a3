#!/usr/bin/env python3
"""Model repository control over HTTP: index, unload, load, config override
(reference src/python/examples/simple_http_model_control.py)."""
import argparse
import json
import sys

import tritonclient.http as httpclient
from tritonclient.utils import InferenceServerException


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8000")
    a = ap.parse_args()
    c = httpclient.InferenceServerClient(a.url, verbose=a.verbose)
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
    # reload with a config override
    cfg = c.get_model_config(model)
    c.load_model(model, config=json.dumps({"max_batch_size": cfg.get("max_batch_size", 0),
                                           "version_policy": {"latest": {"num_versions": 1}}}))
    if not c.is_model_ready(model):
        print("FAILED : load_model with config")
        sys.exit(1)
    c.unload_model(model, unload_dependents=True)
    c.load_model(model)
    print("PASS: model control")


if __name__ == "__main__":
    main()
