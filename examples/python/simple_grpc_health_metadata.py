#!/usr/bin/env python3
"""Health, metadata, config and statistics over gRPC (reference
src/python/examples/simple_grpc_health_metadata.py)."""
import argparse
import sys

import tritonclient.grpc as grpcclient


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    a = ap.parse_args()
    c = grpcclient.InferenceServerClient(a.url, verbose=a.verbose)
    if not c.is_server_live(headers={"test": "1", "dummy": "2"}):
        print("FAILED : is_server_live")
        sys.exit(1)
    if not c.is_server_ready():
        print("FAILED : is_server_ready")
        sys.exit(1)
    if not c.is_model_ready("simple"):
        print("FAILED : is_model_ready")
        sys.exit(1)
    md = c.get_server_metadata()
    if not md.name:
        print("FAILED : get_server_metadata")
        sys.exit(1)
    print(md)
    mm = c.get_model_metadata("simple", headers={"test": "1"})
    if mm.name != "simple":
        print("FAILED : get_model_metadata")
        sys.exit(1)
    print(mm)
    try:
        c.get_model_metadata("wrong_model_name")
        print("FAILED : get_model_metadata wrong_model_name")
        sys.exit(1)
    except Exception as ex:
        print("expected error: " + str(ex))
    cfg = c.get_model_config("simple")
    if cfg.config.name != "simple":
        print("FAILED: get_model_config")
        sys.exit(1)
    print(cfg)
    st = c.get_inference_statistics("simple")
    if len(st.model_stats) != 1:
        print("FAILED: get_inference_statistics")
        sys.exit(1)
    print(st)
    print("PASS: health, metadata, config, statistics")


if __name__ == "__main__":
    main()
