#!/usr/bin/env python3
"""Health, server/model metadata and config over HTTP (reference
src/python/examples/simple_http_health_metadata.py)."""
import argparse
import sys

import tritonclient.http as httpclient


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8000")
    a = ap.parse_args()
    c = httpclient.InferenceServerClient(a.url, verbose=a.verbose)
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
    if "name" not in md or "version" not in md:
        print("FAILED : get_server_metadata")
        sys.exit(1)
    print(md)
    mm = c.get_model_metadata("simple", query_params={"test_1": 1, "test_2": 2})
    if mm["name"] != "simple":
        print("FAILED : get_model_metadata")
        sys.exit(1)
    print(mm)
    try:
        c.get_model_metadata("wrong_model_name")
        print("FAILED : get_model_metadata wrong_model_name")
        sys.exit(1)
    except Exception as ex:
        if "Request for unknown model" not in str(ex) and "unknown model" not in str(ex).lower():
            print("FAILED : get_model_metadata wrong_model_name: " + str(ex))
            sys.exit(1)
    cfg = c.get_model_config("simple")
    if cfg["name"] != "simple":
        print("FAILED : get_model_config")
        sys.exit(1)
    print(cfg)
    print("PASS: health, metadata, config")


if __name__ == "__main__":
    main()
