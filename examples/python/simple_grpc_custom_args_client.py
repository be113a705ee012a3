#!/usr/bin/env python3
"""gRPC client with raw channel arguments instead of the defaults (reference
src/python/examples/simple_grpc_custom_args_client.py)."""
import argparse
import sys

import numpy as np

import tritonclient.grpc as grpcclient


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    a = ap.parse_args()
    channel_args = [("grpc.max_send_message_length", 2**31 - 1), ("grpc.max_receive_message_length", 2**31 - 1),
                    ("grpc.keepalive_time_ms", 2**31 - 1), ("grpc.lb_policy_name", "pick_first")]
    c = grpcclient.InferenceServerClient(a.url, verbose=a.verbose, channel_args=channel_args)
    x = np.arange(16, dtype=np.int32).reshape(1, 16)
    y = np.ones((1, 16), dtype=np.int32)
    inputs = [grpcclient.InferInput("INPUT0", [1, 16], "INT32"), grpcclient.InferInput("INPUT1", [1, 16], "INT32")]
    inputs[0].set_data_from_numpy(x)
    inputs[1].set_data_from_numpy(y)
    r = c.infer("simple", inputs)
    if not (np.array_equal(r.as_numpy("OUTPUT0"), x + y) and np.array_equal(r.as_numpy("OUTPUT1"), x - y)):
        print("custom args infer error: incorrect result")
        sys.exit(1)
    print("PASS: custom args")


if __name__ == "__main__":
    main()
