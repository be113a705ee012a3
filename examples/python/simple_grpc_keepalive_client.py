#!/usr/bin/env python3
"""gRPC client with custom keepalive options (reference
src/python/examples/simple_grpc_keepalive_client.py)."""
import argparse
import sys

import numpy as np

import tritonclient.grpc as grpcclient


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    ap.add_argument("--grpc-keepalive-time", type=int, default=2**31 - 1)
    ap.add_argument("--grpc-keepalive-timeout", type=int, default=20000)
    ap.add_argument("--grpc-keepalive-permit-without-calls", action="store_true")
    ap.add_argument("--grpc-http2-max-pings-without-data", type=int, default=2)
    a = ap.parse_args()
    ka = grpcclient.KeepAliveOptions(keepalive_time_ms=a.grpc_keepalive_time,
                                     keepalive_timeout_ms=a.grpc_keepalive_timeout,
                                     keepalive_permit_without_calls=a.grpc_keepalive_permit_without_calls,
                                     http2_max_pings_without_data=a.grpc_http2_max_pings_without_data)
    c = grpcclient.InferenceServerClient(a.url, verbose=a.verbose, keepalive_options=ka)
    x = np.arange(16, dtype=np.int32).reshape(1, 16)
    y = np.ones((1, 16), dtype=np.int32)
    inputs = [grpcclient.InferInput("INPUT0", [1, 16], "INT32"), grpcclient.InferInput("INPUT1", [1, 16], "INT32")]
    inputs[0].set_data_from_numpy(x)
    inputs[1].set_data_from_numpy(y)
    r = c.infer("simple", inputs)
    if not (np.array_equal(r.as_numpy("OUTPUT0"), x + y) and np.array_equal(r.as_numpy("OUTPUT1"), x - y)):
        print("keepalive infer error: incorrect result")
        sys.exit(1)
    print("PASS: KeepAlive")


if __name__ == "__main__":
    main()
