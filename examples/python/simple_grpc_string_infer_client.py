#!/usr/bin/env python3
"""BYTES tensors over gRPC on `simple_string` (reference
src/python/examples/simple_grpc_string_infer_client.py)."""
import argparse
import sys

import numpy as np

import tritonclient.grpc as grpcclient


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    a = ap.parse_args()
    client = grpcclient.InferenceServerClient(a.url, verbose=a.verbose)
    in0 = np.arange(16, dtype=np.int32)
    x = np.array([str(v) for v in in0], dtype=np.object_).reshape(1, 16)
    y = np.array(["1"] * 16, dtype=np.object_).reshape(1, 16)
    inputs = [grpcclient.InferInput("INPUT0", [1, 16], "BYTES"), grpcclient.InferInput("INPUT1", [1, 16], "BYTES")]
    inputs[0].set_data_from_numpy(x)
    inputs[1].set_data_from_numpy(y)
    r = client.infer("simple_string", inputs, outputs=[grpcclient.InferRequestedOutput("OUTPUT0"),
                                                       grpcclient.InferRequestedOutput("OUTPUT1")])
    s, d = r.as_numpy("OUTPUT0"), r.as_numpy("OUTPUT1")
    for i in range(16):
        print("%d + 1 = %s" % (in0[i], s[0][i].decode()))
        print("%d - 1 = %s" % (in0[i], d[0][i].decode()))
        if int(s[0][i]) != in0[i] + 1 or int(d[0][i]) != in0[i] - 1:
            print("error: incorrect result")
            sys.exit(1)
    print("PASS: string")


if __name__ == "__main__":
    main()
