#!/usr/bin/env python3
"""BYTES tensors over HTTP: `simple_string` adds/subtracts numbers carried as
strings (reference src/python/examples/simple_http_string_infer_client.py)."""
import argparse
import sys

import numpy as np

import tritonclient.http as httpclient


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8000")
    a = ap.parse_args()
    client = httpclient.InferenceServerClient(a.url, verbose=a.verbose)
    in0 = np.arange(16, dtype=np.int32)
    x = np.array([str(v).encode("utf-8") for v in in0], dtype=np.object_).reshape(1, 16)
    y = np.array([b"1"] * 16, dtype=np.object_).reshape(1, 16)
    for binary in (True, False):
        inputs = [httpclient.InferInput("INPUT0", [1, 16], "BYTES"), httpclient.InferInput("INPUT1", [1, 16], "BYTES")]
        inputs[0].set_data_from_numpy(x, binary_data=binary)
        inputs[1].set_data_from_numpy(y, binary_data=not binary)
        outputs = [httpclient.InferRequestedOutput("OUTPUT0", binary_data=binary),
                   httpclient.InferRequestedOutput("OUTPUT1", binary_data=not binary)]
        r = client.infer("simple_string", inputs, outputs=outputs)
        s, d = r.as_numpy("OUTPUT0"), r.as_numpy("OUTPUT1")
        for i in range(16):
            sv, dv = int(s[0][i]), int(d[0][i])
            print("%d + 1 = %d" % (in0[i], sv))
            print("%d - 1 = %d" % (in0[i], dv))
            if sv != in0[i] + 1 or dv != in0[i] - 1:
                print("error: incorrect result")
                sys.exit(1)
    print("PASS: string")


if __name__ == "__main__":
    main()
