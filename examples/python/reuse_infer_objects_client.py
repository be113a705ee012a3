#!/usr/bin/env python3
"""Reuse InferInput / InferRequestedOutput objects across requests, switching
between in-band data and system shared memory (reference
src/python/examples/reuse_infer_objects_client.py)."""
import argparse
import sys

import numpy as np

import tritonclient.grpc as grpcclient
import tritonclient.http as httpclient
import tritonclient.utils.shared_memory as shm


def check(r, x, y):
    if not (np.array_equal(r.as_numpy("OUTPUT0"), x + y) and np.array_equal(r.as_numpy("OUTPUT1"), x - y)):
        print("error: incorrect result")
        sys.exit(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default=None)
    ap.add_argument("-i", "--protocol", default="http", choices=["http", "grpc", "HTTP", "gRPC"])
    a = ap.parse_args()
    mod = httpclient if a.protocol.lower() == "http" else grpcclient
    url = a.url or ("localhost:8000" if mod is httpclient else "localhost:8001")
    c = mod.InferenceServerClient(url, verbose=a.verbose)
    c.unregister_system_shared_memory()
    x = np.arange(16, dtype=np.int32).reshape(1, 16)
    y = np.ones((1, 16), dtype=np.int32)
    nbytes = x.nbytes
    inputs = [mod.InferInput("INPUT0", [1, 16], "INT32"), mod.InferInput("INPUT1", [1, 16], "INT32")]
    outputs = [mod.InferRequestedOutput("OUTPUT0"), mod.InferRequestedOutput("OUTPUT1")]
    # 1) in-band
    inputs[0].set_data_from_numpy(x)
    inputs[1].set_data_from_numpy(y)
    check(c.infer("simple", inputs, outputs=outputs), x, y)
    # 2) the same objects switched to shared memory
    h_in = shm.create_shared_memory_region("input_data", "/reuse_in", nbytes * 2)
    h_out = shm.create_shared_memory_region("output_data", "/reuse_out", nbytes * 2)
    shm.set_shared_memory_region(h_in, [x, y])
    c.register_system_shared_memory("input_data", "/reuse_in", nbytes * 2)
    c.register_system_shared_memory("output_data", "/reuse_out", nbytes * 2)
    inputs[0].set_shared_memory("input_data", nbytes)
    inputs[1].set_shared_memory("input_data", nbytes, offset=nbytes)
    outputs[0].set_shared_memory("output_data", nbytes)
    outputs[1].set_shared_memory("output_data", nbytes, offset=nbytes)
    c.infer("simple", inputs, outputs=outputs)
    s = shm.get_contents_as_numpy(h_out, np.int32, [1, 16])
    d = shm.get_contents_as_numpy(h_out, np.int32, [1, 16], offset=nbytes)
    if not (np.array_equal(s, x + y) and np.array_equal(d, x - y)):
        print("error: incorrect shm result")
        sys.exit(1)
    # 3) back to in-band outputs on the same objects
    outputs[0].unset_shared_memory()
    outputs[1].unset_shared_memory()
    inputs[0].set_data_from_numpy(x)
    inputs[1].set_data_from_numpy(y)
    check(c.infer("simple", inputs, outputs=outputs), x, y)
    c.unregister_system_shared_memory()
    shm.destroy_shared_memory_region(h_in)
    shm.destroy_shared_memory_region(h_out)
    print("PASS: reuse infer objects")


if __name__ == "__main__":
    main()
