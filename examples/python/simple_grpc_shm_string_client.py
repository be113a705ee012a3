#!/usr/bin/env python3
"""BYTES tensors in system shared memory over gRPC (reference
src/python/examples/simple_grpc_shm_string_client.py)."""
import argparse
import sys

import numpy as np

import tritonclient.grpc as grpcclient
import tritonclient.utils.shared_memory as shm
from tritonclient import utils


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    a = ap.parse_args()
    c = grpcclient.InferenceServerClient(a.url, verbose=a.verbose)
    c.unregister_system_shared_memory()
    in0 = np.arange(16, dtype=np.int32)
    x = np.array([str(v) for v in in0], dtype=np.object_)
    y = np.array(["1"] * 16, dtype=np.object_)
    xs, ys = utils.serialize_byte_tensor(x), utils.serialize_byte_tensor(y)
    sx, sy = utils.serialized_byte_size(xs), utils.serialized_byte_size(ys)
    # string outputs have data-dependent size: reserve generously
    out_size = 4 * 16 * 8
    h_out = shm.create_shared_memory_region("output_data", "/output_simple_str", out_size * 2)
    c.register_system_shared_memory("output_data", "/output_simple_str", out_size * 2)
    h_in = shm.create_shared_memory_region("input_data", "/input_simple_str", sx + sy)
    shm.set_shared_memory_region(h_in, [xs])
    shm.set_shared_memory_region(h_in, [ys], offset=sx)
    c.register_system_shared_memory("input_data", "/input_simple_str", sx + sy)
    inputs = [grpcclient.InferInput("INPUT0", [1, 16], "BYTES"), grpcclient.InferInput("INPUT1", [1, 16], "BYTES")]
    inputs[0].set_shared_memory("input_data", sx)
    inputs[1].set_shared_memory("input_data", sy, offset=sx)
    outputs = [grpcclient.InferRequestedOutput("OUTPUT0"),
               grpcclient.InferRequestedOutput("OUTPUT1")]
    outputs[0].set_shared_memory("output_data", out_size)
    outputs[1].set_shared_memory("output_data", out_size, offset=out_size)
    r = c.infer("simple_string", inputs, outputs=outputs)
    s = shm.get_contents_as_numpy(h_out, np.object_, r.get_output("OUTPUT0").shape)
    d = shm.get_contents_as_numpy(h_out, np.object_, r.get_output("OUTPUT1").shape, offset=out_size)
    for i in range(16):
        print("%s + 1 = %s" % (x[i], s[0][i].decode()))
        print("%s - 1 = %s" % (x[i], d[0][i].decode()))
        if int(s[0][i]) != in0[i] + 1 or int(d[0][i]) != in0[i] - 1:
            print("shm infer error: incorrect result")
            sys.exit(1)
    c.unregister_system_shared_memory()
    shm.destroy_shared_memory_region(h_out)
    shm.destroy_shared_memory_region(h_in)
    print("PASS: system shared memory (BYTES)")


if __name__ == "__main__":
    main()
