#!/usr/bin/env python3
"""System (POSIX) shared memory for inputs and outputs over gRPC (reference
src/python/examples/simple_grpc_shm_client.py)."""
import argparse
import sys

import numpy as np

import tritonclient.grpc as grpcclient
import tritonclient.utils.shared_memory as shm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    a = ap.parse_args()
    c = grpcclient.InferenceServerClient(a.url, verbose=a.verbose)
    c.unregister_system_shared_memory()
    x = np.arange(16, dtype=np.int32)
    y = np.ones(16, dtype=np.int32)
    nbytes = x.nbytes
    h_out = shm.create_shared_memory_region("output_data", "/output_simple", nbytes * 2)
    c.register_system_shared_memory("output_data", "/output_simple", nbytes * 2)
    h_in = shm.create_shared_memory_region("input_data", "/input_simple", nbytes * 2)
    shm.set_shared_memory_region(h_in, [x])
    shm.set_shared_memory_region(h_in, [y], offset=nbytes)
    c.register_system_shared_memory("input_data", "/input_simple", nbytes * 2)
    inputs = [grpcclient.InferInput("INPUT0", [1, 16], "INT32"), grpcclient.InferInput("INPUT1", [1, 16], "INT32")]
    inputs[0].set_shared_memory("input_data", nbytes)
    inputs[1].set_shared_memory("input_data", nbytes, offset=nbytes)
    outputs = [grpcclient.InferRequestedOutput("OUTPUT0"),
               grpcclient.InferRequestedOutput("OUTPUT1")]
    outputs[0].set_shared_memory("output_data", nbytes)
    outputs[1].set_shared_memory("output_data", nbytes, offset=nbytes)
    r = c.infer("simple", inputs, outputs=outputs)
    o0 = r.get_output("OUTPUT0")
    s = shm.get_contents_as_numpy(h_out, np.int32, o0.shape)
    o1 = r.get_output("OUTPUT1")
    d = shm.get_contents_as_numpy(h_out, np.int32, o1.shape, offset=nbytes)
    for i in range(16):
        print("%d + %d = %d" % (x[i], y[i], s[0][i]))
        print("%d - %d = %d" % (x[i], y[i], d[0][i]))
        if x[i] + y[i] != s[0][i] or x[i] - y[i] != d[0][i]:
            print("shm infer error: incorrect result")
            sys.exit(1)
    print(c.get_system_shared_memory_status())
    c.unregister_system_shared_memory()
    assert len(shm.mapped_shared_memory_regions()) == 2
    shm.destroy_shared_memory_region(h_out)
    shm.destroy_shared_memory_region(h_in)
    assert len(shm.mapped_shared_memory_regions()) == 0
    print("PASS: system shared memory")


if __name__ == "__main__":
    main()
