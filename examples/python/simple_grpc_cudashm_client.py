#!/usr/bin/env python3
"""Device (HIP) shared memory over gRPC: inputs and outputs live in GPU
memory, registered by IPC handle (reference
src/python/examples/simple_grpc_cudashm_client.py; `cuda_shared_memory` is
the MI355X `hip_shared_memory` module under its reference name)."""
import argparse
import sys

import numpy as np

import tritonclient.grpc as grpcclient
import tritonclient.utils.cuda_shared_memory as cudashm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    ap.add_argument("-d", "--device", type=int, default=0)
    a = ap.parse_args()
    c = grpcclient.InferenceServerClient(a.url, verbose=a.verbose)
    c.unregister_cuda_shared_memory()
    x = np.arange(16, dtype=np.int32)
    y = np.ones(16, dtype=np.int32)
    nbytes = x.nbytes
    h_out = cudashm.create_shared_memory_region("output_data", nbytes * 2, a.device)
    c.register_cuda_shared_memory("output_data", cudashm.get_raw_handle(h_out), a.device, nbytes * 2)
    h_in = cudashm.create_shared_memory_region("input_data", nbytes * 2, a.device)
    cudashm.set_shared_memory_region(h_in, [x, y])
    c.register_cuda_shared_memory("input_data", cudashm.get_raw_handle(h_in), a.device, nbytes * 2)
    inputs = [grpcclient.InferInput("INPUT0", [1, 16], "INT32"), grpcclient.InferInput("INPUT1", [1, 16], "INT32")]
    inputs[0].set_shared_memory("input_data", nbytes)
    inputs[1].set_shared_memory("input_data", nbytes, offset=nbytes)
    outputs = [grpcclient.InferRequestedOutput("OUTPUT0"),
               grpcclient.InferRequestedOutput("OUTPUT1")]
    outputs[0].set_shared_memory("output_data", nbytes)
    outputs[1].set_shared_memory("output_data", nbytes, offset=nbytes)
    r = c.infer("simple", inputs, outputs=outputs)
    s = cudashm.get_contents_as_numpy(h_out, np.int32, r.get_output("OUTPUT0").shape)
    d = cudashm.get_contents_as_numpy(h_out, np.int32, r.get_output("OUTPUT1").shape, offset=nbytes)
    for i in range(16):
        print("%d + %d = %d" % (x[i], y[i], s[0][i]))
        print("%d - %d = %d" % (x[i], y[i], d[0][i]))
        if x[i] + y[i] != s[0][i] or x[i] - y[i] != d[0][i]:
            print("cudashm infer error: incorrect result")
            sys.exit(1)
    print(c.get_cuda_shared_memory_status())
    c.unregister_cuda_shared_memory()
    assert len(cudashm.allocated_shared_memory_regions()) == 2
    cudashm.destroy_shared_memory_region(h_out)
    cudashm.destroy_shared_memory_region(h_in)
    assert len(cudashm.allocated_shared_memory_regions()) == 0
    print("PASS: cuda shared memory")


if __name__ == "__main__":
    main()
