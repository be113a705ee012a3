#!/usr/bin/env python3
"""Create a client and run an inference many times; reports resident memory
growth (reference src/python/examples/memory_growth_test.py)."""
import argparse
import resource
import sys

import numpy as np

import tritonclient.grpc as grpcclient
import tritonclient.http as httpclient


def rss_kb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default=None)
    ap.add_argument("-i", "--protocol", default="http", choices=["http", "grpc"])
    ap.add_argument("-r", "--repetitions", type=int, default=100)
    ap.add_argument("--max-growth-kb", type=int, default=64 * 1024)
    a = ap.parse_args()
    mod = httpclient if a.protocol == "http" else grpcclient
    url = a.url or ("localhost:8000" if a.protocol == "http" else "localhost:8001")
    x = np.arange(16, dtype=np.int32).reshape(1, 16)
    start = None
    for i in range(a.repetitions):
        c = mod.InferenceServerClient(url, verbose=a.verbose)
        inputs = [mod.InferInput("INPUT0", [1, 16], "INT32"), mod.InferInput("INPUT1", [1, 16], "INT32")]
        inputs[0].set_data_from_numpy(x)
        inputs[1].set_data_from_numpy(x)
        r = c.infer("simple", inputs)
        assert np.array_equal(r.as_numpy("OUTPUT0"), x * 2)
        c.close()
        if i == 10:
            start = rss_kb()
    growth = rss_kb() - (start or rss_kb())
    print("max RSS growth after warm-up: %d KB" % growth)
    if growth > a.max_growth_kb:
        print("error: memory grew by %d KB" % growth)
        sys.exit(1)
    print("PASS: memory growth")


if __name__ == "__main__":
    main()
