#!/usr/bin/env python3
"""Two sequences over one gRPC bidirectional stream (start_stream /
async_stream_infer) (reference src/python/examples/simple_grpc_sequence_stream_infer_client.py)."""
import argparse
import queue
import sys
from functools import partial

import numpy as np

import tritonclient.grpc as grpcclient


def callback(user_data, result, error):
    user_data.put(error if error else result)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    ap.add_argument("-t", "--stream-timeout", type=float, default=None)
    ap.add_argument("-d", "--dyna", action="store_true", help="use simple_dyna_sequence")
    ap.add_argument("-o", "--offset", type=int, default=0, help="add to the sequence ids")
    a = ap.parse_args()
    model = "simple_dyna_sequence" if a.dyna else "simple_sequence"
    values = [11, 7, 5, 3, 2, 0, 1]
    q = queue.Queue()
    with grpcclient.InferenceServerClient(a.url, verbose=a.verbose) as client:
        client.start_stream(callback=partial(callback, q), stream_timeout=a.stream_timeout)
        ids = (1000 + a.offset, 1001 + a.offset)
        n = 0
        for sid, sign in zip(ids, (1, -1)):
            for i, v in enumerate(values):
                x = grpcclient.InferInput("INPUT", [1, 1], "INT32")
                x.set_data_from_numpy(np.array([[sign * v]], dtype=np.int32))
                client.async_stream_infer(model, [x], request_id="{}_{}".format(sid, i), sequence_id=sid,
                                          sequence_start=i == 0, sequence_end=i == len(values) - 1)
                n += 1
        results = {}
        for _ in range(n):
            r = q.get(timeout=60)
            if isinstance(r, Exception):
                print("error: " + str(r))
                sys.exit(1)
            rid = r.get_response().id
            results[rid] = int(r.as_numpy("OUTPUT")[0][0])
        client.stop_stream()
    for sid in ids:
        print("sequence %d: %s" % (sid, [results["{}_{}".format(sid, i)] for i in range(len(values))]))
    print("PASS: Sequence")


if __name__ == "__main__":
    main()
