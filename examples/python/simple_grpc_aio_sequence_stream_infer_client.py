#!/usr/bin/env python3
"""asyncio gRPC stream_infer over two sequences (reference
src/python/examples/simple_grpc_aio_sequence_stream_infer_client.py)."""
import argparse
import asyncio
import sys

import numpy as np

import tritonclient.grpc.aio as grpcclient


async def main(a):
    values = [11, 7, 5, 3, 2, 0, 1]
    ids = (1000 + a.offset, 1001 + a.offset)

    async def requests():
        for sid, sign in zip(ids, (1, -1)):
            for i, v in enumerate(values):
                x = grpcclient.InferInput("INPUT", [1, 1], "INT32")
                x.set_data_from_numpy(np.array([[sign * v]], dtype=np.int32))
                yield {"model_name": "simple_sequence", "inputs": [x], "request_id": "{}_{}".format(sid, i),
                       "sequence_id": sid, "sequence_start": i == 0, "sequence_end": i == len(values) - 1}

    async with grpcclient.InferenceServerClient(a.url, verbose=a.verbose) as c:
        got = {}
        async for result, error in c.stream_infer(requests()):
            if error is not None:
                print("error: " + str(error))
                sys.exit(1)
            got[result.get_response().id] = int(result.as_numpy("OUTPUT")[0][0])
    if len(got) != 2 * len(values):
        print("error: expected %d responses, got %d" % (2 * len(values), len(got)))
        sys.exit(1)
    for sid in ids:
        print("sequence %d: %s" % (sid, [got["{}_{}".format(sid, i)] for i in range(len(values))]))
    print("PASS: Sequence")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    ap.add_argument("-o", "--offset", type=int, default=0)
    asyncio.run(main(ap.parse_args()))
