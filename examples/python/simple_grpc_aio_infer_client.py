#!/usr/bin/env python3
"""asyncio gRPC client: control plane and concurrent inferences (reference
src/python/examples/simple_grpc_aio_infer_client.py)."""
import argparse
import asyncio
import sys

import numpy as np

import tritonclient.grpc.aio as grpcclient


async def main(a):
    async with grpcclient.InferenceServerClient(a.url, verbose=a.verbose) as c:
        if not (await c.is_server_live() and await c.is_server_ready() and await c.is_model_ready("simple")):
            print("FAILED: server/model not ready")
            sys.exit(1)
        print(await c.get_server_metadata())
        print(await c.get_model_metadata("simple"))
        print(await c.get_model_config("simple"))
        print(await c.get_inference_statistics("simple"))
        x = np.arange(16, dtype=np.int32).reshape(1, 16)
        y = np.ones((1, 16), dtype=np.int32)
        inputs = [grpcclient.InferInput("INPUT0", [1, 16], "INT32"), grpcclient.InferInput("INPUT1", [1, 16], "INT32")]
        inputs[0].set_data_from_numpy(x)
        inputs[1].set_data_from_numpy(y)
        results = await asyncio.gather(*[c.infer("simple", inputs) for _ in range(4)])
        for r in results:
            if not (np.array_equal(r.as_numpy("OUTPUT0"), x + y) and np.array_equal(r.as_numpy("OUTPUT1"), x - y)):
                print("aio infer error: incorrect result")
                sys.exit(1)
    print("PASS: aio infer")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-u", "--url", default="localhost:8001")
    asyncio.run(main(ap.parse_args()))
