#!/usr/bin/env python3
"""Raw image bytes through the `preprocess_inception_ensemble` ensemble
(server-side decode + INCEPTION preprocessing + classification) (reference
src/python/examples/ensemble_image_client.py)."""
import argparse
import os
import sys

import numpy as np

import tritonclient.grpc as grpcclient
import tritonclient.http as httpclient


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-c", "--classes", type=int, default=1)
    ap.add_argument("-m", "--model-name", default="preprocess_inception_ensemble")
    ap.add_argument("-u", "--url", default=None)
    ap.add_argument("-i", "--protocol", default="HTTP", choices=["HTTP", "gRPC", "http", "grpc"])
    ap.add_argument("image_filename")
    a = ap.parse_args()
    protocol = a.protocol.lower()
    mod = grpcclient if protocol == "grpc" else httpclient
    client = mod.InferenceServerClient(a.url or ("localhost:8001" if protocol == "grpc" else "localhost:8000"),
                                       verbose=a.verbose)
    files = ([os.path.join(a.image_filename, f) for f in sorted(os.listdir(a.image_filename))]
             if os.path.isdir(a.image_filename) else [a.image_filename])
    blobs = []
    for f in files:
        with open(f, "rb") as fh:
            blobs.append(fh.read())
    data = np.array(blobs, dtype=np.object_).reshape(len(blobs), 1)
    inp = mod.InferInput("INPUT", list(data.shape), "BYTES")
    inp.set_data_from_numpy(data)
    out = mod.InferRequestedOutput("OUTPUT", class_count=a.classes)
    r = client.infer(a.model_name, [inp], outputs=[out])
    res = r.as_numpy("OUTPUT")
    if len(res) != len(files):
        print("error: expected %d results" % len(files))
        sys.exit(1)
    for f, rows in zip(files, res):
        print("Image '{}':".format(f))
        for cls in np.atleast_1d(rows):
            print("    " + (cls.decode() if isinstance(cls, bytes) else str(cls)))
    print("PASS")


if __name__ == "__main__":
    main()
