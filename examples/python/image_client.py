#!/usr/bin/env python3
"""Image classification client (reference src/python/examples/image_client.py).

Reads model metadata/config to find the input layout, preprocesses images
(NONE / INCEPTION / VGG scaling, NCHW or NHWC), sends batches over HTTP or
gRPC (sync, async, or gRPC streaming) and prints the top-k classes returned
by the server's classification extension.  Images are decoded with PIL when
available, else with the framework's PPM/raw decoder.
"""
import argparse
import os
import queue
import sys
from functools import partial

import numpy as np

import tritonclient.grpc as grpcclient
import tritonclient.grpc.model_config_pb2 as mc
import tritonclient.http as httpclient
from tritonclient.utils import InferenceServerException, triton_to_np_dtype


def load_image(path):
    try:
        from PIL import Image

        return np.asarray(Image.open(path).convert("RGB"))
    except Exception:
        from triton_client_amd.utils.image import decode_image

        with open(path, "rb") as f:
            return decode_image(f.read())


def completion_callback(user_data, result, error):
    """async_infer / stream callback: the client calls it as callback(result=..., error=...)."""
    user_data.put(error if error else result)


def parse_model(metadata, config, protocol):
    """-> (max_batch_size, input_name, output_name, c, h, w, format, dtype)."""
    if protocol == "grpc":
        inputs, outputs = metadata.inputs, metadata.outputs
        cfg = config.config
        max_batch = cfg.max_batch_size
        in_fmt = mc.ModelInput.Format.Name(cfg.input[0].format) if cfg.input else "FORMAT_NONE"
        in_name, in_dt, in_shape = inputs[0].name, inputs[0].datatype, list(inputs[0].shape)
        out_name = outputs[0].name
    else:
        inputs, outputs = metadata["inputs"], metadata["outputs"]
        max_batch = config.get("max_batch_size", 0)
        in_fmt = config["input"][0].get("format", "FORMAT_NONE") if config.get("input") else "FORMAT_NONE"
        in_name, in_dt, in_shape = inputs[0]["name"], inputs[0]["datatype"], list(inputs[0]["shape"])
        out_name = outputs[0]["name"]
    if len(inputs) != 1 or len(outputs) != 1:
        raise Exception("expecting 1 input and 1 output, got {} and {}".format(len(inputs), len(outputs)))
    dims = in_shape[1:] if max_batch > 0 else in_shape
    if len(dims) != 3:
        raise Exception("expecting input to have 3 dims, model '{}' input has {}".format(in_name, len(dims)))
    fmt = "NHWC" if in_fmt == "FORMAT_NHWC" else "NCHW"
    if fmt == "NHWC":
        h, w, c = dims
    else:
        c, h, w = dims
    return max_batch, in_name, out_name, c, h, w, fmt, in_dt


def preprocess(img, fmt, dtype, c, h, w, scaling):
    from triton_client_amd.utils.image import resize_bilinear

    if c == 1:
        img = img.mean(axis=2, keepdims=True)
    img = resize_bilinear(img.astype(np.float32), h, w)
    npdt = triton_to_np_dtype(dtype)
    if scaling == "INCEPTION":
        img = img / 127.5 - 1.0
    elif scaling == "VGG":
        img = img - (np.array([123.0, 117.0, 104.0], dtype=np.float32) if c == 3 else 128.0)
    img = img.astype(npdt)
    return np.transpose(img, (2, 0, 1)) if fmt == "NCHW" else img


def postprocess(results, output_name, batch_size, supports_batching):
    out = results.as_numpy(output_name)
    if supports_batching and len(out) != batch_size:
        raise Exception("expected {} results, got {}".format(batch_size, len(out)))
    lines = []
    for rows in (out if supports_batching else [out]):
        for cls in rows:
            s = cls.decode() if isinstance(cls, bytes) else str(cls)
            parts = s.split(":")
            lines.append("    {} ({}) = {}".format(parts[0], parts[1], parts[2] if len(parts) > 2 else ""))
    return lines


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-a", "--async", dest="async_set", action="store_true")
    ap.add_argument("--streaming", action="store_true")
    ap.add_argument("-m", "--model-name", required=True)
    ap.add_argument("-x", "--model-version", default="")
    ap.add_argument("-b", "--batch-size", type=int, default=1)
    ap.add_argument("-c", "--classes", type=int, default=1)
    ap.add_argument("-s", "--scaling", choices=["NONE", "INCEPTION", "VGG"], default="NONE")
    ap.add_argument("-u", "--url", default=None)
    ap.add_argument("-i", "--protocol", default="HTTP", choices=["HTTP", "gRPC", "http", "grpc"])
    ap.add_argument("--device-preprocess", action="store_true",
                    help="scale/transpose/convert on the GPU with the K6 layout_pack kernel (FP32/FP16 models)")
    ap.add_argument("image_filename")
    a = ap.parse_args()
    protocol = a.protocol.lower()
    if a.streaming and protocol != "grpc":
        raise Exception("Streaming is only allowed with gRPC protocol")
    mod = grpcclient if protocol == "grpc" else httpclient
    url = a.url or ("localhost:8001" if protocol == "grpc" else "localhost:8000")
    try:
        client = mod.InferenceServerClient(url, verbose=a.verbose) if protocol == "grpc" else \
            mod.InferenceServerClient(url, verbose=a.verbose, concurrency=1)
        md = client.get_model_metadata(a.model_name, a.model_version)
        cfg = client.get_model_config(a.model_name, a.model_version)
    except InferenceServerException as e:
        print("failed to retrieve the metadata/config: " + str(e))
        sys.exit(1)
    max_batch, in_name, out_name, c, h, w, fmt, dtype = parse_model(md, cfg, protocol)
    supports_batching = max_batch > 0
    if not supports_batching and a.batch_size != 1:
        print("ERROR: This model doesn't support batching.")
        sys.exit(1)
    if os.path.isdir(a.image_filename):
        files = sorted(os.path.join(a.image_filename, f) for f in os.listdir(a.image_filename))
    else:
        files = [a.image_filename]
    images = None
    if a.device_preprocess:
        from triton_client_amd.utils.image import preprocess_batch_device, resize_bilinear

        resized = []
        for f in files:
            img = load_image(f)
            if c == 1:
                img = img.mean(axis=2, keepdims=True)
            resized.append(resize_bilinear(img.astype(np.float32), h, w))
        packed = preprocess_batch_device(resized, a.scaling, fmt, dtype)
        if packed is not None:
            images = list(packed)
    if images is None:
        images = [preprocess(load_image(f), fmt, dtype, c, h, w, a.scaling) for f in files]
    # batches (cycling over the images to fill the last batch)
    requests, batched_names = [], []
    idx = 0
    done = False
    while not done:
        batch, names = [], []
        for _ in range(a.batch_size):
            batch.append(images[idx])
            names.append(files[idx])
            idx = (idx + 1) % len(images)
            if idx == 0:
                done = True
        data = np.stack(batch, axis=0) if supports_batching else batch[0]
        inp = mod.InferInput(in_name, list(data.shape), dtype)
        inp.set_data_from_numpy(data)
        out = mod.InferRequestedOutput(out_name, class_count=a.classes)
        requests.append(([inp], [out]))
        batched_names.append(names)
    responses = []
    if a.streaming:
        q = queue.Queue()
        client.start_stream(partial(completion_callback, q))
        for i, (inp, out) in enumerate(requests):
            client.async_stream_infer(a.model_name, inp, request_id=str(i), model_version=a.model_version,
                                      outputs=out)
        for _ in requests:
            r = q.get(timeout=120)
            if isinstance(r, Exception):
                print("inference failed: " + str(r))
                sys.exit(1)
            responses.append(r)
        client.stop_stream()
    elif a.async_set:
        if protocol == "grpc":
            q = queue.Queue()
            for i, (inp, out) in enumerate(requests):
                client.async_infer(a.model_name, inp, partial(completion_callback, q),
                                   request_id=str(i), model_version=a.model_version, outputs=out)
            for _ in requests:
                r = q.get(timeout=120)
                if isinstance(r, Exception):
                    print("inference failed: " + str(r))
                    sys.exit(1)
                responses.append(r)
        else:
            handles = [client.async_infer(a.model_name, inp, request_id=str(i), model_version=a.model_version,
                                          outputs=out) for i, (inp, out) in enumerate(requests)]
            responses = [hd.get_result() for hd in handles]
    else:
        for i, (inp, out) in enumerate(requests):
            responses.append(client.infer(a.model_name, inp, request_id=str(i), model_version=a.model_version,
                                          outputs=out))
    for r in responses:
        rid = int(r.get_response().id if protocol == "grpc" else r.get_response()["id"])
        print("Request {}, batch size {}".format(rid, a.batch_size))
        for name, line in zip(batched_names[rid] * a.classes, postprocess(r, out_name, a.batch_size,
                                                                          supports_batching)):
            print(line)
    print("PASS")


if __name__ == "__main__":
    main()
