"""Tiny image codec + classification preprocessing (no PIL/OpenCV on the box).

Mirrors the preprocessing of reference src/python/examples/image_client.py:154-194
(INCEPTION scaling ``x/127.5 - 1``, VGG mean subtraction, NCHW/NHWC) using
numpy only.  Decodes binary PPM (P6) / PGM (P5) and a raw ``TCIMG`` container
(``b"TCIMG" + u16 H + u16 W + u8 C + HWC bytes``) used by the examples.
"""

import struct

import numpy as np


def encode_raw(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    if img.ndim == 2:
        img = img[:, :, None]
    h, w, c = img.shape
    return b"TCIMG" + struct.pack("<HHB", h, w, c) + img.tobytes()


def encode_ppm(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    return b"P6\n%d %d\n255\n" % (w, h) + img.tobytes()


def decode_image(blob):
    blob = bytes(blob)
    if blob[:5] == b"TCIMG":
        h, w, c = struct.unpack_from("<HHB", blob, 5)
        return np.frombuffer(blob, dtype=np.uint8, offset=10, count=h * w * c).reshape(h, w, c)
    if blob[:2] in (b"P6", b"P5"):
        parts = []
        pos = 2
        while len(parts) < 3:
            while blob[pos : pos + 1].isspace():
                pos += 1
            if blob[pos : pos + 1] == b"#":
                while blob[pos : pos + 1] not in (b"\n", b""):
                    pos += 1
                continue
            start = pos
            while not blob[pos : pos + 1].isspace():
                pos += 1
            parts.append(int(blob[start:pos]))
        pos += 1
        w, h, _ = parts
        c = 3 if blob[:2] == b"P6" else 1
        return np.frombuffer(blob, dtype=np.uint8, offset=pos, count=h * w * c).reshape(h, w, c)
    raise ValueError("unsupported image encoding (expected PPM/PGM/TCIMG)")


def resize_bilinear(img, h, w):
    ih, iw = img.shape[:2]
    if (ih, iw) == (h, w):
        return img.astype(np.float32)
    ys = (np.arange(h) + 0.5) * ih / h - 0.5
    xs = (np.arange(w) + 0.5) * iw / w - 0.5
    y0 = np.clip(np.floor(ys).astype(int), 0, ih - 1)
    x0 = np.clip(np.floor(xs).astype(int), 0, iw - 1)
    y1 = np.clip(y0 + 1, 0, ih - 1)
    x1 = np.clip(x0 + 1, 0, iw - 1)
    wy = np.clip(ys - y0, 0, 1)[:, None, None]
    wx = np.clip(xs - x0, 0, 1)[None, :, None]
    f = img.astype(np.float32)
    top = f[y0][:, x0] * (1 - wx) + f[y0][:, x1] * wx
    bot = f[y1][:, x0] * (1 - wx) + f[y1][:, x1] * wx
    return top * (1 - wy) + bot * wy


def preprocess(img, c, h, w, scaling="INCEPTION", fmt="NCHW", dtype=np.float32):
    if c == 1 and img.shape[2] == 3:
        img = img.mean(axis=2, keepdims=True)
    elif c == 3 and img.shape[2] == 1:
        img = np.repeat(img, 3, axis=2)
    x = resize_bilinear(img, h, w)
    if scaling == "INCEPTION":
        x = x / 127.5 - 1.0
    elif scaling == "VGG":
        mean = np.array([123.0, 117.0, 104.0] if c == 3 else [128.0], np.float32)
        x = x - mean
    x = x.astype(dtype)
    if fmt == "NCHW":
        x = np.transpose(x, (2, 0, 1))
    return np.ascontiguousarray(x)


def inception_preprocess(img, h, w, fmt="NCHW"):
    return preprocess(img, 3, h, w, "INCEPTION", fmt)


_SCALE_BIAS = {
    "NONE": lambda c: ([1.0] * c, [0.0] * c),
    "INCEPTION": lambda c: ([1.0 / 127.5] * c, [-1.0] * c),
    "VGG": lambda c: ([1.0] * c, [-m for m in ([123.0, 117.0, 104.0] if c == 3 else [128.0])]),
}
_DEVICE_DTYPES = {"FP32": np.float32, "FP16": np.float16}


def preprocess_batch_device(resized, scaling="INCEPTION", fmt="NCHW", dtype="FP32", device=0):
    """Scale + HWC->CHW transpose + dtype convert of a batch of resized HWC
    fp32 images in ONE K6 ``layout_pack`` launch on the GPU (LDS-tiled
    transpose; replaces the numpy scale/transpose of ``preprocess``, reference
    src/python/examples/image_client.py:154-194 and
    src/c++/examples/image_client.cc:86-188).  The images are uploaded once as
    a host->device copy, the packed [n, C, H, W] (or [n, H, W, C]) batch comes
    back as numpy.  ``dtype`` is the model's Triton datatype (FP32 or FP16).
    Returns None when the datatype has no device path (integer models)."""
    if dtype not in _DEVICE_DTYPES:
        return None
    import torch

    from triton_client_amd.ops import hip

    imgs = [np.ascontiguousarray(r, dtype=np.float32) for r in resized]
    h, w, c = imgs[0].shape
    dev = torch.device("cuda", device)
    src = torch.from_numpy(np.stack(imgs, axis=0)).to(dev, non_blocking=False)
    shape = (len(imgs), c, h, w) if fmt == "NCHW" else (len(imgs), h, w, c)
    dst = torch.empty(shape, device=dev, dtype=torch.float32 if dtype == "FP32" else torch.float16)
    scale, bias = _SCALE_BIAS[scaling](c)
    stream = torch.cuda.current_stream(dev).cuda_stream
    per = c * h * w * dst.element_size()
    for i0 in range(0, len(imgs), 64):  # K6 takes up to 64 source pointers per launch
        n = min(64, len(imgs) - i0)
        hip.layout_pack([src[i].data_ptr() for i in range(i0, i0 + n)], "FP32", "NHWC", dst.data_ptr() + i0 * per,
                        dtype, fmt, c, h, w, scale=scale, bias=bias, stream=stream)
    return dst.cpu().numpy()
