"""GPU examples: HIP (cuda-named) shared memory and DenseNet image
classification (image_client / grpc_image_client / ensemble_image_client)
against the GPU server."""

import os
import subprocess

import numpy as np
import pytest

from tests.test_examples import run_example

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def image_dir(tmp_path_factory):
    from triton_client_amd.utils.image import encode_ppm

    d = tmp_path_factory.mktemp("imgs")
    rng = np.random.default_rng(3)
    for i in range(3):
        img = rng.integers(0, 255, size=(240 + 16 * i, 320, 3), dtype=np.uint8)
        with open(os.path.join(d, "img%d.ppm" % i), "wb") as f:
            f.write(encode_ppm(img))
    return str(d)


@pytest.mark.parametrize("script,proto", [("simple_http_cudashm_client.py", "http"),
                                          ("simple_grpc_cudashm_client.py", "grpc")])
def test_cudashm_examples(gpu_server, script, proto):
    url = gpu_server.http_url if proto == "http" else gpu_server.grpc_url
    r = run_example(script, url, [])
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-1500:] + r.stderr[-1500:]


@pytest.mark.parametrize("proto,extra", [("http", []), ("grpc", ["-a"]), ("grpc", ["--streaming"]),
                                         ("http", ["-a", "-b", "2"]), ("http", ["--device-preprocess", "-b", "2"])])
def test_image_client(gpu_server, image_dir, proto, extra):
    url = gpu_server.http_url if proto == "http" else gpu_server.grpc_url
    r = run_example("image_client.py", url, ["-m", "densenet_onnx", "-s", "INCEPTION", "-c", "3", "-i", proto]
                    + extra + [image_dir], timeout=300)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-1500:] + r.stderr[-1500:]
    assert r.stdout.count("class_") >= 3


def test_grpc_image_client(gpu_server, image_dir):
    r = run_example("grpc_image_client.py", gpu_server.grpc_url,
                    ["-m", "densenet_onnx", "-c", "2", "-b", "2", os.path.join(image_dir, "img0.ppm")], timeout=300)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-1500:] + r.stderr[-1500:]


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_ensemble_image_client(gpu_server, image_dir, proto):
    url = gpu_server.http_url if proto == "http" else gpu_server.grpc_url
    r = run_example("ensemble_image_client.py", url, ["-c", "2", "-i", proto, image_dir], timeout=300)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-1500:] + r.stderr[-1500:]


# -- C++ examples ------------------------------------------------------------------
@pytest.mark.parametrize("name,proto", [("simple_http_cudashm_client", "http"),
                                        ("simple_grpc_cudashm_client", "grpc")])
def test_cpp_cudashm_examples(gpu_server, name, proto):
    from tests.test_cpp_examples import run_bin

    url = gpu_server.http_url if proto == "http" else gpu_server.grpc_url
    r = run_bin(name, url, [])
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-1500:] + r.stderr[-1500:]


@pytest.mark.parametrize("proto,extra", [("http", []), ("grpc", ["-a"]), ("grpc", ["--streaming", "-b", "2"]),
                                         ("http", ["--device-preprocess", "-b", "2"])])
def test_cpp_image_client(gpu_server, image_dir, proto, extra):
    from tests.test_cpp_examples import run_bin

    url = gpu_server.http_url if proto == "http" else gpu_server.grpc_url
    r = run_bin("image_client", url, ["-m", "densenet_onnx", "-s", "INCEPTION", "-c", "3", "-i", proto] + extra
                + [image_dir], timeout=300)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-1500:] + r.stderr[-1500:]


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_cpp_ensemble_image_client(gpu_server, image_dir, proto):
    from tests.test_cpp_examples import run_bin

    url = gpu_server.http_url if proto == "http" else gpu_server.grpc_url
    r = run_bin("ensemble_image_client", url, ["-c", "2", "-i", proto, os.path.join(image_dir, "img1.ppm")],
                timeout=300)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-1500:] + r.stderr[-1500:]


@pytest.mark.gpu
def test_perf_analyzer_hip_shm_with_gpu_metrics(gpu_server, tmp_path):
    """Native perf_analyzer against densenet_onnx over HIP shm with the real
    amdgpu sysfs metrics of GPU 0 (--collect-metrics)."""
    import json

    from triton_client_amd.perf import native

    j = tmp_path / "pa.json"
    r = subprocess.run([native.BIN_PATH, "-m", "densenet_onnx", "-b", "8", "-i", "grpc", "-u", gpu_server.grpc_url,
                        "--shared-memory", "hip", "--output-shared-memory-size", str(8 * 1000 * 4),
                        "--concurrency-range", "8", "-p", "500", "-r", "4", "--collect-metrics",
                        "--metrics-interval", "50", "--json-report", str(j)],
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    pt = json.load(open(j))["points"][0]
    assert pt["throughput"] > 0 and pt["errors"] == 0
    print("densenet bs8 c8:", pt["throughput"], "infer/s", pt.get("gpu"))
    assert "gpu" in pt, r.stdout[-1500:]
    # the card under test (matched to HIP device 0 by PCI address) holds the server's weights and graphs
    assert pt["gpu"]["util_pct"] >= 0 and pt["gpu"]["mem_mib"] > 100


@pytest.mark.parametrize("scaling", ["INCEPTION", "VGG"])
def test_device_preprocess_gives_host_results(gpu_server, image_dir, scaling):
    """K6 device preprocessing (Python and C++ image_client) classifies every
    image exactly like the host preprocessing path."""
    from tests.test_cpp_examples import run_bin

    args = ["-m", "densenet_onnx", "-s", scaling, "-c", "3", "-i", "grpc"]
    outs = [run_example("image_client.py", gpu_server.grpc_url, args + extra + [image_dir], timeout=300)
            for extra in ([], ["--device-preprocess"])]
    outs += [run_bin("image_client", gpu_server.grpc_url, args + extra + [image_dir], timeout=300)
             for extra in ([], ["--device-preprocess"])]
    for r in outs:
        assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-1500:] + r.stderr[-1500:]
    # result lines are "<score> (<class index>) = <label>": scores may differ in
    # the last digits (x * (1/127.5) on device vs x / 127.5 on the host)
    classes = [[ln.split("(")[1].split(")")[0] for ln in r.stdout.splitlines() if "(" in ln and ") =" in ln]
               for r in outs]
    assert classes[0] and classes[0] == classes[1], (classes[0], classes[1])
    assert classes[2] and classes[2] == classes[3], (classes[2], classes[3])
