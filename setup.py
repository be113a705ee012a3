"""Packaging for the MI355X client framework (reference src/python/library/setup.py:36-139).

Same distribution name and extras as the reference (``tritonclient[http]``,
``[grpc]``, ``[cuda]``, ``[all]``; ``[hip]`` is the MI355X name of ``[cuda]``),
plus the native libraries this framework builds in-tree with ``make``:

  tritonclient/utils/shared_memory/libcshm.so   POSIX shm C ABI
  triton_client_amd/ops/lib/libtcamd_hip.so     HIP runtime glue + gfx950 kernels
  triton_client_amd/ops/lib/libtcamd_host.so    host codecs
  csrc/cpp/build/{lib,bin}                      C++ clients, perf_analyzer, tcserve
    (shipped under triton_client_amd/native/ when present)

``VERSION`` comes from the environment as in the reference (default 2.0.0.dev0).
"""

import os
import shutil
from itertools import chain

from setuptools import find_packages, setup

HERE = os.path.dirname(os.path.abspath(__file__))
VERSION = os.environ.get("VERSION", "2.0.0.dev0")


def req_file(name):
    path = os.path.join(HERE, "requirements", name)
    with open(path) as f:
        return [ln.strip() for ln in f if ln.strip() and not ln.startswith("#")]


install_requires = req_file("requirements.txt")
extras_require = {
    "http": req_file("requirements_http.txt"),
    "grpc": req_file("requirements_grpc.txt"),
    "hip": req_file("requirements_hip.txt"),
}
extras_require["cuda"] = extras_require["hip"]
extras_require["all"] = sorted(set(chain(*extras_require.values())))


def _native_payload():
    """Copy the C++ build outputs into the package tree (if built)."""
    src = os.path.join(HERE, "csrc", "cpp", "build")
    dst = os.path.join(HERE, "triton_client_amd", "native")
    files = []
    for sub in ("lib", "bin"):
        d = os.path.join(src, sub)
        if not os.path.isdir(d):
            continue
        os.makedirs(os.path.join(dst, sub), exist_ok=True)
        for name in os.listdir(d):
            shutil.copy2(os.path.join(d, name), os.path.join(dst, sub, name))
            files.append("native/%s/%s" % (sub, name))
    return files


def _packages():
    """All packages, minus the protocols disabled by the CMake options
    TRITON_ENABLE_PYTHON_{HTTP,GRPC} (passed through the environment)."""
    pk = find_packages(include=["tritonclient*", "triton_client_amd*", "tritonclientutils",
                                "tritonhttpclient", "tritongrpcclient", "tritonshmutils"])
    off = lambda k: os.environ.get(k, "ON").upper() in ("OFF", "0", "FALSE", "NO")
    if off("TRITON_ENABLE_PYTHON_HTTP"):
        pk = [p for p in pk if not (p.startswith("tritonclient.http") or p == "tritonhttpclient")]
    if off("TRITON_ENABLE_PYTHON_GRPC"):
        pk = [p for p in pk if not (p.startswith("tritonclient.grpc") or p == "tritongrpcclient")]
    return pk


if __name__ == "__main__":
    setup(
        name="tritonclient",
        version=VERSION,
        author="triton-mi355x",
        description="KServe-v2 / Triton clients (HTTP, gRPC, shared memory, HIP shared memory) for AMD MI355X",
        license="BSD",
        url="https://github.com/triton-inference-server/client",
        keywords=["grpc", "http", "triton", "tensorrt", "inference", "server", "service", "client", "rocm", "mi355x"],
        classifiers=[
            "Intended Audience :: Developers",
            "Topic :: Scientific/Engineering :: Artificial Intelligence",
            "License :: OSI Approved :: BSD License",
            "Programming Language :: Python :: 3",
            "Operating System :: POSIX :: Linux",
        ],
        packages=_packages(),
        install_requires=install_requires,
        extras_require=extras_require,
        package_data={
            "tritonclient.utils.shared_memory": ["libcshm.so"],
            "tritonclient.grpc": ["proto/*.proto"],
            "triton_client_amd.ops": ["lib/*.so"],
            "triton_client_amd": _native_payload() if os.environ.get("TCAMD_PACKAGE_NATIVE") else [],
        },
        entry_points={"console_scripts": ["tcamd-server=triton_client_amd.server.__main__:main"]},
        zip_safe=False,
    )
