"""C8/C9: the CMake package (exported TritonClient:: targets, version
scripts) builds, installs, and is consumable out of tree; the installed
shared libraries export only the client API (reference
src/c++/library/CMakeLists.txt, lib*client.ldscript)."""

import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(REPO, "csrc", "cpp")

pytestmark = pytest.mark.skipif(shutil.which("cmake") is None or not os.path.exists("/opt/conda/lib/libnghttp2.so.14"),
                                reason="cmake / nghttp2 not available")


@pytest.fixture(scope="module")
def installed(tmp_path_factory):
    root = tmp_path_factory.mktemp("tcpkg")
    build, prefix = root / "build", root / "prefix"
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    subprocess.run(["cmake", "-S", CPP, "-B", str(build), "-DCMAKE_INSTALL_PREFIX=" + str(prefix),
                    "-DCMAKE_BUILD_TYPE=Release"] + gen, check=True, capture_output=True)
    subprocess.run(["cmake", "--build", str(build), "-j8"], check=True, capture_output=True)
    subprocess.run(["cmake", "--install", str(build)], check=True, capture_output=True)
    return root, prefix


def _exported(lib):
    out = subprocess.run(["nm", "-DC", "--defined-only", lib], check=True, capture_output=True, text=True).stdout
    return [ln.split(" ", 2)[2] for ln in out.splitlines() if ln.count(" ") >= 2]


def test_installed_layout(installed):
    _, prefix = installed
    for f in ("lib/libhttpclient.so", "lib/libgrpcclient.so", "lib/libhttpclient_static.a",
              "lib/libgrpcclient_static.a", "lib/libjson_utils_static.a", "lib/libshm_utils_static.a",
              "lib/cmake/TritonClient/TritonClientConfig.cmake", "lib/cmake/TritonClient/TritonClientTargets.cmake",
              "include/tritonclient/grpc_client.h", "include/tritonclient/http_client.h"):
        assert (prefix / f).exists(), f


@pytest.mark.parametrize("lib,allowed", [("libhttpclient.so", ("triton::client",)),
                                         ("libgrpcclient.so", ("triton::client", "inference::", "tcamd_pb::"))])
def test_symbol_export_scripts(installed, lib, allowed):
    _, prefix = installed
    syms = _exported(str(prefix / "lib" / lib))
    assert len(syms) > 50
    stray = [s for s in syms if not any(a in s for a in allowed)]
    assert not stray, stray[:10]


def test_out_of_tree_consumer(installed, cpu_server):
    root, prefix = installed
    cb = root / "consumer"
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    subprocess.run(["cmake", "-S", os.path.join(REPO, "tests", "cmake_consumer"), "-B", str(cb),
                    "-DCMAKE_PREFIX_PATH=" + str(prefix)] + gen, check=True, capture_output=True)
    r = subprocess.run(["cmake", "--build", str(cb), "-j8"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    for exe in ("consumer_shared", "consumer_static"):
        r = subprocess.run([str(cb / exe), cpu_server.http_url, cpu_server.grpc_url], capture_output=True,
                           text=True, timeout=60)
        assert r.returncode == 0, (exe, r.stdout, r.stderr)
        assert "http ok" in r.stdout and "grpc ok" in r.stdout
