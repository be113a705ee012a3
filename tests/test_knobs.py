"""The knob table (triton_client_amd/utils/knobs.py) against the native
registry (csrc/runtime/knobs.hip), the sources, README and the tests it names;
plus the CPU-testable knobs themselves (library override / lazy load, the
BYTES auto-path thresholds, the native front end's environment)."""

import glob
import json
import os
import re
import subprocess
import sys
import time

import numpy as np
import pytest

from triton_client_amd.utils.knobs import BY_NAME, KNOBS

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_ENV_READ = re.compile(r'(?:environ(?:\.get)?\(|environ\[|getenv\()\s*"((?:TCAMD|TCSERVE|TC)_[A-Z0-9_]+)"')


def _sources():
    pats = ["triton_client_amd/**/*.py", "tritonclient/**/*.py", "csrc/**/*.hip", "csrc/**/*.h", "csrc/**/*.cc",
            "bench.py", "__graft_entry__.py"]
    for p in pats:
        for f in glob.glob(os.path.join(REPO, p), recursive=True):
            if "/build" not in f and "/proto/" not in f:
                yield f


def _native_table():
    src = open(os.path.join(REPO, "csrc/runtime/knobs.hip")).read()
    body = src[src.index("kDefs[] = {"):src.index("};", src.index("kDefs[] = {"))]
    return re.findall(r'\{"(TCAMD_[A-Z0-9_]+)", ([^,]+),', body)


def test_native_table_matches_registry():
    table = _native_table()
    native = [k for k in KNOBS if k.kind == "native"]
    assert [n for n, _ in table] == [k.name for k in native]
    for (n, d), k in zip(table, native):
        assert eval(d.replace("ll", "")) == k.default, n  # noqa: S307 - integer literals from our own source


def test_native_registry_at_runtime():
    from triton_client_amd.ops import hip

    live = hip.knobs()
    assert sorted(live) == sorted(k.name for k in KNOBS if k.kind == "native")
    for name, v in live.items():
        assert v["default"] == BY_NAME[name].default and v["doc"], name


def test_sources_read_only_registered_knobs():
    seen = set()
    for f in _sources():
        text = open(f, errors="replace").read()
        for name in _ENV_READ.findall(text):
            seen.add(name)
            assert name in BY_NAME, "%s reads %s, which is not in triton_client_amd/utils/knobs.py" % (f, name)
        if f.endswith(".hip") and not f.endswith("knobs.hip"):
            # kernel host code goes through the registry (switchable in-process)
            assert not re.search(r'getenv\("TCAMD_', text), f
    # the source-scanned knobs (native ones come from the registry table)
    for k in KNOBS:
        if k.kind != "native":
            assert k.name in seen, "%s is in the table but no source reads it" % k.name


def test_every_knob_in_readme_and_its_test_exists():
    readme = open(os.path.join(REPO, "README.md")).read()
    sec = readme[readme.index("## Tuning knobs"):]
    sec = sec[:sec.index("\n## ", 4)] if "\n## " in sec[4:] else sec
    for k in KNOBS:
        assert "`%s`" % k.name in sec, "README 'Tuning knobs' misses %s" % k.name
        path, func = k.test.split("::")
        assert os.path.exists(os.path.join(REPO, path)), k.test
        assert re.search(r"^def %s\(" % func, open(os.path.join(REPO, path)).read(), re.M), k.test
        assert func in sec, "README names no test for %s" % k.name


def test_native_knob_set_and_restore():
    from triton_client_amd.ops import hip

    d = hip.knobs()["TCAMD_X3_MAX_SPLITS"]["value"]
    with hip.knob(TCAMD_X3_MAX_SPLITS=2, TCAMD_K3_MODE=1):
        assert hip.knobs()["TCAMD_X3_MAX_SPLITS"]["value"] == 2
        assert hip.knobs()["TCAMD_K3_MODE"]["value"] == 1
    assert hip.knobs()["TCAMD_X3_MAX_SPLITS"]["value"] == d
    assert hip.knobs()["TCAMD_K3_MODE"]["value"] == 0
    with pytest.raises(KeyError, match="unknown native knob"):
        hip.knob_set("TCAMD_NO_SUCH_KNOB", 1)


def _py(code, **env):
    e = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    for k in list(e):
        if k.startswith(("TCAMD_", "TCSERVE_")):
            del e[k]
    e.update(env)
    return subprocess.run([sys.executable, "-c", code], cwd=REPO, env=e, capture_output=True, text=True, timeout=120)


def test_hip_lib_override_and_lazy_load():
    from triton_client_amd.ops import hip

    # eager load of a missing override fails at import; lazy defers it to first use
    r = _py("import triton_client_amd.ops.hip", TCAMD_HIP_LIB="/nonexistent/libtcamd_hip.so")
    assert r.returncode != 0 and "not built" in r.stderr
    r = _py("from triton_client_amd.ops import hip\n"
            "try:\n    hip.lib()\nexcept ImportError as e:\n    print('deferred', e)",
            TCAMD_HIP_LIB="/nonexistent/libtcamd_hip.so", TCAMD_LAZY_HIP="1")
    assert r.returncode == 0 and r.stdout.startswith("deferred"), r.stderr
    # an A/B build at another path loads and binds
    r = _py("from triton_client_amd.ops import hip; print(hip._PATH, len(hip.knobs()))", TCAMD_HIP_LIB=hip._PATH)
    assert r.returncode == 0 and r.stdout.split() == [hip._PATH, str(len(hip.knobs()))], r.stderr
    # a native knob is seeded from its environment variable
    r = _py("from triton_client_amd.ops import hip; print(hip.knobs()['TCAMD_X3_WS_MIN']['value'])",
            TCAMD_X3_WS_MIN="777")
    assert r.returncode == 0 and r.stdout.strip() == "777", r.stderr


def test_bytes_auto_path_knobs():
    code = ("from tritonclient.utils import hip_shared_memory as m\n"
            "print([m._bytes_on_host(n, 'auto') for n in (10, 11)], "
            "[m._bytes_on_host(n, 'auto', get=True) for n in (4, 5, 10**7)])")
    r = _py(code)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "[True, True] [True, True, True]"  # defaults: host to 8192, get always host
    r = _py(code, TCAMD_BYTES_HOST_MAX="10", TCAMD_BYTES_GET_DEVICE_MIN="5")
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "[True, False] [True, False, False]"


def _loop_threads(pid):
    names = []
    for t in glob.glob("/proc/%d/task/*/comm" % pid):
        try:
            names.append(open(t).read().strip())
        except OSError:
            pass
    return sorted(n for n in names if n.startswith("tcs-loop"))


def test_tcserve_env_knobs(tmp_path):
    """TCSERVE_IO_THREADS sets the event-loop count, TCSERVE_HTTP=0 leaves REST
    on aiohttp (tcserve terminates gRPC only), TCSERVE_LIB picks the library."""
    import urllib.request

    from triton_client_amd.perf.harness import ServerProcess
    from triton_client_amd.server import native_frontend

    if not native_frontend.available():
        pytest.skip("libtcserve not built")
    r = _py("from triton_client_amd.server import native_frontend as n; print(n.LIB_PATH)", TCSERVE_LIB="/x/libtcserve.so")
    assert r.returncode == 0 and r.stdout.strip() == "/x/libtcserve.so", r.stderr
    seen = {}
    for http in ("1", "0"):
        srv = ServerProcess(gpu=False, models="add_sub_batched", log_path=str(tmp_path / ("srv%s.log" % http)),
                            env={"TCSERVE_HTTP": http, "TCSERVE_IO_THREADS": "3"})
        try:
            srv.wait_ready(timeout=120)
            deadline = time.time() + 10
            while len(_loop_threads(srv.proc.pid)) < 3 and time.time() < deadline:
                time.sleep(0.1)
            assert _loop_threads(srv.proc.pid) == ["tcs-loop0", "tcs-loop1", "tcs-loop2"]
            # a binary-tensor infer: tcserve serves it natively when it owns the HTTP port
            a = np.arange(16, dtype=np.int32)
            hdr = json.dumps({"inputs": [{"name": n, "shape": [1, 16], "datatype": "INT32",
                                          "parameters": {"binary_data_size": 64}} for n in ("INPUT0", "INPUT1")],
                              "parameters": {"binary_data_output": True}}).encode()
            req = urllib.request.Request("http://%s/v2/models/add_sub_batched/infer" % srv.http_url,
                                         data=hdr + a.tobytes() + a.tobytes(), method="POST",
                                         headers={"Inference-Header-Content-Length": str(len(hdr))})
            with urllib.request.urlopen(req, timeout=10) as resp:
                assert resp.status == 200
                seen[http] = resp.headers.get("Server") or ""
        finally:
            srv.stop()
    assert "aiohttp" not in seen["1"]  # tcserve answered
    assert "aiohttp" in seen["0"], seen
