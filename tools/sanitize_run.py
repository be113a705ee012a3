"""Run the C++ client tests and examples built with a sanitizer preset
(``make -C csrc/cpp asan`` / ``tsan``: host code only) against the in-process
CPU test server and report every binary's result.

  python tools/sanitize_run.py --build build-asan [--out profiles/r1_sanitizers.md]
"""

import argparse
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# (binary, protocol, args)
CASES = [
    ("cc_client_test", None, []),
    ("client_timeout_test", "http", ["-i", "http", "-t", "20000000"]),
    ("client_timeout_test", "grpc", ["-i", "grpc", "-a", "-t", "20000000"]),
    ("client_timeout_test", "grpc", ["-i", "grpc", "-s", "-t", "20000000"]),
    ("client_timeout_test", "grpc", ["-i", "grpc", "-p", "-t", "20000"]),
    ("memory_leak_test", "http", ["-i", "http", "-r", "100", "-M", "identity_int32", "-m", "0", "-w", "1"]),
    ("memory_leak_test", "grpc", ["-i", "grpc", "-r", "100", "-M", "identity_int32", "-m", "0", "-w", "1"]),
    ("simple_http_async_infer_client", "http", []),
    ("simple_grpc_async_infer_client", "grpc", []),
    ("simple_grpc_sequence_stream_infer_client", "grpc", []),
    ("simple_http_shm_client", "http", []),
    ("simple_grpc_shm_client", "grpc", []),
    ("simple_grpc_custom_repeat", "grpc", ["-r", "6"]),
    ("simple_http_string_infer_client", "http", []),
    ("reuse_infer_objects_client", "grpc", ["-i", "grpc"]),
    ("perf_analyzer", "grpc", ["-m", "simple", "-i", "grpc", "-a", "--concurrency-range", "1:8:7", "-p", "300",
                               "-r", "3", "-s", "50"]),
    ("perf_analyzer", "http", ["-m", "simple", "-i", "http", "--concurrency-range", "4", "-p", "300", "-r", "3",
                               "-s", "50"]),
    ("perf_analyzer", "grpc", ["-m", "simple", "-i", "grpc", "--streaming", "--concurrency-range", "4", "-p", "300",
                               "-r", "3", "-s", "50"]),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", default="build-asan")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from triton_client_amd.server import ServerHandle

    bindir = os.path.join(REPO, "csrc", "cpp", a.build, "bin")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    h = ServerHandle().start()
    rows = []
    failed = 0
    try:
        for name, proto, args in CASES:
            if name == "cc_client_test":
                cmd = [os.path.join(bindir, name), h.http_url, h.grpc_url]
            else:
                url = h.http_url if proto == "http" else h.grpc_url
                cmd = [os.path.join(bindir, name), "-u", url] + args
            t = time.time()
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
            out = r.stdout + r.stderr
            report = [ln for ln in out.splitlines() if "Sanitizer" in ln or "runtime error" in ln]
            ok = r.returncode == 0 and not report
            failed += not ok
            rows.append((name + " " + " ".join(args), r.returncode, time.time() - t, report[:3]))
            print("%-4s rc=%d %5.1fs %s %s" % ("ok" if ok else "FAIL", r.returncode, time.time() - t, name,
                                               " ".join(args)), flush=True)
            for ln in report[:5]:
                print("     ", ln)
            if not ok and not report:
                print(out[-3000:])
    finally:
        h.stop()
    if a.out:
        with open(a.out, "w") as f:
            f.write("# C++ clients under %s (host-code sanitizers)\n\n" % a.build)
            f.write("`make -C csrc/cpp %s` then `python tools/sanitize_run.py --build %s` against the in-process "
                    "CPU test server; sanitizer reports halt the binary.\n\n" % (a.build.replace("build-", ""), a.build))
            f.write("| binary + args | rc | s | sanitizer reports |\n|---|---:|---:|---|\n")
            for cmd, rc, s, rep in rows:
                f.write("| `%s` | %d | %.1f | %s |\n" % (cmd, rc, s, "; ".join(rep) or "none"))
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
