"""G3: the dependency-free Node gRPC client (clients/grpc_generated/javascript)
against the CPU server: health, metadata, typed int_contents and raw inputs."""

import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(REPO, "clients", "grpc_generated", "javascript")


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_node_grpc_client(cpu_server):
    r = subprocess.run(["node", os.path.join(JS, "client.js"), cpu_server.grpc_url], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "server live: true" in r.stdout and "model ready: true" in r.stdout
    assert '"name":"simple"' in r.stdout
    assert r.stdout.count("15 + 1 = 16; 15 - 1 = 14") == 2
    assert "PASS: js grpc client" in r.stdout


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_node_grpc_error_status(cpu_server):
    code = ("const {GRPCInferenceServiceClient}=require(%r);"
            "const c=new GRPCInferenceServiceClient(%r);"
            "c.modelMetadata('no_such_model').then(()=>{console.log('unexpected');c.close();process.exit(1)})"
            ".catch(e=>{console.log(e.message);c.close()});") % (os.path.join(JS, "triton_grpc.js"), cpu_server.grpc_url)
    r = subprocess.run(["node", "-e", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "grpc-status" in r.stdout and "no_such_model" in r.stdout


def test_go_example_uses_generated_service():
    src = open(os.path.join(REPO, "clients", "grpc_generated", "go", "grpc_simple_client.go")).read()
    for sym in ("NewGRPCInferenceServiceClient", "ServerLive", "ServerReady", "ModelMetadata", "ModelInfer",
                "RawInputContents", "RawOutputContents"):
        assert sym in src, sym
    assert src.count("{") == src.count("}")
