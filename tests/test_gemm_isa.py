"""K17's dynamic tile claim (csrc/kernels/gemm.hip claim_tile) is inline asm:
hipcc does not know the atomic's destination VGPR is written late, so the
built code must leave that register alone until the consumer reads it behind
the kernel's counted ring wait.  This CPU test compiles the kernel for gfx950
and checks, in every K17 instantiation, that the claim's destination register
is referenced by exactly one other instruction, a read (no copy, spill or
reuse of it in between)."""

import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def k17_asm(tmp_path_factory):
    if not os.path.exists(HIPCC) or shutil.which("python") is None:
        pytest.skip("no hipcc")
    out = tmp_path_factory.mktemp("isa") / "gemm.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "csrc"), "-S",
                    "--cuda-device-only", os.path.join(ROOT, "csrc", "kernels", "gemm.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    text = out.read_text()
    kernels = {}
    for m in re.finditer(r"^(_Z\w*k17_gemm_kernel\w*):[^\n]*\n(.*?)s_endpgm", text, re.S | re.M):
        kernels[m.group(1)] = m.group(2)
    return kernels


def _refs(line, reg):
    """True when the instruction ``line`` names VGPR ``reg`` (alone or in a range)."""
    for m in re.finditer(r"(?<![\w\[])v(\d+)\b", line):
        if int(m.group(1)) == reg:
            return True
    for m in re.finditer(r"(?<!\w)v\[(\d+):(\d+)\]", line):
        if int(m.group(1)) <= reg <= int(m.group(2)):
            return True
    return False


def test_k17_claim_register_is_left_alone(k17_asm):
    # 3 tile heights x (3 epilogues x bf16 / fp32 out + the erf GELU's fp32 and x3 forms)
    assert len(k17_asm) == 24, sorted(k17_asm)
    for name, body in k17_asm.items():
        lines = [ln.split(";")[0].strip() for ln in body.splitlines()]
        lines = [ln for ln in lines if ln and not ln.startswith(".") and not ln.endswith(":")]
        claims = [ln for ln in lines if re.match(r"global_atomic_add v\d+, v\[\d+:\d+\], v\d+, off sc0$", ln)]
        assert len(claims) == 1, (name, claims)
        reg = int(re.match(r"global_atomic_add v(\d+),", claims[0]).group(1))
        users = [ln for ln in lines if _refs(ln, reg) and ln != claims[0]]
        assert len(users) == 1, (name, reg, users)
        ops = users[0].split(None, 1)[1].split(",")
        assert not _refs(ops[0], reg), (name, users[0])  # read as a source, never rewritten
