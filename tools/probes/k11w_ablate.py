#!/usr/bin/env python3
"""Build timing-ablation variants of the K11w kernel into k12ab/ (git-ignored
scratch libraries, never the production one): each patches the source in a
temporary copy, compiles densenet_x3.hip and links it with the tree's other
kernel objects.  tools/probes/k11w_ablate.sh times them with k11x_ab.py.

  noconv : producers skip the conversion (no VALU, no stage writes)
  nomma1 : consumers skip the 1x1 MFMAs (operand reads kept)
  no3x3  : consumers skip the 3x3 MFMAs (operand reads kept)
  pf4/pf6: producer X steps in flight; noprio: producers without s_setprio 1
"""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "csrc/kernels/densenet_x3.hip")
HIPCC = "/opt/rocm/bin/hipcc"


def patch_last(s, old, new):
    i = s.rindex(old)
    return s[:i] + new + s[i + len(old):]


def variants(s):
    k = s.index("x3_dense_ws_kernel(X3FusedParams p)")
    head, body = s[:k], s[k:]
    # tuning arms (A/B against the production build)
    for pf in (4, 6):
        yield "pf%d" % pf, s.replace("constexpr int kPfW = 3;", "constexpr int kPfW = %d;" % pf, 1)
    yield "noprio", head + body.replace("    __builtin_amdgcn_s_setprio(1);", "", 1)
    yield "noconv", head + body.replace("convert(g + 1, slot);", "", 1)
    mma1 = "acc = x3_32(a1[st & 1][kc][0], a1[st & 1][kc][1], ld16(q), ld16(q + kCvtF), acc);"
    yield "nomma1", head + body.replace(mma1, "acc[0] += __builtin_bit_cast(float, ld16(q)[0] ^ ld16(q + kCvtF)[1] ^ "
                                              "a1[st & 1][kc][0][2] ^ a1[st & 1][kc][1][3]);", 1)
    mma3 = "acc[pg] = x3_16(w2h[t], w2l[t], bq[step % (kLead + 1)][0], bq[step % (kLead + 1)][1], acc[pg]);"
    yield "no3x3", head + body.replace(mma3, "acc[pg][0] += __builtin_bit_cast(float, bq[step % (kLead + 1)][0][0] ^ "
                                             "bq[step % (kLead + 1)][1][1] ^ w2h[t][0] ^ w2l[t][1]);", 1)


def main():
    s = open(SRC).read()
    objs = [o for o in glob.glob(os.path.join(ROOT, "build/*/*.o")) if not o.endswith("/densenet_x3.o")]
    out = os.path.join(ROOT, "k12ab")
    os.makedirs(out, exist_ok=True)
    only = set(sys.argv[1].split(",")) if len(sys.argv) > 1 else None
    for name, text in variants(s):
        if only and name not in only:
            continue
        assert text != s, name
        tmp = os.path.join(ROOT, "csrc/kernels", "_abl_%s.hip" % name)
        try:
            open(tmp, "w").write(text)
            obj = "/tmp/_abl_%s.o" % name
            subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I",
                            os.path.join(ROOT, "csrc"), "-c", "-o", obj, tmp], check=True)
        finally:
            os.remove(tmp)
        lib = os.path.join(out, "libtcamd_hip_k11w_%s.so" % name)
        subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", "-o", lib, obj, *objs,
                        "-L/opt/rocm/lib", "-lamdhip64"], check=True)
        print(lib, flush=True)


if __name__ == "__main__":
    sys.exit(main())
