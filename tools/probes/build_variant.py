#!/usr/bin/env python3
"""Build a scratch libtcamd_hip variant into the git-ignored k12ab/ for an A/B
against the production build (tools/probes/lib_ab.sh): one kernel source with
literal text replacements applied in a temporary copy, linked with the tree's
other kernel objects (make must have run).

    python tools/probes/build_variant.py NAME csrc/kernels/densenet_x3.hip 'OLD=>NEW' ['OLD2=>NEW2' ...]

Each OLD must occur exactly once.  \\n in OLD / NEW is a newline."""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HIPCC = "/opt/rocm/bin/hipcc"


def main():
    name, src = sys.argv[1], os.path.join(ROOT, sys.argv[2])
    text = open(src).read()
    for rep in sys.argv[3:]:
        old, new = (t.replace("\\n", "\n") for t in rep.split("=>", 1))
        assert text.count(old) == 1, "%r occurs %d times" % (old, text.count(old))
        text = text.replace(old, new)
    stem = os.path.splitext(os.path.basename(src))[0]
    tmp = os.path.join(os.path.dirname(src), "_variant_%s.hip" % name)
    obj = "/tmp/_variant_%s.o" % name
    try:
        open(tmp, "w").write(text)
        subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "csrc"),
                        "-c", "-o", obj, tmp], check=True)
    finally:
        os.remove(tmp)
    objs = [o for o in glob.glob(os.path.join(ROOT, "build/*/*.o")) if os.path.basename(o) != stem + ".o"]
    os.makedirs(os.path.join(ROOT, "k12ab"), exist_ok=True)
    lib = os.path.join(ROOT, "k12ab", "libtcamd_hip_%s.so" % name)
    subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", "-o", lib, obj, *objs, "-L/opt/rocm/lib",
                    "-lamdhip64"], check=True)
    print(lib)


if __name__ == "__main__":
    main()
