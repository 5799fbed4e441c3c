#!/usr/bin/env python3
"""Build a variant libblindno.so with extra preprocessor defines for ONE source file, linked
with the regular objects of every other file (build.py must have run first):

    python tools/build_variant.py NAME FILE.hip -DMACRO=VALUE [...]
    -> variants/NAME/libblindno.so   (use with BLINDNO_LIB=variants/NAME/libblindno.so)

For A/B kernel measurements (tools/kbench.py) without touching the in-tree library."""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd")
sys.path.insert(0, PKG)
import build as B  # noqa: E402


def main():
    name, src, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
    out = os.path.join(ROOT, "variants", name)
    os.makedirs(out, exist_ok=True)
    hipcc = B._hipcc()
    obj = os.path.join(out, src[:-4] + ".o")
    cmd = [hipcc, *B.CXXFLAGS, *B.FILE_FLAGS.get(src, []), *defs, "-c", os.path.join(B.CSRC, src), "-o", obj]
    subprocess.run(cmd, check=True)
    objs = [o for o in sorted(glob.glob(os.path.join(B.BUILD, "*.o"))) if os.path.basename(o) != src[:-4] + ".o"]
    lib = os.path.join(out, "libblindno.so")
    subprocess.run([hipcc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib, obj, *objs], check=True)
    print(lib)


if __name__ == "__main__":
    main()
