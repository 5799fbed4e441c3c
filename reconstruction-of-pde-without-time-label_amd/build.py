#!/usr/bin/env python3
"""Build libblindno.so (all HIP kernels + the C ABI of include/blindno.h) for gfx950.

    python build.py [--force] [--jobs N]

hipcc cross-compiles without a GPU.  The library is written in-tree at
``blindno/libblindno.so`` so it travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "blindno", "libblindno.so")
BUILD = os.path.join(HERE, "build")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
ARCH = os.environ.get("BLINDNO_ARCH", "gfx950")

CXXFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
            "-fvisibility=hidden", "-Wall", "-Wno-unused-function", "-Wno-unused-result"]


# per-file extra flags.  project.hip: its packed fp32 math is written explicitly (the SLP
# vectoriser's own packing is off), and MFMA results go straight to VGPRs (no
# v_accvgpr_read between the fc1 MFMA and the GELU that consumes it)
FILE_FLAGS = {"project.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"],
              "bagproj.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"]}


def _hipcc():
    h = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(h):
        raise RuntimeError("hipcc not found (ROCm toolchain required to build libblindno)")
    return h


def _newer(src_list, dst):
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return any(os.path.getmtime(s) > t for s in src_list)


def build(force: bool = False, jobs: int = 8, verbose: bool = True) -> str:
    hipcc = _hipcc()
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(INCLUDE, "blindno.h")]
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or _newer([s] + headers, o):
            todo.append((s, o))

    def compile_one(so):
        s, o = so
        cmd = [hipcc, *CXXFLAGS, *FILE_FLAGS.get(os.path.basename(s), []), "-c", s, "-o", o]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {s}:\n{r.stderr}")
        return s, r.stderr

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for s, err in ex.map(compile_one, todo):
            if verbose:
                print(f"[blindno build] compiled {os.path.basename(s)}", file=sys.stderr)
                if err.strip():
                    print(err, file=sys.stderr)
    if force or todo or _newer(objs, OUT):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        if verbose:
            print(f"[blindno build] linked {OUT}", file=sys.stderr)
    build_cabi_test(hipcc, force, verbose)
    return OUT


CABI_SRC = os.path.join(os.path.dirname(HERE), "tests", "cabi", "test_cabi.cpp")
CABI_BIN = os.path.join(os.path.dirname(HERE), "tests", "cabi", "test_cabi")


def build_cabi_test(hipcc: str, force: bool = False, verbose: bool = True) -> str:
    """The C++ caller of the C ABI (tests/cabi/test_cabi.cpp -> tests/cabi/test_cabi), linked
    against the in-tree libblindno.so through an $ORIGIN-relative rpath (the tree moves to the
    GPU box as a whole)."""
    if not os.path.exists(CABI_SRC):
        return ""
    if not force and not _newer([CABI_SRC, OUT, os.path.join(INCLUDE, "blindno.h")], CABI_BIN):
        return CABI_BIN
    rel = os.path.relpath(os.path.dirname(OUT), os.path.dirname(CABI_BIN))
    cmd = [hipcc, "-O2", "-std=c++17", f"--offload-arch={ARCH}", "-I", INCLUDE, CABI_SRC,
           "-L", os.path.dirname(OUT), "-lblindno", f"-Wl,-rpath,$ORIGIN/{rel}", "-o", CABI_BIN]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"C ABI test build failed:\n{r.stderr}")
    if verbose:
        print(f"[blindno build] built {CABI_BIN}", file=sys.stderr)
    return CABI_BIN


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args()
    print(build(force=a.force, jobs=a.jobs))
