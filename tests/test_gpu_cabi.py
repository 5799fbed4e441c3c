"""The C ABI driven from C++ with no Python in the loop (tests/cabi/test_cabi.cpp, built by
build.py): whole-op SpectralConv2d / SpectralConv1d forward against a double-precision host
restatement of the reference operation, backward through the bilinear adjoint identities,
invalid shapes rejected by error code (needs a GPU)."""
import os
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cabi", "test_cabi")

pytestmark = pytest.mark.gpu


def test_cabi_whole_op_spectral_conv():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    assert os.path.exists(BIN), "tests/cabi/test_cabi not built (run __graft_entry__.build())"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout and r.stdout.count(" ok") >= 14
