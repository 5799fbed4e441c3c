"""The torch-operator registration (blindno.torch_ops) on CPU: every op is in the dispatcher under
``torch.ops.blindno``, its schema is what the module documents, its fake-tensor shape function
gives the shapes the HIP kernels produce (so torch.compile / export can trace through it), and a
real call with CPU tensors fails loudly (there is no CPU path)."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

from blindno import BlindnoError, torch_ops
from blindno.fno import FNO1d, FNO2d, fno_params


def test_every_op_registered():
    for name in torch_ops.REGISTERED:
        op = getattr(torch.ops.blindno, name)
        assert op.default._schema.name == f"blindno::{name}"


def test_fake_shapes_spectral():
    with FakeTensorMode():
        x = torch.empty(2, 3, 20, 18)
        w = torch.empty(3, 4, 4, 5, 2)
        y, X = torch.ops.blindno.spectral_conv2d(x, w, w)
        assert y.shape == (2, 4, 20, 18) and X.shape == (2, 5, 3, 8, 2)
        x = torch.empty(2, 3, 6, 10)                     # P1 < 2 m1: all rows kept
        w = torch.empty(3, 3, 4, 6, 2)
        assert torch.ops.blindno.spectral_conv2d(x, w, w)[1].shape == (2, 6, 3, 6, 2)
        x1 = torch.empty(3, 4, 20)
        w1 = torch.empty(4, 2, 7, dtype=torch.complex64)
        y1, X1 = torch.ops.blindno.spectral_conv1d(x1, w1)
        assert y1.shape == (3, 2, 20) and X1.shape == (3, 7, 4, 1, 2) and X1.dtype == torch.float32


def test_fake_shapes_models():
    m2 = FNO2d(6, 8, 3, 5, 1)
    m1 = FNO1d(7, 8, 2, 3, 2)
    p2 = [p.detach() for p in fno_params(m2, 2)]
    p1 = [p.detach() for p in fno_params(m1, 1)]
    with FakeTensorMode(allow_non_fake_inputs=True) as mode:
        inp = torch.empty(2, 24, 20, 5)
        fp2 = [mode.from_tensor(p) for p in p2]
        # P = (30, 25); crop (P1 - pad(W), P2 - pad(H)) = (25, 19), 2d_FPE/FNOModules.py:234
        assert torch.ops.blindno.fno2d(inp, fp2, 3, 6, 6).shape == (2, 25, 19, 1)
        inp1 = torch.empty(4, 30, 3)
        fp1 = [mode.from_tensor(p) for p in p1]
        assert torch.ops.blindno.fno1d(inp1, fp1, 2, 7).shape == (4, 30, 2)
        z = torch.empty(2, 8, 30, 25)
        out = torch.ops.blindno.project_mlp(z, torch.empty(128, 8), torch.empty(128), torch.empty(1, 128),
                                           torch.empty(1), 24, 20)
        assert out.shape == (2, 24, 20, 1)
        u = torch.empty(3, 5, 100)
        assert torch.ops.blindno.bag_mean(u, torch.empty(100, 2), torch.empty(16, 3), torch.empty(16)).shape \
            == (3, 100, 16)
        x = torch.empty(7, 1, 70, 70)
        y = torch.ops.blindno.conv2d(x, torch.empty(16, 1, 3, 3), torch.empty(16), [2, 2], [1, 1])
        assert y.shape == (7, 16, 35, 35)
        assert torch.ops.blindno.mse_loss(torch.empty(3, 4), torch.empty(3, 4)).shape == ()
        assert torch.ops.blindno.time_averaged_relative_l2(torch.empty(5, 9), torch.empty(5, 9)).dtype \
            == torch.float64


def test_cpu_tensors_fail_loudly():
    with pytest.raises(BlindnoError):
        torch.ops.blindno.spectral_conv2d(torch.zeros(1, 2, 8, 8), torch.zeros(2, 2, 2, 2, 2),
                                         torch.zeros(2, 2, 2, 2, 2))
    with pytest.raises(BlindnoError):
        torch.ops.blindno.conv2d(torch.zeros(1, 1, 8, 8), torch.zeros(2, 1, 3, 3), None, [1, 1], [1, 1])
