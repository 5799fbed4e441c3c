"""NIOFP2D_FNO_attn (token self-attention over the bag, 2d_FPE/NIOModules.py:300-408) on the
HIP path vs the reference's golden vectors and the float64 oracle (needs a GPU).

Tolerances as SURVEY.md 8c: forward rel-L2 <= 1e-5, gradients rel-L2 <= 1e-4.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden, rel_l2
from test_gpu_parity import FWD_TOL, GRAD_TOL, _load, _run

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import blindno
    blindno.load_library()


def _grid(n, device="cuda"):
    gx, gy = np.meshgrid(np.linspace(-1, 1, n, dtype=np.float32),
                         np.linspace(-1, 1, n, dtype=np.float32), indexing="ij")
    return torch.tensor(np.stack([gx, gy], 2), device=device)


@pytest.mark.parametrize("case,heads,train", [
    ("nio2d_fno_attn_train", ("fno_drift", "fno_diffusion"), True),
    ("nio2d_fno_attn_eval", ("fno_drift", "fno_diffusion"), False),
    ("nc_nio2d_fno_attn_train", ("fno_Fx", "fno_Fy"), True)])
def test_niofp2d_fno_attn_golden(case, heads, train):
    from blindno import NIOFP2D_FNO_attn
    g = load_golden(case)
    m = _load(NIOFP2D_FNO_attn(2, 3, 100, 25, 2, 6, 5, 2, 20, 20, heads=heads), g)
    m.train(train)
    idx = g["idx"] if train else None
    _run(m, g, lambda m, i: m(i["x"], i["grid"], bag_idx=idx), ["x", "grid"])


def test_niofp2d_fno_attn_numpy_draw_matches_reference():
    """Without bag_idx the train-mode draw consumes numpy's global RNG like the reference
    (randint(50, T), choice(T, L, replace=False))."""
    from blindno import NIOFP2D_FNO_attn
    g = load_golden("nio2d_fno_attn_train")
    m = _load(NIOFP2D_FNO_attn(2, 3, 100, 25, 2, 6, 5, 2, 20, 20), g).cuda().train()
    np.random.seed(19)
    out = m(torch.from_numpy(g["in.x"]).cuda(), torch.from_numpy(g["in.grid"]).cuda())
    assert rel_l2(out.detach().cpu().numpy(), g["out"]) <= FWD_TOL


@pytest.mark.parametrize("N,T,L,B", [(61, 100, 77, 2),      # ragged S (3721), reference grid
                                     (20, 256, 254, 1),     # T = L + 2 = 256 tokens (the cap)
                                     (33, 60, 1, 2)])       # a single-snapshot bag
def test_niofp2d_fno_attn_vs_oracle(N, T, L, B):
    import oracle
    from blindno import NIOFP2D_FNO_attn
    torch.manual_seed(11)
    m = NIOFP2D_FNO_attn(2, 3, 100, 25, 2, 8, 6, 2, N, N).cuda().train()
    x = torch.randn(B, T, N, N).cuda()
    grid = _grid(N).requires_grad_(True)
    idx = np.random.RandomState(4).choice(T, L, replace=False)
    out = m(x, grid, bag_idx=idx)
    cot = torch.randn_like(out)
    (out * cot).sum().backward()
    p = {k: v.detach().cpu().double().requires_grad_(True) for k, v in m.state_dict().items()}
    gref = grid.detach().cpu().double().requires_grad_(True)
    ref = oracle.niofp2d_fno_attn(p, x.cpu(), gref, idx=idx.tolist())
    assert rel_l2(out.detach().cpu().numpy(), ref.detach().numpy()) <= FWD_TOL
    (ref * cot.cpu().double()).sum().backward()
    for k, prm in m.named_parameters():
        if p[k].grad is not None:
            e = rel_l2(prm.grad.cpu().numpy(), p[k].grad.numpy())
            assert e <= GRAD_TOL, (k, e)
    assert m.fc0.weight.grad is None        # fc0 is read through .data, as in the reference
    assert rel_l2(grid.grad.cpu().numpy(), gref.grad.numpy()) <= GRAD_TOL


def test_bag_attention_too_many_tokens_raises():
    import blindno
    from blindno import ops
    u = torch.zeros(1, 255, 64, device="cuda")
    with pytest.raises(blindno.BlindnoError):
        ops.BagAttnFn.apply(u, torch.zeros(64, 2, device="cuda"), torch.zeros(4, 1, device="cuda"),
                            torch.zeros(4, device="cuda"))
