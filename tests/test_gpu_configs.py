"""Full-geometry parity at every BASELINE.json config, through the path bench.py times
(needs a GPU).

Each test builds the config's model at the reference's own sizes (SURVEY.md section 8 "Configs
restated"), runs ONE training step on a recorded with-replacement bag draw exactly as
``bench.py`` does -- for A, B, C, E: ``train.GraphedBagStep`` (HIP graph per distinct-count
key, deduplicated bag with multiplicity weights, grouped heads, fused snapshot encoder); for
D: ``train.GraphedBagStep`` keyed by the drawn L (no deduplication: the branch's train-mode
BatchNorm counts the bag's repeats; ``test_config_d_graphed_niofp2d_nc_128``), and the eager
NIO step beside it -- and compares the step's output and every trained parameter's
gradient (MSE loss, the reference's criterion) with the float64 oracle (``oracle.fno_ref``)
evaluated on the same inputs, weights and bag.  The oracle runs in fp64 on the GPU (plain
torch ops; it shares nothing with the HIP kernels) so the 128^2 / 256^2 cases finish in
seconds.

Tolerances (fp32 HIP vs fp64): forward rel-L2 <= 1e-5, gradients rel-L2 <= 1e-4
per parameter tensor.  Config D (ten train-mode BatchNorm'd convolutions) is held to a bar
relative to what a plain fp32 evaluation of the same graph achieves against fp64 -- see
``test_config_d_niofp2d``.
"""
import numpy as np
import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu

FWD_TOL = 1e-5
GRAD_TOL = 1e-4


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import blindno
    blindno.load_library()


def _oracle_params(model, skip=("branch.",)):
    out = {}
    for k, v in model.state_dict().items():
        if k.startswith(tuple(skip)) or not v.is_floating_point() and not v.is_complex():
            continue
        v = v.detach().to("cuda")
        v = v.to(torch.complex128) if v.is_complex() else v.double()
        out[k] = v.requires_grad_(True)
    return out


def _bn_preceded_bias(k):
    """The branch ConvBlocks' conv biases: each feeds a batch-statistics BatchNorm, so its true
    gradient is exactly 0 (the trunk's ``hidden_layers.0.bias`` / ``batch_layers.0.bias`` are
    NOT of this kind and are checked)."""
    return k.startswith("branch.") and k.endswith(".layers.0.bias")


def _check_grads(model, opt, p64, min_count, tol=GRAD_TOL, skip=()):
    """Compare the flat gradient buffer the graph filled (``opt.grad``) per parameter tensor
    (names ending in ``skip`` are left out)."""
    names = {id(p): k for k, p in model.named_parameters()}
    n = 0
    worst = 0.0
    for prm, off, sz in zip(opt.params, opt.offsets, opt.sizes):
        k = names[id(prm)]
        if skip and (skip(k) if callable(skip) else k.endswith(tuple(skip))):
            continue
        ref = p64[k].grad
        assert ref is not None, k
        ref = torch.view_as_real(ref) if ref.is_complex() else ref
        got = opt.grad[off:off + sz].view(ref.shape)
        e = rel_l2(got.cpu().numpy(), ref.cpu().numpy())
        worst = max(worst, e)
        assert e <= tol, (k, e)
        n += 1
    assert n >= min_count
    return worst


def _graphed_step_vs_oracle(model, x, y, grid, draws, oracle_fwd, min_params, fwd_tol=FWD_TOL,
                            grad_tol=GRAD_TOL):
    import blindno
    from blindno.train import DataParallel, FlatAdam, GraphedBagStep, trained_parameters
    model = model.cuda().train()
    opt = FlatAdam(trained_parameters(model), lr=1e-3)
    p64 = _oracle_params(model)
    gs = GraphedBagStep(model, blindno.mse_loss, opt, DataParallel(opt), x, y, grid)
    res = []
    for idx in draws:
        key = gs.replay(idx)
        torch.cuda.synchronize()
        assert gs.dedup and key < len(idx), "bench path must run the deduplicated bag"
        out = gs.out[key].clone()
        for v in p64.values():
            v.grad = None
        ref = oracle_fwd(p64, x.double(), grid.double(), idx)
        e_fwd = rel_l2(out.cpu().numpy(), ref.detach().cpu().numpy())
        assert e_fwd <= fwd_tol, e_fwd
        # every output channel on its own (drift / diffusion: the diffusion channel is the worse
        # conditioned one, so the whole-output figure alone could hide a regression there)
        e_ch = [rel_l2(out[..., c].cpu().numpy(), ref[..., c].detach().cpu().numpy())
                for c in range(out.shape[-1])]
        print(f"  L={len(idx)} key={key}: fwd {e_fwd:.2e} per channel "
              + " ".join(f"{e:.2e} ({e / fwd_tol:.2f} of bar)" for e in e_ch))
        assert max(e_ch) <= fwd_tol, e_ch
        loss = ((ref - y.double()) ** 2).mean()
        assert abs(float(gs.loss[key]) - float(loss.detach())) <= fwd_tol * float(loss.detach())
        loss.backward()
        e_grad = _check_grads(model, opt, p64, min_params, grad_tol)
        res.append((len(idx), key, e_fwd, e_grad))
    return res


def _grid2d(n):
    from blindno.train import grid2d
    return grid2d(n, n, "cuda")


def _draws(T, seed, k=2):
    rs = np.random.RandomState(seed)
    return [rs.choice(T, rs.randint(50, T)) for _ in range(k)]


@pytest.mark.parametrize("B", [2, 4])
def test_config_c_niofp2d_fno_128(B):
    """Config C, the headline: NIOFP2D_FNO(2,3,100,25,3,12,32,2) at 128^2 (P = 160, FNO_input
    m = 12 on ~55 distinct snapshots per bag, heads m = 32 width 12 as one grouped chain),
    T = 100, two recorded draws (two graph keys); B = 4 is the benched batch."""
    import oracle
    from blindno import Encoder2D, NIOFP2D_FNO, ops
    torch.manual_seed(0)
    m = NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 32, 2, branch_last_kernel=Encoder2D.kernel_for_grid(128))
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(B, 100, 128, 128, device="cuda", generator=g)
    y = torch.randn(B, 128, 128, 2, device="cuda", generator=g)
    assert ops.GROUPED_HEADS
    res = _graphed_step_vs_oracle(m, x, y, _grid2d(128), _draws(100, 7),
                                  lambda p, x, gr, idx: oracle.niofp2d_fno(p, x, gr, idx=idx.tolist()), 40)
    print("config C", res)


def test_config_e_niofp2d_fno_256():
    """Config E geometry in fp32: NIOFP2D_FNO at 256^2 (P = 320), B = 1, T = 100."""
    import oracle
    from blindno import Encoder2D, NIOFP2D_FNO
    torch.manual_seed(2)
    m = NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 32, 2, branch_last_kernel=Encoder2D.kernel_for_grid(256))
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(1, 100, 256, 256, device="cuda", generator=g)
    y = torch.randn(1, 256, 256, 2, device="cuda", generator=g)
    res = _graphed_step_vs_oracle(m, x, y, _grid2d(256), _draws(100, 8, k=1),
                                  lambda p, x, gr, idx: oracle.niofp2d_fno(p, x, gr, idx=idx.tolist()), 40)
    print("config E", res)


# BASELINE config E's "fp16 channel-mix + fp32 spectral accumulate", stated separately from
# SURVEY 8c's fp32 bars: fp16 operands (unit roundoff 2^-11) put each layer's spectral branch
# ~1e-3 off; the bench line's parity leg uses the same bars (bench.MIX16_TOL)
MIX16_FWD_TOL, MIX16_GRAD_TOL = 5e-3, 2e-2


def test_config_e_fp16_mix_256():
    """Config E as BASELINE.json names it: the same step with the channel mix on fp16 operands
    (blindno.set_mix_precision("fp16")), against the fp64 oracle within the fp16 bars.  (At
    initialisation the spectral branch is a small part of each layer's output, so the model-level
    error stays near fp32's; test_fp16_mix_spectral_layer checks the layer itself.)"""
    import blindno
    import oracle
    from blindno import Encoder2D, NIOFP2D_FNO
    torch.manual_seed(2)
    m = NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 32, 2, branch_last_kernel=Encoder2D.kernel_for_grid(256))
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(1, 100, 256, 256, device="cuda", generator=g)
    y = torch.randn(1, 256, 256, 2, device="cuda", generator=g)
    blindno.set_mix_precision("fp16")
    try:
        res = _graphed_step_vs_oracle(m, x, y, _grid2d(256), _draws(100, 8, k=1),
                                      lambda p, x, gr, idx: oracle.niofp2d_fno(p, x, gr, idx=idx.tolist()),
                                      40, fwd_tol=MIX16_FWD_TOL, grad_tol=MIX16_GRAD_TOL)
    finally:
        blindno.set_mix_precision("fp32")
    print("config E fp16 mix", res)


@pytest.mark.parametrize("scale", [1.0, 1e6, 1e-6])
def test_fp16_mix_spectral_layer(scale):
    """One SpectralConv2d (head shape: C = 12, m = 32, P = 160, 4 samples) with the fp16 mix vs
    the fp64 oracle, forward and every gradient, at input scales 1e6 and 1e-6 too: the block
    scaling keeps the unnormalised spectra inside fp16's range (no inf / flush to zero)."""
    import blindno
    import oracle
    from blindno import SpectralConv2d
    torch.manual_seed(5)
    sc = SpectralConv2d(12, 12, 32, 32).cuda()
    x = (torch.randn(4, 12, 160, 160, device="cuda") * scale).requires_grad_(True)
    blindno.set_mix_precision("fp16")
    try:
        y = sc(x)
        cot = torch.randn_like(y)
        (y * cot).sum().backward()
        torch.cuda.synchronize()
    finally:
        blindno.set_mix_precision("fp32")
    w1, w2 = [w.detach().double().requires_grad_(True) for w in (sc.weights1, sc.weights2)]
    x64 = x.detach().double().requires_grad_(True)
    ref = oracle.spectral_conv2d(x64, w1, w2)
    (ref * cot.double()).sum().backward()
    assert torch.isfinite(y).all()
    e = rel_l2(y.detach().cpu().numpy(), ref.detach().cpu().numpy())
    assert 1e-6 < e <= MIX16_FWD_TOL, e
    for got, want in ((x.grad, x64.grad), (sc.weights1.grad, w1.grad), (sc.weights2.grad, w2.grad)):
        eg = rel_l2(got.cpu().numpy(), want.cpu().numpy())
        assert eg <= MIX16_GRAD_TOL, eg


@pytest.mark.parametrize("cfg", ["A", "B"])
def test_config_ab_niofp_fno_1d(cfg):
    """Config A: 1d_FPE NIOFP_FNO(3,30,15,2), N = 64, T = 256, B = 32.  Config B: 1d_GPE
    NIOFP_FNO(3,20,40,1) head fno_V, N = 256, T = 101, B = 32."""
    import oracle
    from blindno import NIOFP_FNO
    from blindno.train import grid1d
    if cfg == "A":
        args, heads, N, T, cout = (3, 30, 15, 2), ("fno_drift", "fno_diffusion"), 64, 256, 2
    else:
        args, heads, N, T, cout = (3, 20, 40, 1), ("fno_V",), 256, 101, 1
    torch.manual_seed(4)
    m = NIOFP_FNO(*args, "cuda", heads=heads)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(32, T, N, device="cuda", generator=g)
    y = torch.randn(32, N, cout, device="cuda", generator=g)
    res = _graphed_step_vs_oracle(m, x, y, grid1d(N, "cuda"), _draws(T, 9),
                                  lambda p, x, gr, idx: oracle.niofp_fno(p, x, gr, idx=idx.tolist(), heads=heads),
                                  10)
    print("config", cfg, res)


def test_config_d_niofp2d_nc_128():
    """Config D: 2d_Non_conservative_FPE NIOFP2D (Encoder2D branch with the grid-adaptive (4,2)
    final kernel, FFN trunk, DeepONet combiner, heads fno_Fx/fno_Fy) at 128^2, B = 2, one
    recorded draw, eager step (the graphed step bench.py replays: the test below).

    The branch is piecewise linear (ten Conv -> BatchNorm -> LeakyReLU blocks): a pre-activation
    within fp32 rounding of 0 can take either branch in two correct evaluations, and one flip
    moves a gradient by ~1e-3.  The fp64 oracle therefore takes every branch LeakyReLU's side
    from the HIP forward (``branch_masks``, recorded by hooks) -- the same linear piece -- and the
    SURVEY 8c bars hold as fixed numbers (forward 1e-5, gradients 1e-4)."""
    import blindno
    import oracle
    from blindno import Encoder2D, NIOFP2D
    from test_gpu_encoder import _branch_masks
    torch.manual_seed(6)
    m = NIOFP2D(2, 3, 100, 25, 3, 12, 32, 2, heads=("fno_Fx", "fno_Fy"),
                branch_last_kernel=Encoder2D.kernel_for_grid(128)).cuda().train()
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(2, 100, 128, 128, device="cuda", generator=g)
    y = torch.randn(2, 128, 128, 2, device="cuda", generator=g)
    grid = _grid2d(128)
    idx = _draws(100, 10, k=1)[0]
    heads = ("fno_Fx", "fno_Fy")
    masks, hooks = _branch_masks(m.branch)
    out = m(x, grid, bag_idx=idx)
    for h in hooks:
        h.remove()
    assert len(masks) == 10
    blindno.mse_loss(out, y).backward()
    torch.cuda.synchronize()
    p = {k: v.detach().double().requires_grad_(True) for k, v in m.state_dict().items()
         if v.is_floating_point() and not k.endswith(("running_mean", "running_var"))}
    # before borrowing the HIP branches: an UNCONDITIONED fp64 forward's own LeakyReLU branches
    # may differ from the HIP ones only at near-zero pre-activations -- a handful out of
    # millions; a systematic sign / offset error in the HIP pre-activation would flip many
    own = []
    with torch.no_grad():
        oracle.fno_ref.encoder2d(oracle.fno_ref.sub_params({k: v.detach() for k, v in p.items()}, "branch"),
                                 x.double()[:, list(idx)].unsqueeze(2), record=own)
    assert len(own) == 10
    flips = sum(int((a != b).sum()) for a, b in zip(masks, own))
    total = sum(a.numel() for a in masks)
    print(f"config D LeakyReLU branches: {flips} of {total} differ from an unconditioned fp64 "
          f"forward ({flips / total:.2e}, bar 1e-5)")
    assert flips <= 1e-5 * total, (flips, total)
    ref64 = oracle.niofp2d(p, x.double(), grid.double(), idx=idx.tolist(), heads=heads, branch_masks=masks)
    ((ref64 - y.double()) ** 2).mean().backward()
    e = rel_l2(out.detach().cpu().numpy(), ref64.detach().cpu().numpy())
    print(f"config D fwd {e:.2e}")
    assert e <= FWD_TOL, e
    n, worst = 0, []
    for k, prm in m.named_parameters():
        if k.startswith("fc0.") or _bn_preceded_bias(k):
            continue     # fc0 is read through .data; a conv bias ahead of batch-stat BN has grad 0
        assert prm.grad is not None and p[k].grad is not None, k
        e = rel_l2(prm.grad.cpu().numpy(), p[k].grad.cpu().numpy())
        worst.append((e, k))
        assert e <= GRAD_TOL, (k, e)
        n += 1
    assert n > 60
    print("config D worst grads", sorted(worst)[-5:])


def _record_branch_masks(enc, store):
    """Forward hooks appending each ConvBlock's LeakyReLU branch (output > 0) to ``store``.  Run
    inside a graph capture, the comparison is a captured kernel: its output tensor is rewritten
    by every replay of that graph (``store`` keeps the tensors -- and their pool memory -- alive)."""
    names = ("convblock1", "convblock2_1", "convblock2_2", "convblock3_1", "convblock3_2", "convblock4_1",
             "convblock4_2", "convblock7_1", "convblock7_2", "convblock7_3")
    return [getattr(enc, n).register_forward_hook(lambda mod, i, o: store.append(o.detach() > 0))
            for n in names]


@pytest.mark.parametrize("B", [2])
def test_config_d_graphed_niofp2d_nc_128(B):
    """Config D as bench.py times it: the NIOFP2D training step replayed from a HIP graph per
    drawn L (train.GraphedBagStep; BatchNorm in train mode inside the graph, the buffers saved and
    restored around the capture's warm-up), at 128^2, two recorded draws (two graph keys), output,
    loss and every trained parameter's gradient (the flat buffer the graph fills) vs the fp64
    oracle.  The LeakyReLU branches of the fp64 evaluation are those the REPLAY took (recorded by
    comparisons captured into the graph), with the flip bound of test_config_d_niofp2d_nc_128;
    SURVEY 8c bars as fixed numbers."""
    import blindno
    import oracle
    from blindno import Encoder2D, NIOFP2D
    from blindno.train import DataParallel, FlatAdam, GraphedBagStep, trained_parameters
    heads = ("fno_Fx", "fno_Fy")
    torch.manual_seed(6)
    m = NIOFP2D(2, 3, 100, 25, 3, 12, 32, 2, heads=heads,
                branch_last_kernel=Encoder2D.kernel_for_grid(128)).cuda().train()
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(B, 100, 128, 128, device="cuda", generator=g)
    y = torch.randn(B, 128, 128, 2, device="cuda", generator=g)
    grid = _grid2d(128)
    opt = FlatAdam(trained_parameters(m, exclude_prefixes=("fc0.",)), lr=5e-4)
    rec = []
    hooks = _record_branch_masks(m.branch, rec)
    gs = GraphedBagStep(m, blindno.mse_loss, opt, DataParallel(opt), x, y, grid)
    assert not gs.dedup
    draws = _draws(100, 13)
    assert len(draws[0]) != len(draws[1])
    masks_of = {}
    for idx in draws:
        n0 = len(rec)
        key = gs.replay(idx)
        assert key == len(idx)
        if len(rec) > n0:
            # warm-up (eager) then capture: the last ten are the graph's own mask tensors
            assert len(rec) - n0 == 20
            masks_of[key] = rec[-10:]
    for k in masks_of:
        assert masks_of[k][0].shape[0] == B * k
    for idx in draws:
        key = gs.replay(idx)          # each key replayed again, in the other order
    for idx in reversed(draws):
        key = gs.replay(idx)
        torch.cuda.synchronize()
        out = gs.out[key].clone()
        masks = masks_of[key]
        p = {k: v.detach().double().requires_grad_(True) for k, v in m.state_dict().items()
             if v.is_floating_point() and not k.endswith(("running_mean", "running_var"))}
        own = []
        with torch.no_grad():
            oracle.fno_ref.encoder2d(oracle.fno_ref.sub_params({k: v.detach() for k, v in p.items()}, "branch"),
                                     x.double()[:, list(idx)].unsqueeze(2), record=own)
        flips = sum(int((a != b).sum()) for a, b in zip(masks, own))
        total = sum(a.numel() for a in masks)
        print(f"  graphed D L={key}: {flips} of {total} LeakyReLU branches differ from an unconditioned "
              f"fp64 forward ({flips / total:.2e}, bar 1e-5)")
        assert flips <= 1e-5 * total, (flips, total)
        ref = oracle.niofp2d(p, x.double(), grid.double(), idx=idx.tolist(), heads=heads, branch_masks=masks)
        e_fwd = rel_l2(out.cpu().numpy(), ref.detach().cpu().numpy())
        e_ch = [rel_l2(out[..., c].cpu().numpy(), ref[..., c].detach().cpu().numpy()) for c in range(2)]
        print(f"  graphed D L={key}: fwd {e_fwd:.2e}, Fx {e_ch[0]:.2e}, Fy {e_ch[1]:.2e}")
        assert max([e_fwd] + e_ch) <= FWD_TOL, (e_fwd, e_ch)
        loss = ((ref - y.double()) ** 2).mean()
        assert abs(float(gs.loss[key]) - float(loss.detach())) <= FWD_TOL * float(loss.detach())
        loss.backward()
        # conv biases ahead of batch-statistics BatchNorm: the true gradient is exactly 0
        worst = _check_grads(m, opt, p, 60, skip=_bn_preceded_bias)
        print(f"  graphed D L={key}: worst gradient {worst:.2e} (bar {GRAD_TOL})")
    for h in hooks:
        h.remove()


def test_config_c_after_training_steps():
    """Config C after 30 Adam steps (lr 5e-4) of the benched graphed step: trained weights make
    the spectral weight-gradient sums over the bag cancel heavily (the encoder's first layer),
    which an accumulation that is merely fp32-adequate at initialisation no longer survives.
    Same bar as above against the fp64 oracle."""
    import blindno
    import oracle
    from blindno import Encoder2D, NIOFP2D_FNO
    from blindno.train import DataParallel, FlatAdam, GraphedBagStep, trained_parameters
    torch.manual_seed(0)
    m = NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 32, 2, branch_last_kernel=Encoder2D.kernel_for_grid(128)).cuda().train()
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(2, 100, 128, 128, device="cuda", generator=g)
    y = torch.randn(2, 128, 128, 2, device="cuda", generator=g)
    grid = _grid2d(128)
    opt = FlatAdam(trained_parameters(m), lr=5e-4)
    gs = GraphedBagStep(m, blindno.mse_loss, opt, DataParallel(opt), x, y, grid)
    for idx in _draws(100, 11, k=30):
        gs.step(idx)
    idx = _draws(100, 12, k=1)[0]
    key = gs.replay(idx)
    torch.cuda.synchronize()
    out = gs.out[key].clone()
    p64 = _oracle_params(m)
    ref = oracle.niofp2d_fno(p64, x.double(), grid.double(), idx=idx.tolist())
    e = rel_l2(out.cpu().numpy(), ref.detach().cpu().numpy())
    assert e <= FWD_TOL, e
    ((ref - y.double()) ** 2).mean().backward()
    worst = _check_grads(m, opt, p64, 40)
    print("config C trained: fwd", e, "worst grad", worst)


def test_config_c_channel_margins_across_draws():
    """Config C's benched step (B = 4), after 40 training steps, on five recorded draws: every
    output channel's forward
    error against fp64 must stay within the 1e-5 bar AND within 2x (+ 1e-6) of what a plain fp32
    evaluation of the same graph reaches against fp64 on that draw (the conditioning floor; the
    diffusion channel's floor is close to the bar).  The per-channel
    margins are printed, so a regression toward the floor shows before it fails."""
    import oracle
    from oracle import fno_ref
    import blindno
    from blindno import Encoder2D, NIOFP2D_FNO
    from blindno.train import DataParallel, FlatAdam, GraphedBagStep, trained_parameters
    torch.manual_seed(0)
    B = 4
    m = NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 32, 2,
                    branch_last_kernel=Encoder2D.kernel_for_grid(128)).cuda().train()
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(B, 100, 128, 128, device="cuda", generator=g)
    y = torch.randn(B, 128, 128, 2, device="cuda", generator=g)
    grid = _grid2d(128)
    opt = FlatAdam(trained_parameters(m), lr=5e-4)
    gs = GraphedBagStep(m, blindno.mse_loss, opt, DataParallel(opt), x, y, grid)
    # trained as bench.py trains before its parity leg (40 Adam steps at config C's lr): the
    # diffusion channel's conditioning is that of a trained model, not of the initial weights
    for idx in _draws(100, 5, k=40):
        gs.step(idx)
    torch.cuda.synchronize()
    p64 = _oracle_params(m)
    p32 = {k: v.detach().float() if not v.is_complex() else v.detach().to(torch.complex64)
           for k, v in p64.items()}
    worst = []
    for idx in _draws(100, 23, k=5):
        key = gs.replay(idx)
        torch.cuda.synchronize()
        out = gs.out[key].double()
        with torch.no_grad():
            ref = oracle.niofp2d_fno(p64, x.double(), grid.double(), idx=idx.tolist())
            fno_ref.set_precision("fp32")
            try:
                r32 = oracle.niofp2d_fno(p32, x, grid, idx=idx.tolist()).double()
            finally:
                fno_ref.set_precision("fp64")
        line = []
        for c in range(out.shape[-1]):
            e = rel_l2(out[..., c].cpu().numpy(), ref[..., c].cpu().numpy())
            f = rel_l2(r32[..., c].cpu().numpy(), ref[..., c].cpu().numpy())
            line.append(f"ch{c} gpu {e:.2e} fp32-floor {f:.2e} ({e / FWD_TOL:.2f} of bar)")
            worst.append(e / FWD_TOL)
            assert e <= FWD_TOL, (len(idx), c, e)
            assert e <= 2 * f + 1e-6, (len(idx), c, e, f)
        print(f"  L={len(idx)} key={key}: " + "; ".join(line))
    print(f"  worst channel at {max(worst):.2f} of the bar")
