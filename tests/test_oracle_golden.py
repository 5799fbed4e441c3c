"""Pin the CPU oracle to golden vectors captured from the reference itself.

Tolerances: the reference runs in fp32 (pocketfft), the oracle in float64 with
explicit DFT sums, so agreement is at fp32 rounding: forward rel-L2 <= 1e-5,
gradients rel-L2 <= 1e-4.
"""
import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden, rel_l2
from recipe import make_array, make_state

FWD_TOL = 1e-5
GRAD_TOL = 1e-4


def _params(g, prefix="p."):
    return {k[len(prefix):]: torch.from_numpy(v) for k, v in g.items() if k.startswith(prefix)}


def _check(g, out, params, inputs, skip_missing=()):
    assert rel_l2(out.detach().numpy(), g["out"]) <= FWD_TOL
    cot = torch.from_numpy(g["cot"]).double()
    (out * cot).sum().backward()
    n = 0
    for k, v in g.items():
        if k.startswith("g."):
            name = k[2:]
            p = params[name]
            assert p.grad is not None, name
            assert rel_l2(p.grad.numpy(), v) <= GRAD_TOL, (name, rel_l2(p.grad.numpy(), v))
            n += 1
        elif k.startswith("gin."):
            name = k[4:]
            assert rel_l2(inputs[name].grad.numpy(), v) <= GRAD_TOL, name
            n += 1
    assert n > 0


def _leaf(g, prefix="p."):
    out = {}
    for k, v in _params(g, prefix).items():
        t = v.to(torch.complex128 if v.is_complex() else torch.float64)
        if t.is_floating_point() or t.is_complex():
            t.requires_grad_(True)
        out[k] = t
    return out


@pytest.mark.parametrize("case", ["sc2d_a", "sc2d_overlap", "sc2d_nyq"])
def test_spectral_conv2d(case):
    g = load_golden(case)
    p = _leaf(g)
    x = torch.from_numpy(g["in.x"]).double().requires_grad_(True)
    y = oracle.spectral_conv2d(x, p["weights1"], p["weights2"])
    _check(g, y, p, {"x": x})


@pytest.mark.parametrize("case", ["sc1d", "sc1d_nyq"])
def test_spectral_conv1d(case):
    g = load_golden(case)
    p = _leaf(g)
    x = torch.from_numpy(g["in.x"]).double().requires_grad_(True)
    y = oracle.spectral_conv1d(x, p["weights1"])
    _check(g, y, p, {"x": x})


@pytest.mark.parametrize("case", ["fno2d", "fno2d_input61", "fno2d_head61"])
def test_fno2d(case):
    g = load_golden(case)
    p = _leaf(g)
    x = torch.from_numpy(g["in.x"]).double().requires_grad_(True)
    _check(g, oracle.fno2d(p, x), p, {"x": x})


@pytest.mark.parametrize("case", ["fno1d", "fno1d_input64"])
def test_fno1d(case):
    g = load_golden(case)
    p = _leaf(g)
    x = torch.from_numpy(g["in.x"]).double().requires_grad_(True)
    _check(g, oracle.fno1d(p, x), p, {"x": x})


@pytest.mark.parametrize("case,heads", [("nio2d_fno_train", ("fno_drift", "fno_diffusion")),
                                        ("nio2d_fno_eval", ("fno_drift", "fno_diffusion")),
                                        ("nc_nio2d_fno_eval", ("fno_Fx", "fno_Fy"))])
def test_niofp2d_fno(case, heads):
    g = load_golden(case)
    p = _leaf(g)
    x = torch.from_numpy(g["in.x"]).double().requires_grad_(True)
    grid = torch.from_numpy(g["in.grid"]).double().requires_grad_(True)
    idx = g["idx"].tolist() if "idx" in g else None
    if idx is not None:
        assert len(idx) == int(g["L"])
    y = oracle.niofp2d_fno(p, x, grid, idx=idx, heads=heads)
    _check(g, y, p, {"x": x, "grid": grid})


@pytest.mark.parametrize("case,heads", [("nio2d_fno_attn_train", ("fno_drift", "fno_diffusion")),
                                        ("nio2d_fno_attn_eval", ("fno_drift", "fno_diffusion")),
                                        ("nc_nio2d_fno_attn_train", ("fno_Fx", "fno_Fy"))])
def test_niofp2d_fno_attn(case, heads):
    """Token self-attention variant (2d_FPE/NIOModules.py:300-408): bag drawn WITHOUT
    replacement in train mode, fc0 = Linear(1, width)."""
    g = load_golden(case)
    p = _leaf(g)
    x = torch.from_numpy(g["in.x"]).double().requires_grad_(True)
    grid = torch.from_numpy(g["in.grid"]).double().requires_grad_(True)
    idx = g["idx"].tolist() if "idx" in g else None
    if idx is not None:
        assert len(idx) == int(g["L"]) and len(set(idx)) == len(idx)
    y = oracle.niofp2d_fno_attn(p, x, grid, idx=idx, heads=heads)
    _check(g, y, p, {"x": x, "grid": grid})


def test_cpu_ref_niofp2d_nc():
    """cpu_ref.niofp2d_fft (the NIO model as the reference executes it: F.conv2d, F.batch_norm,
    addmm) on the nio2d_nc_train golden (80^2, Encoder2D branch, FFN trunk, heads Fx/Fy), fp32
    with the bars of the fp64 oracle's check (BatchNorm over 50 images)."""
    import json
    from oracle import cpu_ref
    g = load_golden("nio2d_nc_train")
    shapes = [(k, tuple(s)) for k, s in json.loads(str(g["layout_json"]))]
    st = make_state(shapes, seed=int(g["recipe_seed"]))
    p = {k: torch.from_numpy(v).float().requires_grad_(v.dtype.kind == "f") for k, v in st.items()}
    x = torch.from_numpy(g["in.x"]).float()
    grid = torch.from_numpy(g["in.grid"]).float()
    y = cpu_ref.niofp2d_fft(p, x, grid, idx=g["idx"].tolist(), heads=("fno_Fx", "fno_Fy"))
    assert rel_l2(y.detach().numpy(), g["out"]) <= 1e-4
    (y * torch.from_numpy(g["cot"]).float()).sum().backward()
    gmax = max(float(v) for k, v in g.items() if k.startswith("gnorm."))
    n = 0
    for k, v in g.items():
        if k.startswith("g."):
            assert rel_l2(p[k[2:]].grad.numpy(), v) <= 1e-3, k
            n += 1
        if k.startswith("gnorm."):
            got = float(p[k[6:]].grad.norm())
            assert abs(got - float(v)) <= 1e-3 * abs(float(v)) + 1e-5 * gmax, k
    assert n > 0


@pytest.mark.parametrize("case,heads", [("nio1d_fno_train", ("fno_drift", "fno_diffusion")),
                                        ("nio1d_fno_eval", ("fno_drift", "fno_diffusion")),
                                        ("gpe_nio_fno_train", ("fno_V",))])
def test_niofp_fno_1d(case, heads):
    g = load_golden(case)
    p = _leaf(g)
    x = torch.from_numpy(g["in.x"]).double().requires_grad_(True)
    grid = torch.from_numpy(g["in.grid"]).double().requires_grad_(True)
    idx = g["idx"].tolist() if "idx" in g else None
    y = oracle.niofp_fno(p, x, grid, idx=idx, heads=heads)
    _check(g, y, p, {"x": x, "grid": grid})


def test_niofp2d_nio_branch_trunk():
    """NIOFP2D (config D's model) at the reference grid 80^2; parameters from the
    shared numpy recipe (the 11M-parameter encoder cannot be a fixture)."""
    import json
    g = load_golden("nio2d_nc_train")
    shapes = [(k, tuple(s)) for k, s in json.loads(str(g["layout_json"]))]
    st = make_state(shapes, seed=int(g["recipe_seed"]))
    p = {k: torch.from_numpy(v).double().requires_grad_(v.dtype.kind == "f") for k, v in st.items()}
    x = torch.from_numpy(g["in.x"]).double()
    assert np.array_equal(g["in.x"], make_array((1, 51, 80, 80), 401, "nio2d_nc.x"))
    grid = torch.from_numpy(g["in.grid"]).double()
    y = oracle.niofp2d(p, x, grid, idx=g["idx"].tolist(), heads=("fno_Fx", "fno_Fy"))
    assert rel_l2(y.detach().numpy(), g["out"]) <= 1e-4   # BN over 50 images in fp32
    (y * torch.from_numpy(g["cot"]).double()).sum().backward()
    gmax = max(float(v) for k, v in g.items() if k.startswith("gnorm."))
    for k, v in g.items():
        if k.startswith("g."):
            assert rel_l2(p[k[2:]].grad.numpy(), v) <= 1e-3, k
        if k.startswith("gnorm."):
            # conv biases ahead of train-mode BatchNorm have exactly zero gradient; the fp32
            # reference leaves ~1e-8 noise there, hence the absolute term
            got = float(p[k[6:]].grad.norm())
            assert abs(got - float(v)) <= 1e-3 * abs(float(v)) + 1e-5 * gmax, k


NIO1D_CASES = {
    # fixture: (heads, final kernels, conv4) -- 1d_FPE/NIOModules.py:15-84, 1d_GPE/NIOModules.py:160-223
    "nio1d_train": (("fno_drift", "fno_diffusion"), (5, 4, 15), False),
    "gpe_nio1d_train": (("fno_V",), (5, 7, 4), True),
}


def nio1d_params(g):
    """Recipe parameters of a 1D NIO fixture (float64 leaves)."""
    import json
    shapes = [(k, tuple(s)) for k, s in json.loads(str(g["layout_json"]))]
    st = make_state(shapes, seed=int(g["recipe_seed"]), complex_names=json.loads(str(g["complex_json"])))
    return st, {k: torch.from_numpy(v).to(torch.complex128 if v.dtype.kind == "c" else torch.float64)
                .requires_grad_(v.dtype.kind in "fc") for k, v in st.items()}


@pytest.mark.parametrize("case", sorted(NIO1D_CASES))
def test_niofp_nio_1d(case):
    """1D NIO (Encoder branch + FFN trunk + DeepONet + FNO1d heads) in train mode, recipe
    parameters, recorded bag draw.  The fixture is the reference's fp32 run; ten train-mode
    BatchNorms make the encoder gradients fp32-sensitive (as nio2d_nc_train): fwd 1e-5,
    gradients 1e-3, prefix/norm entries of the big convolutions 1e-3."""
    heads, kernels, conv4 = NIO1D_CASES[case]
    g = load_golden(case)
    _, p = nio1d_params(g)
    x = torch.from_numpy(g["in.x"]).double().requires_grad_(True)
    grid = torch.from_numpy(g["in.grid"]).double()
    y = oracle.niofp(p, x, grid, idx=g["idx"].tolist(), heads=heads, kernels=kernels, conv4=conv4)
    assert rel_l2(y.detach().numpy(), g["out"]) <= FWD_TOL
    (y * torch.from_numpy(g["cot"]).double()).sum().backward()
    gmax = max(float(v) for k, v in g.items() if k.startswith("gnorm."))
    n = 0
    for k, v in g.items():
        if k.startswith("g."):
            assert rel_l2(p[k[2:]].grad.numpy(), v) <= 1e-3, (k, rel_l2(p[k[2:]].grad.numpy(), v))
            n += 1
        elif k.startswith("gpre."):
            got = p[k[5:]].grad.reshape(-1)[:v.size].numpy()
            assert rel_l2(got, v) <= 1e-3, k
            n += 1
        elif k.startswith("gnorm."):
            got = float(p[k[6:]].grad.norm())
            assert abs(got - float(v)) <= 1e-3 * abs(float(v)) + 1e-5 * gmax, k
    assert n > 20
    assert rel_l2(x.grad.numpy(), g["gin.x"]) <= 1e-3


def test_adam_two_steps():
    g = load_golden("adam_fno2d")
    names = [k[3:] for k in g if k.startswith("p0.")]
    for name in names:
        p = torch.from_numpy(g["p0." + name]).double()
        m = torch.zeros_like(p)
        v = torch.zeros_like(p)
        for step in (1, 2):
            p, m, v = oracle.adam_step(p, torch.from_numpy(g[f"g{step}." + name]), m, v, step, lr=0.0005)
            assert rel_l2(p.numpy(), g[f"p{step}." + name]) <= 1e-6, (name, step)


def test_metrics():
    g = load_golden("metric_train_rel_l2")
    e0, e1 = oracle.train_rel_l2_2ch(torch.from_numpy(g["pred"]), torch.from_numpy(g["out"]))
    assert rel_l2(e0.numpy(), g["e_drift"]) <= 1e-6 and rel_l2(e1.numpy(), g["e_diffusion"]) <= 1e-6
    g = load_golden("metric_rel_l2")
    assert abs(oracle.rel_l2(g["a"], g["b"]) - float(g["val"])) <= 1e-6 * float(g["val"])
    g = load_golden("metric_time_avg_rel_l2_2d")
    assert abs(oracle.time_averaged_relative_l2(g["pt_pred"], g["pt_ref"]) - float(g["val"])) <= 1e-12
    g = load_golden("metric_time_avg_L2_1d")
    v = oracle.time_averaged_L2_error(g["t"], g["rho_ref"], g["t"], g["rho_pred"], g["x"])
    assert abs(v - float(g["val"])) <= 1e-12


def test_gpe_solver_oracle():
    """oracle.gpe_ref (explicit DFT) vs the reference's numpy-FFT solver (a14)."""
    from oracle import gpe_ref
    for order in (2, 4):
        g = load_golden(f"gpe_solve_o{order}")
        x = g["x"]
        t, rec = gpe_ref.solve(gpe_ref.initial_condition(2, x), x, float(g["dt"]), float(g["t_final"]), order,
                               float(g["g"]), float(g["kappa"]), g["V"])
        assert np.allclose(t, g["t"])
        assert rel_l2(rec, g["psi"]) <= 1e-11, (order, rel_l2(rec, g["psi"]))
    g = load_golden("gpe_solve_ic")
    x = np.linspace(-10, 10, 32)
    for ic in (1, 3):
        _, rec = gpe_ref.solve(gpe_ref.initial_condition(ic, x), x, 0.01, 0.2, 2, 1.0, 0.5, g[f"V_ic{ic}"])
        assert rel_l2(rec, g[f"psi_ic{ic}"]) <= 1e-11


def test_gpe_datagen_oracle():
    from oracle import gpe_ref
    g = load_golden("gpe_datagen")
    x = np.linspace(-10, 10, 128)
    rng = np.random.RandomState(int(g["seed"]))
    V = gpe_ref.training_potentials(3, x, 1001, rng=rng)
    assert np.array_equal(V, g["V"])
    _, rec = gpe_ref.solve(gpe_ref.initial_condition(2, x), x, 0.005, 5.0, 2, 2.0, 2.0, V[0])
    assert rel_l2(np.abs(rec)[::10], g["y"][0]) <= 1e-10


# ---------------------------------------------------------------- fp32 torch.fft restatement
# (oracle.cpu_ref: bench.py's CPU baseline and the GPU-vs-CPU parity leg), pinned to the
# same reference goldens in the reference's own precision (fp32 vs fp32: fwd 1e-5, grads 1e-4)

def _leaf32(g, prefix="p."):
    out = {}
    for k, v in _params(g, prefix).items():
        t = v.to(torch.complex64 if v.is_complex() else torch.float32)
        out[k] = t.requires_grad_(True)
    return out


def _check32(g, out, params, inputs):
    assert rel_l2(out.detach().numpy(), g["out"]) <= FWD_TOL
    (out * torch.from_numpy(g["cot"]).float()).sum().backward()
    n = 0
    for k, v in g.items():
        if k.startswith("g."):
            assert rel_l2(params[k[2:]].grad.numpy(), v) <= GRAD_TOL, k
            n += 1
        elif k.startswith("gin."):
            assert rel_l2(inputs[k[4:]].grad.numpy(), v) <= GRAD_TOL, k
            n += 1
    assert n > 0


@pytest.mark.parametrize("case", ["sc2d_a", "sc2d_overlap", "sc2d_nyq"])
def test_cpu_ref_spectral_conv2d(case):
    from oracle import cpu_ref
    g = load_golden(case)
    p = _leaf32(g)
    x = torch.from_numpy(g["in.x"]).float().requires_grad_(True)
    _check32(g, cpu_ref.spectral_conv2d_fft(x, p["weights1"], p["weights2"]), p, {"x": x})


@pytest.mark.parametrize("case", ["sc1d", "sc1d_nyq"])
def test_cpu_ref_spectral_conv1d(case):
    from oracle import cpu_ref
    g = load_golden(case)
    p = _leaf32(g)
    x = torch.from_numpy(g["in.x"]).float().requires_grad_(True)
    _check32(g, cpu_ref.spectral_conv1d_fft(x, p["weights1"]), p, {"x": x})


@pytest.mark.parametrize("case,heads", [("nio2d_fno_train", ("fno_drift", "fno_diffusion")),
                                        ("nio2d_fno_eval", ("fno_drift", "fno_diffusion")),
                                        ("nc_nio2d_fno_eval", ("fno_Fx", "fno_Fy"))])
def test_cpu_ref_niofp2d_fno(case, heads):
    from oracle import cpu_ref
    g = load_golden(case)
    p = _leaf32(g)
    x = torch.from_numpy(g["in.x"]).float().requires_grad_(True)
    grid = torch.from_numpy(g["in.grid"]).float().requires_grad_(True)
    idx = g["idx"].tolist() if "idx" in g else None
    _check32(g, cpu_ref.niofp2d_fno_fft(p, x, grid, idx=idx, heads=heads), p, {"x": x, "grid": grid})


@pytest.mark.parametrize("case,heads", [("nio1d_fno_train", ("fno_drift", "fno_diffusion")),
                                        ("nio1d_fno_eval", ("fno_drift", "fno_diffusion")),
                                        ("gpe_nio_fno_train", ("fno_V",))])
def test_cpu_ref_niofp_fno_1d(case, heads):
    from oracle import cpu_ref
    g = load_golden(case)
    p = _leaf32(g)
    x = torch.from_numpy(g["in.x"]).float().requires_grad_(True)
    grid = torch.from_numpy(g["in.grid"]).float().requires_grad_(True)
    idx = g["idx"].tolist() if "idx" in g else None
    _check32(g, cpu_ref.niofp_fno_fft(p, x, grid, idx=idx, heads=heads), p, {"x": x, "grid": grid})


# ---------------------------------------------------------------- PermInvUNet_attn
def unet_recipe_params(g):
    """The golden's parameters, regenerated from recipe.py (make_golden_unet.py loads the same
    values into the reference module)."""
    import json
    shapes = [(k, tuple(s)) for k, s in json.loads(str(g["layout_json"]))]
    cplx = json.loads(str(g["complex_json"]))
    return make_state(shapes, seed=int(g["recipe_seed"]), complex_names=cplx)


def unet_oracle_run(g, dim, variant, train, prec="fp64", perturb=None):
    """(out, {name: grad}, dx) of the oracle on a UNet golden's inputs and cotangent.
    ``perturb`` (a seed): inputs and parameters multiplied by 1 + 2^-24 N(0, 1) first, i.e.
    an fp32-rounding-sized input perturbation (the conditioning envelope below)."""
    st = unet_recipe_params(g)
    if "run_mean" in g:                      # eval: running stats after the train forward
        depth = int(g["depth"])
        chs = [int(g["base_ch"]) * 2 ** i for i in range(depth + 1)]
        off = np.cumsum([0] + chs)
        for i in range(depth + 1):
            st[f"skip_norms.{i}.running_mean"] = g["run_mean"][off[i]:off[i + 1]]
            st[f"skip_norms.{i}.running_var"] = g["run_var"][off[i]:off[i + 1]]
    rdt, cdt = (torch.float64, torch.complex128) if prec == "fp64" else (torch.float32, torch.complex64)
    oracle.set_precision(prec)
    try:
        p = {k: torch.from_numpy(np.asarray(v)).to(cdt if np.iscomplexobj(v) else rdt)
             .requires_grad_(np.asarray(v).dtype.kind in "fc") for k, v in st.items()}
        x = torch.from_numpy(g["in.x"]).to(rdt)
        if perturb is not None:
            gen = torch.Generator().manual_seed(perturb)

            def jit(t):
                if not t.is_floating_point():
                    return t
                return (t.double() * (1 + 2.0 ** -24 * torch.randn(t.shape, generator=gen,
                                                                   dtype=torch.float64))).to(t.dtype)
            x = jit(x)
            with torch.no_grad():
                for k in p:
                    if p[k].is_floating_point() and k.split(".")[-1] in ("weight", "bias", "weights1", "weights2"):
                        p[k].copy_(jit(p[k]))
        x.requires_grad_(True)
        idx = g["idx"].tolist() if "idx" in g else None
        y = oracle.unet_ref.perminv_unet_attn(p, x, int(g["depth"]), dim, idx=idx, bn_train=train,
                                              variant=variant)
        (y * torch.from_numpy(g["cot"]).to(rdt)).sum().backward()
    finally:
        oracle.set_precision("fp64")
    grads = {k: v.grad.detach().to(torch.complex128 if v.is_complex() else torch.float64).numpy()
             for k, v in p.items() if v.grad is not None}
    return y.detach().double().numpy(), grads, x.grad.double().numpy()


def unet_fp32_envelope(g, dim, variant, train, o64, g64, x64, n=3, include_ref=True):
    """Largest distance from fp64 over fp32 evaluations of the same model: the oracle in fp32
    unperturbed and with n fp32-sized input perturbations, and the reference's own fp32
    gradients.  The UNet's ConvNeXt LayerNorms over 1-2 channels make some gradients hinge on a
    few near-degenerate pixels, so one fp32 run is a noisy yardstick; the envelope is not."""
    env_o, env_g, env_x = 0.0, {}, 0.0
    for seed in [None] + list(range(1, n + 1)):
        o32, g32, x32 = unet_oracle_run(g, dim, variant, train, "fp32", perturb=seed)
        env_o = max(env_o, rel_l2(o32, o64))
        env_x = max(env_x, rel_l2(x32, x64))
        for k in g64:
            env_g[k] = max(env_g.get(k, 0.0), rel_l2(g32[k], g64[k]))
    for k in g64:
        if include_ref and "g." + k in g:
            env_g[k] = max(env_g[k], rel_l2(g["g." + k], g64[k]))
    return env_o, env_g, env_x


def unet_grad_bar(e32):
    """Gradient tolerance of one parameter: 1e-4 or, where the model's own fp32
    evaluation is further from fp64 than that (bias / LayerNorm sums with cancellation), three
    times the fp32 oracle's own distance."""
    return max(GRAD_TOL, 3.0 * e32)


@pytest.mark.parametrize("case,dim,variant,train", [
    ("unet2d_train", 2, "fpe", True), ("unet2d_eval", 2, "fpe", False),
    ("nc_unet2d_train", 2, "nc", True), ("unet1d_bag_train", 1, "fpe", True),
    ("unet1d_all", 1, "fpe", True)])
def test_perminv_unet_attn(case, dim, variant, train):
    """PermInvUNet_attn (2d_FPE/NIOModules.py:1086-1181), its NC copy with ConvBlocks
    (2d_Non_conservative_FPE/NIOModules.py:932-1053) and the 1D models
    (1d_FPE/NIOModules.py:212-443): the fp64 oracle against the reference's fp32 outputs and
    gradients; gradient bars per unet_grad_bar (the fp32 oracle run gives the conditioning)."""
    g = load_golden(case)
    o64, g64, x64 = unet_oracle_run(g, dim, variant, train)
    _, env_g, env_x = unet_fp32_envelope(g, dim, variant, train, o64, g64, x64, n=2, include_ref=False)
    assert rel_l2(g["out"], o64) <= FWD_TOL
    n = 0
    scale = max(float(np.linalg.norm(v)) for v in g64.values())
    for k, v in g.items():
        if k.startswith("g."):
            name = k[2:]
            if np.linalg.norm(g64[name]) <= 1e-10 * scale:
                # structurally zero (a conv bias in front of a train-mode BatchNorm): fp32 noise
                assert np.linalg.norm(v) <= 1e-5 * scale, name
            else:
                # the reference against the envelope of the oracle's own fp32 runs
                e, e32 = rel_l2(v, g64[name]), env_g[name]
                assert e <= unet_grad_bar(e32), (name, e, e32)
            n += 1
        elif k.startswith("gnorm."):
            name = k[6:]
            assert abs(np.linalg.norm(g64[name]) - float(v)) <= GRAD_TOL * float(v), name
            n += 1
    assert rel_l2(g["gin.x"], x64) <= unet_grad_bar(env_x)
    assert n > 20
