"""FPE density propagation (§8f2, blindno.fpe / blindno_fp_propagate).

PARITY UNPINNED: fplanck is absent, so the checks are the oracle's independent
cell-by-cell assembly of the same master equation (oracle/fpe_ref.py), its physical invariants
(mass conservation, Boltzmann stationary state, detailed balance), and on the GPU the batched
LDS-resident Taylor integrator against scipy.sparse.linalg.expm_multiply (rel-L2 <= 1e-9, fp64).
"""
import numpy as np
import pytest
import torch

from conftest import rel_l2

NM = 1e-9


def _sim2d(periodic_y=True, with_potential=True):
    from blindno import fpe
    kT = fpe.K_B * 300.0
    pot = (lambda x, y: 0.8 * kT * np.cos(2 * np.pi * x / (200 * NM)) * np.sin(np.pi * y / (240 * NM))) \
        if with_potential else None
    force = lambda x, y: np.array([3e-14 * np.sin(2 * np.pi * y / (240 * NM)) + 0 * x,   # noqa: E731
                                   -2e-14 * np.cos(2 * np.pi * x / (200 * NM)) + 0 * y])
    drag = lambda x, y: 1e-9 * (1.0 + 0.3 * np.exp(-(x ** 2 + y ** 2) / (80 * NM) ** 2))   # noqa: E731
    bnd = [fpe.boundary.reflecting, fpe.boundary.periodic if periodic_y else fpe.boundary.reflecting]
    return fpe.fokker_planck(temperature=300, drag=drag, extent=[200 * NM, 240 * NM], resolution=10 * NM,
                             potential=pot, force=force, boundary=bnd)


def _sim1d():
    from blindno import fpe
    kT = fpe.K_B * 300.0
    U = lambda x: 2.0 * kT * ((x / (250 * NM)) ** 2 - 1) ** 2    # noqa: E731  double well
    return fpe.fokker_planck(temperature=300, drag=2e-9, extent=800 * NM, resolution=10 * NM,
                             potential=U, boundary=fpe.boundary.reflecting)


def _dense_from_coefficients(sim):
    c = sim.coefficients()
    nx, ny = sim.grid_dims()
    N = nx * ny
    M = np.zeros((N, N))
    for i in range(N):
        ix, iy = divmod(i, ny)
        M[i, i] -= c[0, i]
        M[i, ((ix - 1) % nx) * ny + iy] += c[1, i]
        M[i, ((ix + 1) % nx) * ny + iy] += c[2, i]
        if sim.ndim == 2:
            M[i, ix * ny + (iy - 1) % ny] += c[3, i]
            M[i, ix * ny + (iy + 1) % ny] += c[4, i]
    return M


def _oracle_matrix(sim):
    from oracle import fpe_ref
    periodic = [b.name == "periodic" for b in sim.boundary]
    return fpe_ref.master_matrix(sim.potential_values, sim.force_values, sim.diffusion, sim.resolution,
                                 sim.beta, periodic)


@pytest.mark.parametrize("which", ["1d", "2d_periodic", "2d_reflecting"])
def test_rates_match_oracle_assembly(which):
    sim = _sim1d() if which == "1d" else _sim2d(periodic_y=(which == "2d_periodic"))
    M = _dense_from_coefficients(sim)
    Mo = _oracle_matrix(sim).toarray()
    assert np.abs(M - Mo).max() <= 1e-12 * np.abs(Mo).max()


def test_oracle_invariants():
    from oracle import fpe_ref
    sim = _sim2d()
    M = _oracle_matrix(sim)
    assert np.abs(np.asarray(M.sum(axis=0))).max() <= 1e-9 * abs(M.diagonal()).max()   # mass
    # potential only, reflecting: Boltzmann exp(-beta U) is stationary and detailed balance holds
    sim1 = _sim1d()
    M1 = _oracle_matrix(sim1).toarray()
    pb = np.exp(-sim1.beta * sim1.potential_values)
    pb /= pb.sum()
    assert np.abs(M1 @ pb).max() <= 1e-10 * np.abs(np.diag(M1)).max() * pb.max()
    flux = M1 * pb[None, :]                       # flux[j, i] = rate(i -> j) p_i
    off = flux - np.diag(np.diag(flux))
    assert np.abs(off - off.T).max() <= 1e-12 * np.abs(off).max()
    # expm_multiply keeps mass and relaxes toward Boltzmann
    p0 = np.exp(-((sim1.grid[0] + 250 * NM) / (40 * NM)) ** 2)
    p0 /= p0.sum()
    Pt = fpe_ref.propagate(_oracle_matrix(sim1), p0, 5.0, 3)
    assert abs(Pt[-1].sum() - 1.0) < 1e-10
    assert rel_l2(Pt[-1], pb) < rel_l2(Pt[0], pb)


def test_helpers():
    from blindno import fpe
    sim = _sim2d()
    f = fpe.potential_from_data(sim.grid, sim.force_values[0])
    assert np.allclose(f(*sim.grid), sim.force_values[0], rtol=1e-12, atol=0)
    x = np.linspace(-1, 1, 11)
    g = fpe.potential_from_data(x, x ** 2)
    assert np.allclose(g(x), x ** 2)
    pdf = fpe.gaussian_pdf(center=(0.1, -0.2), width=0.3)
    assert np.isclose(pdf(np.array(0.1), np.array(-0.2)), 1.0)
    with pytest.raises(Exception):
        sim.propagate_interval(fpe.gaussian_pdf(0.0, 1.0), 1e-3, Nsteps=3, device="cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("which,tf,nsteps", [("1d", 2.0, 41), ("2d_periodic", 0.05, 21),
                                             ("2d_reflecting", 0.02, 11)])
def test_gpu_propagation_matches_expm_multiply(which, tf, nsteps):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from blindno import fpe
    from oracle import fpe_ref
    sim = _sim1d() if which == "1d" else _sim2d(periodic_y=(which == "2d_periodic"))
    center = (-250 * NM,) if sim.ndim == 1 else (-50 * NM, 40 * NM)
    pdf = fpe.gaussian_pdf(center=center, width=30 * NM)
    t, Pt = sim.propagate_interval(pdf, tf, Nsteps=nsteps)
    assert np.allclose(t, np.linspace(0, tf, nsteps))
    p0 = pdf(*sim.grid).reshape(-1)
    p0 /= p0.sum()
    ref = fpe_ref.propagate(_oracle_matrix(sim), p0, tf, nsteps)
    got = Pt.reshape(nsteps, -1)
    assert rel_l2(got, ref) <= 1e-9, rel_l2(got, ref)
    assert np.abs(got.sum(axis=1) - 1.0).max() <= 1e-11


@pytest.mark.gpu
def test_gpu_batched_trajectories_match_single():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from blindno import fpe
    sims = [_sim2d(), _sim2d(with_potential=False), _sim2d(periodic_y=False)]
    pdfs = [fpe.gaussian_pdf(center=(c * NM, 0.0), width=30 * NM) for c in (-50, 0, 50)]
    many = fpe.propagate_many(sims, pdfs, 0.01, Nsteps=6)
    for sim, pdf, (t, Pt) in zip(sims, pdfs, many):
        t1, P1 = sim.propagate_interval(pdf, 0.01, Nsteps=6)
        # each trajectory keeps its own substep count (grouped launches): same result to 1e-12
        assert rel_l2(Pt, P1) <= 1e-12


def test_outlier_force_is_refused_before_launch():
    """A force far outside the physical range (rates ~ exp(beta W / 2)) would need an
    effectively unbounded number of Taylor substeps: propagate_many refuses it with a clear
    error before any launch, and a normal trajectory's substep count is its own."""
    from blindno import fpe
    from blindno._lib import BlindnoError
    ok = _sim2d()
    wild = fpe.fokker_planck(temperature=300, drag=1e-9, extent=[200 * NM, 240 * NM], resolution=10 * NM,
                             force=lambda x, y: [1e-11 + 0 * x, 0 * y], boundary=fpe.boundary.reflecting)
    dt = 0.01 / 5
    s_ok = fpe.substeps_for(ok.coefficients(), dt)
    assert s_ok < fpe.MAX_TOTAL_SUBSTEPS
    pdf = fpe.gaussian_pdf(center=(0.0, 0.0), width=30 * NM)
    with pytest.raises(BlindnoError, match="refusing to launch"):
        fpe.propagate_many([ok, wild], [pdf, pdf], 0.01, Nsteps=6, device="cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("gen,kw", [("fpe_1d_dataset", dict(nsteps=120, tf=2e-3)),
                                    ("fpe_2d_dataset", dict(nsteps=110, tf=2e-4)),
                                    ("fpe_2d_nc_dataset", dict(nsteps=105, tf=2e-3))])
def test_dataset_generators(gen, kw, tmp_path):
    """The reference generator scripts (1d_FPE/dataset_1d_drift_diffusion.py,
    2d_FPE/test_datagen.py, 2d_Non_conservative_FPE/testdata_gen.py) at M = 2 and a shortened
    time grid: reference keys and shapes, the numpy-RNG parameter order, mass conservation,
    and (1D) the trajectory against expm_multiply of the oracle matrix."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from blindno import datagen, fpe
    from oracle import fpe_ref
    np.random.seed(5)
    d = getattr(datagen, gen)(M=2, **kw)
    nt = kw["nsteps"]
    keys = {"time", "grid", "trajectories", "F"} if gen == "fpe_2d_nc_dataset" else \
        {"time", "grid", "trajectories", "potential", "drag"}
    assert set(d) == keys
    assert d["time"].shape == (2, 100) and d["trajectories"].shape[:2] == (2, 100)
    full_t = np.linspace(0, kw["tf"], nt)
    for k in range(2):
        assert np.all(np.diff(d["time"][k]) > 0) and np.all(np.isin(d["time"][k], full_t))
        assert np.abs(d["trajectories"][k].reshape(100, -1).sum(-1) - 1.0).max() < 1e-10
    datagen.save_npz(str(tmp_path / "ds.npz"), d)
    assert set(np.load(tmp_path / "ds.npz").files) == keys
    if gen == "fpe_1d_dataset":
        # RNG order: sample 0's wells and its recorded indices come first
        np.random.seed(5)
        while True:
            c = np.random.uniform(-150 * NM, 150 * NM, size=3)
            if all(abs(c[i] - c[j]) > 80 * NM for i in range(3) for j in range(i + 1, 3)):
                break
        w = np.random.uniform(20 * NM, 80 * NM, size=3)
        A = np.random.uniform(1e-20, 2e-20, size=3)
        vf = np.random.uniform(1, 2, size=1)
        sel = np.sort(np.random.choice(range(nt), size=100, replace=False))
        g = d["grid"][0][0]
        U = sum(-A[i] * vf[0] * np.exp(-((g - c[i]) / w[i]) ** 2) for i in range(3))
        assert np.allclose(d["potential"][0], U, rtol=1e-12, atol=0)
        assert np.isclose(d["drag"][0], datagen.DRAG * vf[0])
        assert np.array_equal(d["time"][0], full_t[sel])
        sim = fpe.fokker_planck(temperature=300, drag=d["drag"][0], extent=800 * NM, resolution=10 * NM,
                                potential=fpe.potential_from_data(g, U))
        p0 = np.exp(-(g / (50 * NM)) ** 2)
        ref = fpe_ref.propagate(_oracle_matrix(sim), p0 / p0.sum(), kw["tf"], nt)[sel]
        assert rel_l2(d["trajectories"][0], ref) <= 1e-9


def test_time_averaged_relative_l2_matches_reference_fixture():
    from blindno import timeerror
    from conftest import load_golden
    g = load_golden("metric_time_avg_rel_l2_2d")
    assert abs(timeerror.time_averaged_relative_l2(g["pt_pred"], g["pt_ref"]) - float(g["val"])) <= \
        1e-12 * abs(float(g["val"]))


@pytest.mark.gpu
def test_compute_time_error_pipeline(tmp_path):
    """2d_Non_conservative_FPE/compute_time_error.py as one batched pipeline vs the same steps
    run one trajectory at a time (predict, de-normalise, propagate true and predicted force)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import csv
    from blindno import NIOFP2D_FNO, evaluate, fpe, timeerror
    rs = np.random.RandomState(8)
    M, T, N = 3, 60, 80
    mk = lambda m: dict(trajectories=(rs.rand(m, T, N, N) * 1e-10).astype(np.float32),   # noqa: E731
                        F=(rs.randn(m, 2, N, N) * 1e-13).astype(np.float32))
    train, test = mk(4), mk(M)
    models = {}
    for name, seed in (("fno", 1), ("fno_b", 2)):
        torch.manual_seed(seed)
        models[name] = NIOFP2D_FNO(2, 3, 100, 25, 2, 6, 5, 2, heads=("fno_Fx", "fno_Fy")).cuda()
    kw = dict(nsteps=6, dt=1e-3)
    rows = timeerror.compute_time_error(models, train, test, range(0, 5), outdir=str(tmp_path), batch=2, **kw)
    assert [(r[0], r[1]) for r in rows] == [(i, n) for i in range(M) for n in models]
    st = evaluate.compute_train_stats("2d_Non_conservative_FPE", train)
    grid = timeerror.build_fokker_planck(lambda x, y: np.array([0 * x, 0 * y])).grid
    pdf = fpe.gaussian_pdf(center=(-150 * NM, -150 * NM), width=30 * NM)
    for r in rows[:2]:
        i, name = r[0], r[1]
        x = torch.tensor(evaluate.normalize_input(test["trajectories"][i], st)[None], device="cuda")
        pred = evaluate.predict(models[name], x, evaluate.grid2d(N, N, "cuda")).cpu().numpy()[0]
        pa, pb = evaluate.denormalize("2d_Non_conservative_FPE", pred, st)
        F = test["F"][i]
        assert abs(r[2] - evaluate.rel_l2(pa, F[0])) <= 1e-6 * r[2]
        _, Pref = timeerror.build_fokker_planck(timeerror.force_from_array(grid, F[0], F[1])) \
            .propagate_interval(pdf, kw["dt"], Nsteps=kw["nsteps"])
        _, Ppred = timeerror.build_fokker_planck(timeerror.force_from_array(grid, pa, pb)) \
            .propagate_interval(pdf, kw["dt"], Nsteps=kw["nsteps"])
        e = timeerror.time_averaged_relative_l2(Ppred, Pref)
        # the batched launch shares the stiffest trajectory's substep count: agreement ~1e-9
        assert abs(r[4] - e) <= 1e-6 * e + 1e-12
    with open(tmp_path / "metrics_all.csv") as f:
        got = list(csv.reader(f))
    assert got[0] == ["index", "model", "rel_l2_Fx", "rel_l2_Fy", "ErrL2_density"] and len(got) == 1 + 2 * M


@pytest.mark.gpu
def test_compute_time_error_gpe_pipeline(tmp_path):
    """1d_GPE/compute_time_error_GPE.py as one batched pipeline vs per-trajectory
    solve_GPE_custom + time_averaged_L2_error (GPE solver pinned by gpe_solve_* goldens)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from blindno import NIOFP_FNO, evaluate, gpe, timeerror
    rs = np.random.RandomState(9)
    T, N = 101, 128
    mk = lambda m: dict(y=rs.rand(m, T, N), V=rs.rand(m, N) * 3, g=rs.rand(m), kappa=rs.rand(m) * 0.1)  # noqa: E731
    train, test = mk(4), mk(3)
    models = {}
    for name, seed in (("fno", 1), ("fno_b", 2)):
        torch.manual_seed(seed)
        models[name] = NIOFP_FNO(3, 20, 40, 1, "cpu", heads=("fno_V",)).cuda()
    kw = dict(t_final=0.5, dt=0.005)
    errs = timeerror.compute_time_error_gpe(models, train, test, [2, 0, 7], outdir=str(tmp_path), **kw)
    assert list(errs) == ["fno", "fno_b"] and errs["fno"].shape == (2,)
    sc = evaluate.compute_train_scalers_gpe(train)
    tn = evaluate.normalize_gpe(test, sc)
    x = np.linspace(-10, 10, N)
    i = 2
    pv = evaluate.predict(models["fno_b"], torch.tensor(tn["y"][i][None], dtype=torch.float32, device="cuda"),
                          torch.linspace(0, 1, N, device="cuda").unsqueeze(-1)).cpu().numpy()[0, :, 0] * sc["V_max"]
    ic = lambda xx: gpe.initial_condition(2, xx)   # noqa: E731
    t, pr = gpe.solve_GPE_custom(ic, x, kw["dt"], kw["t_final"], 2, test["g"][i], test["kappa"][i],
                                 tn["V"][i] * sc["V_max"])
    _, pp = gpe.solve_GPE_custom(ic, x, kw["dt"], kw["t_final"], 2, test["g"][i], test["kappa"][i], pv)
    e = gpe.time_averaged_L2_error(t, np.abs(pr), t, np.abs(pp), x)
    assert abs(errs["fno_b"][0] - e) <= 1e-9 * e + 1e-15
    d = np.load(tmp_path / "fno" / "sample_0_V_and_err.npy", allow_pickle=True).item()   # our own file
    assert d["Err_L2_rel"] == errs["fno"][1]
    assert np.load(tmp_path / "ErrL2_relative_fno_Nsamples_2.npy").shape == (2,)


@pytest.mark.gpu
def test_compute_time_error_1d_pipeline(tmp_path):
    """1d_FPE/compute_time_error.py as one batched pipeline vs per-trajectory propagation."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from blindno import NIOFP_FNO, evaluate, fpe, gpe, timeerror
    rs = np.random.RandomState(10)
    T, N = 100, 80
    kT = fpe.K_B * 300
    mk = lambda m: dict(trajectories=(rs.rand(m, T, N) * 1e-5).astype(np.float32),   # noqa: E731
                        potential=(rs.randn(m, N) * 0.3 * kT).astype(np.float32),
                        drag=(rs.rand(m) * 1e-9 + 1e-9).astype(np.float32))
    train, test = mk(5), mk(3)
    models = {}
    for name, seed in (("fno", 1), ("fno_b", 2)):
        torch.manual_seed(seed)
        models[name] = NIOFP_FNO(3, 6, 5, 2, "cpu").cuda()
    kw = dict(nsteps=11, dt=2e-4)
    errs = timeerror.compute_time_error_1d(models, train, test, [1, 2], outdir=str(tmp_path), **kw)
    st = evaluate.compute_train_stats_1d(train)
    i = 1
    x = torch.tensor(evaluate.normalize_input_1d(test["trajectories"][i], st)[None], device="cuda")
    p = evaluate.predict(models["fno"], x, torch.linspace(0, 1, N, device="cuda").unsqueeze(-1)).cpu().numpy()[0]
    pot, drg = evaluate.denormalize_1d(p, st)

    def sim(U, drag):
        s0 = fpe.fokker_planck(temperature=300, drag=drag, extent=800 * NM, resolution=10 * NM)
        return fpe.fokker_planck(temperature=300, drag=drag, extent=800 * NM, resolution=10 * NM,
                                 potential=fpe.potential_from_data(s0.grid[0], U))
    pdf = fpe.gaussian_pdf(center=0.0, width=50 * NM)
    t, Pr = sim(test["potential"][i].astype(np.float64), float(test["drag"][i])).propagate_interval(pdf, kw["dt"], Nsteps=kw["nsteps"])
    _, Pp = sim(pot, float(drg.mean())).propagate_interval(pdf, kw["dt"], Nsteps=kw["nsteps"])
    e = gpe.time_averaged_L2_error(t, Pr, t, Pp, sim(pot, 1e-9).grid)
    assert abs(errs["fno"][0] - e) <= 1e-6 * e + 1e-15
    assert np.load(tmp_path / "fno_b" / "pred_sample_2.npy").shape == (N, 2)
    assert np.load(tmp_path / "ErrL2_fno_Nsamples_2.npy").shape == (2,)
