"""The eval_fno.py path (blindno.evaluate): host math pinned to the reference's own functions
(golden eval_2d_*.npz from tests/golden/make_golden_eval.py), checkpoint loading, and the
batched GPU evaluation against the float64 oracle run sample by sample, as the reference
loops (GPU part marked)."""
import csv
import os

import numpy as np
import pytest
import torch

from conftest import load_golden

KINDS = [("2d_FPE", "eval_2d_fpe"), ("2d_Non_conservative_FPE", "eval_2d_nc")]


def _split(g, prefix):
    return {k[len(prefix):]: v for k, v in g.items() if k.startswith(prefix)}


@pytest.mark.parametrize("kind,case", KINDS)
def test_host_math_matches_reference(kind, case):
    from blindno import evaluate as ev
    g = load_golden(case)
    st = ev.compute_train_stats(kind, _split(g, "train."))
    ref = _split(g, "stats.")
    assert sorted(st) == sorted(ref)
    for k in ref:
        assert np.array_equal(st[k], ref[k]), k
    te = _split(g, "test.")
    for i in range(2):
        assert np.array_equal(ev.normalize_input(te["trajectories"][i], st), g[f"x_norm{i}"])
        pa, pb = ev.denormalize(kind, g["pred"][i], st)
        assert np.array_equal(pa, g[f"pred_a{i}"]) and np.array_equal(pb, g[f"pred_b{i}"])
        ta, tb = ev.true_fields(kind, te, i, st)
        assert np.array_equal(ta, g[f"true_a{i}"]) and np.array_equal(tb, g[f"true_b{i}"])
        assert ev.rel_l2(pa, ta) == float(g[f"rel_a{i}"])
        assert ev.rel_l2(pb, tb) == float(g[f"rel_b{i}"])


def test_checkpoint_robust_loading(tmp_path):
    from blindno import evaluate as ev
    sd = {"module.fc0.weight": torch.ones(2, 3), "module.fc0.bias": torch.zeros(2)}
    p1, p2 = tmp_path / "a.pt", tmp_path / "b.pt"
    torch.save(sd, p1)
    torch.save({"state_dict": sd, "epoch": 3}, p2)
    for p in (p1, p2):
        out = ev.load_checkpoint_robust(str(p))
        assert list(out) == ["fc0.weight", "fc0.bias"]
    torch.save([1, 2], tmp_path / "c.pt")
    with pytest.raises(RuntimeError):
        ev.load_checkpoint_robust(str(tmp_path / "c.pt"))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["2d_FPE", "2d_Non_conservative_FPE"])
def test_batched_gpu_eval_matches_per_sample_oracle(kind, tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import oracle
    from blindno import NIOFP2D_FNO
    from blindno import evaluate as ev
    heads = ("fno_drift", "fno_diffusion") if kind == "2d_FPE" else ("fno_Fx", "fno_Fy")
    rs = np.random.RandomState(3)
    M, T, N = 6, 60, 20
    mk = (lambda m: dict(trajectories=(rs.rand(m, T, N, N) * 1e-10).astype(np.float32),
                         potential=(rs.randn(m, N, N) * 1e-21).astype(np.float32),
                         drag=(rs.rand(m, N, N) * 1e-6).astype(np.float32))) if kind == "2d_FPE" else \
         (lambda m: dict(trajectories=(rs.rand(m, T, N, N) * 1e-10).astype(np.float32),
                         F=(rs.randn(m, 2, N, N) * 1e-12).astype(np.float32)))
    train, test = mk(M), mk(5)
    torch.manual_seed(2)
    m = NIOFP2D_FNO(2, 3, 100, 25, 2, 6, 5, 2, heads=heads).cuda()
    rows = ev.evaluate(kind, m, train, test, range(-1, 7), outdir=str(tmp_path), batch=2)
    assert [r[0] for r in rows] == [0, 1, 2, 3, 4]            # out-of-range indices skipped
    assert m.training                                          # mode restored
    st = ev.compute_train_stats(kind, train)
    p = {k: v.detach().cpu().double() for k, v in m.state_dict().items() if not k.startswith("branch.")}
    grid = ev.grid2d(N, N, "cpu")
    for r in rows:
        i = r[0]
        x = torch.tensor(ev.normalize_input(test["trajectories"][i], st)[None])
        ref = oracle.niofp2d_fno(p, x, grid, idx=None, heads=heads)[0].numpy().astype(np.float32)
        ra, rb = ev.denormalize(kind, ref, st)
        ta, tb = ev.true_fields(kind, test, i, st)
        assert abs(r[1] - ev.rel_l2(ra, ta)) <= 1e-5 * abs(ev.rel_l2(ra, ta))
        assert abs(r[2] - ev.rel_l2(rb, tb)) <= 1e-5 * abs(ev.rel_l2(rb, tb))
    with open(tmp_path / "metrics.csv") as f:
        got = list(csv.reader(f))
    assert got[0] == ev.KINDS[kind]["header"] and len(got) == 6
    d = np.load(tmp_path / "sample_0003_predictions.npy", allow_pickle=True).item()   # our own file
    assert d["index"] == 3 and d[f"{ev.KINDS[kind]['fields'][0]}_pred"].shape == (N, N)
    assert os.path.exists(tmp_path / "sample_0000_predictions.npy")


def test_host_math_1d_matches_reference():
    from blindno import evaluate as ev
    g = load_golden("eval_1d_fpe")
    st = ev.compute_train_stats_1d(_split(g, "train."))
    ref = _split(g, "stats.")
    assert sorted(st) == sorted(ref)
    for k in ref:
        assert np.array_equal(st[k], ref[k]), k
    assert np.array_equal(ev.normalize_input_1d(g["test_traj"], st), g["x_norm"])
    pot, drg = ev.denormalize_1d(g["pred"], st)
    assert np.array_equal(pot, g["pot"]) and np.array_equal(drg, g["drg"])


@pytest.mark.gpu
def test_batched_gpu_eval_1d_matches_per_sample_oracle(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import oracle
    from blindno import NIOFP_FNO
    from blindno import evaluate as ev
    rs = np.random.RandomState(4)
    T, N = 100, 80
    mk = lambda m: dict(trajectories=(rs.rand(m, T, N) * 1e-5).astype(np.float32),   # noqa: E731
                        potential=(rs.randn(m, N) * 1e-20).astype(np.float32),
                        drag=(rs.rand(m) * 1e-5).astype(np.float32))
    train, test = mk(6), mk(5)
    torch.manual_seed(3)
    m = NIOFP_FNO(3, 6, 5, 2, "cpu").cuda()
    rows = ev.evaluate_1d_fpe(m, train, test, range(0, 9), outdir=str(tmp_path), batch=2)
    assert [r[0] for r in rows] == [0, 1, 2, 3, 4]
    st = ev.compute_train_stats_1d(train)
    p = {k: (v.detach().cpu().to(torch.complex128) if v.is_complex() else v.detach().cpu().double())
         for k, v in m.state_dict().items()}
    grid = torch.linspace(0, 1, N).unsqueeze(-1)
    for r in rows:
        i = r[0]
        x = torch.tensor(ev.normalize_input_1d(test["trajectories"][i], st)[None])
        ref = oracle.niofp_fno(p, x, grid, idx=None)[0].numpy().astype(np.float32)
        pot, drg = ev.denormalize_1d(ref, st)
        assert abs(r[1] - float(drg.mean())) <= 1e-4 * abs(float(drg.mean())) + 1e-12
        assert abs(r[3] - ev.rel_l2(pot, test["potential"][i])) <= 1e-4 * ev.rel_l2(pot, test["potential"][i])
        assert r[2] == float(test["drag"][i])
    assert np.load(tmp_path / "pred_sample_3.npy").shape == (N, 2)


@pytest.mark.gpu
def test_batched_gpu_eval_gpe_matches_per_sample_oracle(tmp_path):
    """1d_GPE/eval_fno_GPE.py: divide-by-max scalers, NIOFP_FNO(3, 20, 40, 1) head fno_V."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import oracle
    from blindno import NIOFP_FNO
    from blindno import evaluate as ev
    rs = np.random.RandomState(6)
    T, N = 101, 128
    mk = lambda m: dict(y=rs.rand(m, T, N), V=rs.rand(m, N) * 3, g=rs.rand(m), kappa=rs.rand(m))   # noqa: E731
    train, test = mk(5), mk(4)
    torch.manual_seed(4)
    m = NIOFP_FNO(3, 20, 40, 1, "cpu", heads=("fno_V",)).cuda()
    rows = ev.evaluate_1d_gpe(m, train, test, range(0, 4), outdir=str(tmp_path), batch=3)
    sc = ev.compute_train_scalers_gpe(train)
    assert sc["V_max"] == train["V"].max() / 3.0 and sc["g_max"] == train["g"].max()
    tn = ev.normalize_gpe(test, sc)
    p = {k: (v.detach().cpu().to(torch.complex128) if v.is_complex() else v.detach().cpu().double())
         for k, v in m.state_dict().items()}
    grid = torch.linspace(0, 1, N).unsqueeze(-1)
    for r in rows:
        i = r[0]
        ref = oracle.niofp_fno(p, torch.tensor(tn["y"][i][None]), grid, idx=None, heads=("fno_V",))
        pv = ref[0, :, 0].numpy().astype(np.float32) * sc["V_max"]
        e = ev.rel_l2(pv, tn["V"][i] * sc["V_max"])
        assert abs(r[1] - e) <= 1e-4 * e
    d = np.load(tmp_path / "sample_pred_V_2.npy", allow_pickle=True).item()   # our own file
    assert d["pred_V"].shape == (N,) and d["V_max_used"] == sc["V_max"]


@pytest.mark.gpu
def test_cli_1d_fpe(tmp_path):
    """python -m blindno.evaluate --experiment 1d_FPE: reference-size NIOFP_FNO(3, 30, 15, 2)
    checkpoint with the DDP 'module.' prefix, npz train/test files, per-sample outputs."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from blindno import NIOFP_FNO
    from blindno import evaluate as ev
    rs = np.random.RandomState(12)
    T, N = 100, 80
    for name, m in (("train", 4), ("test", 3)):
        np.savez(tmp_path / f"{name}.npz", trajectories=(rs.rand(m, T, N) * 1e-5).astype(np.float32),
                 potential=(rs.randn(m, N) * 1e-20).astype(np.float32), drag=(rs.rand(m) * 1e-5).astype(np.float32))
    torch.manual_seed(0)
    m = NIOFP_FNO(3, 30, 15, 2, "cpu")
    torch.save({"module." + k: v for k, v in m.state_dict().items()}, tmp_path / "ckpt.pt")
    ev.main(["--experiment", "1d_FPE", "--train_data", str(tmp_path / "train.npz"),
             "--test_data", str(tmp_path / "test.npz"), "--ckpt", str(tmp_path / "ckpt.pt"),
             "--outdir", str(tmp_path / "out"), "--start", "0", "--end", "5", "--strict"])
    for i in range(3):
        assert np.load(tmp_path / "out" / f"pred_sample_{i}.npy").shape == (N, 2)


@pytest.mark.gpu
def test_cli_unet_2d_and_1d(tmp_path):
    """eval_unet.py / eval_unet_bag.py through the CLI (--model PermInvUNet_attn*): a
    module.-prefixed UNet checkpoint drives the batched eval; the 2D predictions match the
    model's own eval-mode forward on the de-normalisation-free metric rows."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from blindno import evaluate as ev
    from blindno import unet
    rs = np.random.RandomState(5)
    T, N = 60, 52
    for name, m in (("train", 4), ("test", 3)):
        np.savez(tmp_path / f"{name}.npz", trajectories=np.abs(rs.randn(m, T, N, N)).astype(np.float32) * 1e-10,
                 potential=(rs.randn(m, N, N) * 1e-21).astype(np.float32),
                 drag=((1 + 0.1 * rs.randn(m, N, N)) * 1e-6).astype(np.float32))
    torch.manual_seed(0)
    m = unet.PermInvUNet_attn(1, 2, 1, 4, (N, N))
    torch.save({"module." + k: v for k, v in m.state_dict().items()}, tmp_path / "u.pt")
    ev.main(["--experiment", "2d_FPE", "--model", "PermInvUNet_attn", "--train_data", str(tmp_path / "train.npz"),
             "--test_data", str(tmp_path / "test.npz"), "--ckpt", str(tmp_path / "u.pt"), "--nx", str(N),
             "--ny", str(N), "--outdir", str(tmp_path / "out2"), "--start", "0", "--end", "2", "--strict"])
    assert os.path.exists(tmp_path / "out2" / "metrics.csv")
    T1, N1 = 100, 80
    for name, k in (("train", 4), ("test", 3)):
        np.savez(tmp_path / f"{name}1.npz", trajectories=(rs.rand(k, T1, N1) * 1e-5).astype(np.float32),
                 potential=(rs.randn(k, N1) * 1e-20).astype(np.float32), drag=(rs.rand(k) * 1e-5).astype(np.float32))
    m1 = unet.PermInvUNet_attn1D_bag(1, 2, 1, 4, 80, device="cpu")
    torch.save(m1.state_dict(), tmp_path / "u1.pt")
    ev.main(["--experiment", "1d_FPE", "--model", "PermInvUNet_attn1D_bag", "--train_data",
             str(tmp_path / "train1.npz"), "--test_data", str(tmp_path / "test1.npz"), "--ckpt",
             str(tmp_path / "u1.pt"), "--outdir", str(tmp_path / "out1"), "--start", "0", "--end", "2", "--strict"])
    for i in range(3):
        assert np.load(tmp_path / "out1" / f"pred_sample_{i}.npy").shape == (N1, 2)
