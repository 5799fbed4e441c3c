"""The native training entry (blindno.trainer: the reference's train_*.py loops on the fast
path -- HIP graphs, flat fused Adam, DataParallel) end to end on tiny synthetic datasets
(needs a GPU): epochs run, eval every save_interval epochs with the reference metric, the best
checkpoint is written (previous one deleted) and loads into blindno.evaluate, loss .npy files
match the reference's names and lengths."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import blindno
    blindno.load_library()


def _npz_2d(path, M=10, T=60, N=61, seed=0):
    rs = np.random.RandomState(seed)
    traj = np.abs(rs.randn(M, T, N, N)).astype(np.float32) * 1e-10
    pot = rs.randn(M, N, N).astype(np.float32) * 1e-21
    drag = (1.0 + 0.1 * rs.randn(M, N, N)).astype(np.float32) * 1e-6
    np.savez(path, trajectories=traj, potential=pot, drag=drag)


def test_trainer_2d_fpe_epochs_checkpoint_and_eval(tmp_path):
    from blindno import evaluate, trainer
    data = str(tmp_path / "ds.npz")
    _npz_2d(data)
    out = str(tmp_path / "result_2d_fno")
    exp = trainer._experiments()["2d_FPE"]
    logs = []
    t = trainer.Trainer(exp, data, out, torch.device("cuda"), epochs=3, save_interval=1, log=logs.append)
    hist = t.fit()
    assert len(t.train_idx) == 8 and len(t.test_idx) == 2
    assert len(hist["train_losses"]) == 3 and len(hist["test_losses"]) == 3
    assert all(np.isfinite(v) for v in hist["train_losses"] + hist["test_losses"])
    for k in ("train_losses", "test_losses", "test_losses_drift", "test_losses_diffusion"):
        assert np.load(os.path.join(out, k + ".npy")).shape == (len(hist[k]),)
    ckpts = [f for f in os.listdir(out) if f.startswith("model_checkpoint_best_")]
    assert len(ckpts) == 1, ckpts                           # previous best deleted
    assert ckpts[0] == f"model_checkpoint_best_{min(hist['test_losses']):.6f}.pt"
    assert any(s.startswith("Epoch 3/3, Train Loss:") for s in logs)
    # the checkpoint drives the reference's eval path (eval_fno.py)
    model = exp.model(61, "cuda")
    sd = evaluate.load_checkpoint_robust(os.path.join(out, ckpts[0]))
    model.load_state_dict(sd)
    model = model.cuda()
    rows = evaluate.evaluate("2d_FPE", model, data, data, range(0, 2), outdir=str(tmp_path / "eval"), batch=2,
                             device="cuda")
    assert len(rows) == 2 and all(np.isfinite(r[1]) and np.isfinite(r[2]) for r in rows)
    assert os.path.exists(tmp_path / "eval" / "metrics.csv")


def test_trainer_1d_gpe(tmp_path):
    from blindno import trainer
    rs = np.random.RandomState(1)
    M, T, N = 12, 60, 128
    d = {"y": np.abs(rs.randn(M, T, N)), "g": rs.rand(M), "kappa": rs.rand(M), "V": rs.rand(M, N)}
    data = str(tmp_path / "gpe.npy")
    np.save(data, d, allow_pickle=True)
    out = str(tmp_path / "results_GPE_fno")
    exp = trainer._experiments()["1d_GPE"]
    t = trainer.Trainer(exp, data, out, torch.device("cuda"), epochs=2, save_interval=2, batch=4,
                        log=lambda s: None)
    hist = t.fit()
    # 9 train samples at batch 4: two graphed steps and one partial (eager) batch per epoch
    assert len(t.train_idx) == 9 and len(hist["train_losses"]) == 2 and len(hist["test_losses"]) == 1
    assert sorted(os.listdir(out)) == sorted([f"model_checkpoint_best_{hist['test_losses'][0]:.6f}.pt",
                                              "test_losses.npy", "train_losses.npy"])


def test_trainer_unet_2d(tmp_path):
    """train_unet.py's loop (2d_FPE/train_unet.py:124-200) on the attention UNet through the
    native trainer: graphed epochs, the two-channel metric, best checkpoint in result_unet."""
    from blindno import trainer
    data = str(tmp_path / "ds.npz")
    _npz_2d(data, M=10, T=60, N=52)
    out = str(tmp_path / "result_unet")
    exp = trainer._experiments("unet")["2d_FPE"]
    t = trainer.Trainer(exp, data, out, torch.device("cuda"), epochs=2, save_interval=1, log=lambda s: None)
    hist = t.fit()
    assert len(hist["train_losses"]) == 2 and all(np.isfinite(hist["train_losses"]))
    ckpts = [f for f in os.listdir(out) if f.startswith("model_checkpoint_best_")]
    assert ckpts == [f"model_checkpoint_best_{min(hist['test_losses']):.6f}.pt"]
    sd = torch.load(os.path.join(out, ckpts[0]), weights_only=True)
    m = exp.model(52, "cuda")
    m.load_state_dict(sd)


def test_trainer_nio_2d(tmp_path):
    """train_nio.py's loop (2d_FPE/train_nio.py:62-267: NIOFP2D with the Encoder2D branch, bs 4,
    lr 5e-4, StepLR, best checkpoint in result_2d_nio) through the native trainer: one HIP graph
    per drawn bag size L (the branch's train-mode BatchNorm takes its statistics over the bag
    with its repeats, so no deduplication), the two-channel metric, all four loss files."""
    from blindno import trainer
    data = str(tmp_path / "ds.npz")
    _npz_2d(data, M=10, T=56, N=61)
    out = str(tmp_path / "result_2d_nio")
    exp = trainer._experiments("nio")["2d_FPE"]
    assert exp.result_dir == "result_2d_nio" and exp.lr == 5e-4 and exp.batch == 4
    t = trainer.Trainer(exp, data, out, torch.device("cuda"), epochs=2, save_interval=1, log=lambda s: None)
    assert not t.graphed.dedup
    # the NIO scripts train the branch CNN (2d_FPE/train_nio.py:115: Adam(model.parameters()));
    # only fc0 (read through .data) stays out of the optimizer
    names = {id(p): k for k, p in t.model.named_parameters()}
    trained = {names[id(p)] for p in t.opt.params}
    assert any(k.startswith("branch.") for k in trained) and not any(k.startswith("fc0.") for k in trained)
    w0 = t.model.branch.convblock1.layers[0].weight.detach().clone()
    lin0 = t.model.branch.linear.weight.detach().clone()
    hist = t.fit()
    assert not torch.equal(w0, t.model.branch.convblock1.layers[0].weight.detach())
    assert not torch.equal(lin0, t.model.branch.linear.weight.detach())
    assert len(hist["train_losses"]) == 2 and all(np.isfinite(hist["train_losses"]))
    assert all(np.isfinite(hist["test_losses"]))
    for k in ("train_losses", "test_losses", "test_losses_drift", "test_losses_diffusion"):
        assert np.load(os.path.join(out, k + ".npy")).shape == (2,)
    ckpts = [f for f in os.listdir(out) if f.startswith("model_checkpoint_best_")]
    assert ckpts == [f"model_checkpoint_best_{min(hist['test_losses']):.6f}.pt"]
    sd = torch.load(os.path.join(out, ckpts[0]), weights_only=True)
    m = exp.model(61, "cuda")
    m.load_state_dict(sd)


@pytest.mark.parametrize("shape", [(7, 13, 16, 16), (5, 3, 9)])
def test_batch_select_matches_index_select(shape):
    """train.BatchSelect (blindno_gather_batch: the bags and targets of the step's batch in one
    launch) is bit-identical to torch.index_select for the aligned (16-B) and unaligned row
    paths, with repeated and out-of-order ids."""
    from blindno.train import BatchSelect
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.randn(*shape, device="cuda", generator=g)
    Y = torch.randn(shape[0], 6, 2, device="cuda", generator=g)
    ids = torch.tensor([4, 0, 4, shape[0] - 1], dtype=torch.int64, device="cuda")
    xb = torch.full((4,) + tuple(shape[1:]), float("nan"), device="cuda")
    yb = torch.full((4, 6, 2), float("nan"), device="cuda")
    BatchSelect([X, Y], [xb, yb])(ids)
    torch.cuda.synchronize()
    assert torch.equal(xb, torch.index_select(X, 0, ids))
    assert torch.equal(yb, torch.index_select(Y, 0, ids))
    # an id past the source's rows (or negative) fills its batch row with NaN, the others intact
    bad = torch.tensor([1, shape[0], 2, -1], dtype=torch.int64, device="cuda")
    BatchSelect([X, Y], [xb, yb])(bad)
    torch.cuda.synchronize()
    assert torch.equal(xb[0], X[1]) and torch.equal(xb[2], X[2]) and torch.equal(yb[2], Y[2])
    assert bool(torch.isnan(xb[1]).all()) and bool(torch.isnan(xb[3]).all())
    assert bool(torch.isnan(yb[1]).all()) and bool(torch.isnan(yb[3]).all())
