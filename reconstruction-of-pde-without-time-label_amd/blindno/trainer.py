"""Native training entry on the fast path: the reference's ``train_*.py`` loops, run on HIP
graphs (``train.GraphedBagStep``), the fused flat Adam (``train.FlatAdam``) and data-parallel
RCCL gradient averaging (``train.DataParallel``).

    python -m blindno.trainer --experiment 2d_FPE --data dataset.npz [--epochs 400] [--outdir ...]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m blindno.trainer --experiment 2d_FPE ...

Reference loops (one per experiment; the flat module-level scripts):
  2d_FPE/train_fno.py:62-270               NIOFP2D_FNO(2,3,100,25,3,12,32,2), bs 4, lr 5e-4,
                                            eval every 5 epochs, result_2d_fno/
  2d_Non_conservative_FPE/train_fno.py     same with heads fno_Fx/fno_Fy (npz key F)
  1d_FPE/train_fno.py:59-191               NIOFP_FNO(3,30,15,2), bs 32, lr 1e-3, eval every 10,
                                            results_fno/
  1d_GPE/train_fno_GPE.py:75-205           NIOFP_FNO(3,20,40,1) head fno_V, bs 32, lr 1e-3,
                                            eval every 10, results_GPE_fno/
  --model nio (the DeepONet-branch NIO, train_nio*.py):
  2d_FPE/train_nio.py:62-267 and            NIOFP2D(2,3,100,25,3,12,32,2) (NC: heads fno_Fx/fno_Fy),
  2d_Non_conservative_FPE/train_nio.py:      bs 4, lr 5e-4, eval every 5, result_2d_nio/
    60-236
  1d_FPE/train_nio.py:60-200                NIOFP(1,3,100,25,3,30,15,2), bs 32, lr 1e-3, eval every
                                            10, results_nio/
  1d_GPE/train_nio_GPE.py:80-212            NIOFP_schrodinger(1,3,100,25,3,20,40,1), bs 32, lr 1e-3,
                                            eval every 10, results_GPE_nio/

What is kept from the reference, exactly:
  * dataset scaling / z-scoring (``blindno.data``, bit-pinned to the reference classes) and the
    80/20 ``random_split`` (2d_FPE/train_fno.py:67-69).  The reference splits before it seeds,
    from torch's default generator, whose initial seed is drawn per process in this torch build
    -- so the reference's split differs run to run; here it is ``random_split`` with a generator
    seeded ``--split-seed`` (default 0), reproducible;
  * seeds ``seed + rank`` for numpy / torch (2d_FPE/train_fno.py:78-81), so the numpy bag draw
    L = randint(50, T), idx = choice(T, L) of every train-mode forward is the reference's;
  * MSE loss, Adam(lr), StepLR(100, 0.5) per epoch -- under DDP stepped ``world`` times per call
    as accelerate does (accelerate/scheduler.py:69-76; ``--scheduler-mode per-epoch`` to turn
    the quirk off);
  * train loss = sum(loss x batch) / len(train split) (the local shard's sum under DDP);
  * eval every ``save_interval`` epochs in eval mode (L = T), per-sample relative L2 with the
    2D/1D-FPE two-channel denominator quirk (2d_FPE/train_fno.py:156-163) or the GPE per-sample
    rel-L2 (1d_GPE/train_fno_GPE.py:144-148), summed over the local test shard and divided by
    len(test split) (2d_FPE/train_fno.py:164-166; ``--eval-mode global`` all-reduces instead);
  * best checkpoint ``model_checkpoint_best_{loss:.6f}.pt`` = the model's state_dict (keys
    ``module.``-prefixed under DDP, as accelerate.save of the DDP model), previous best deleted;
  * ``train_losses.npy`` / ``test_losses.npy`` (+ ``test_losses_drift/diffusion.npy`` where the
    reference writes them).
Collectives run on every rank or on none (no rank-0-only forward: SURVEY.md section 5).  The
loss-curve / field PNGs (matplotlib) are not produced.
"""
from __future__ import annotations

import argparse
import math
import os
import sys
from dataclasses import dataclass, field
from typing import Callable, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

SPLIT_SEED = 0


@dataclass
class Experiment:
    name: str
    dim: int
    dataset: Callable
    model: Callable                       # (grid n, device) -> nn.Module
    lr: float
    batch: int
    save_interval: int
    result_dir: str
    two_channel_metric: bool
    loss_files: Sequence[str] = field(default_factory=lambda: ("train_losses", "test_losses"))
    # parameters the reference never trains: the FNO-NIO models' unused ``branch`` and their
    # ``fc0`` read through ``.data``; the NIO models train their branch CNN (2d_FPE/train_nio.py:115,
    # 1d_FPE/train_nio.py:96: Adam(model.parameters())), so only fc0 is excluded there
    exclude_prefixes: Sequence[str] = ("branch.", "fc0.")


def _experiments(model: str = "fno"):
    """The reference's train_*.py configurations.  ``model="unet"``: the attention-UNet scripts
    (2d_FPE/train_unet.py:62-110, 2d_Non_conservative_FPE/train_unet.py:60-110,
    1d_FPE/train_unet_bag.py:61-92, 1d_GPE/train_unet_GPE.py:80-110): same loop, metric quirk
    and best-checkpoint rule as train_fno.py, their own model / lr / batch / result directory.
    ``model="nio"``: the DeepONet-branch NIO scripts (train_nio*.py, module docstring); the
    branch's train-mode BatchNorm takes its statistics over the drawn bag with its repeats, so
    these graphs are keyed by the drawn L (no deduplication)."""
    from . import data, nio, unet
    from .encoders import Encoder2D
    all4 = ("train_losses", "test_losses", "test_losses_drift", "test_losses_diffusion")
    if model == "nio":
        def nio2d(heads):
            return lambda n, dev: nio.NIOFP2D(2, 3, 100, 25, 3, 12, 32, 2, heads=heads,
                                              branch_last_kernel=Encoder2D.kernel_for_grid(n))
        return {
            "2d_FPE": Experiment("2d_FPE", 2, data.TrajectoryDataset2D, nio2d(("fno_drift", "fno_diffusion")),
                                 5e-4, 4, 5, "result_2d_nio", True, all4, ("fc0.",)),
            "2d_Non_conservative_FPE": Experiment(
                "2d_Non_conservative_FPE", 2, data.TrajectoryDataset2DForce, nio2d(("fno_Fx", "fno_Fy")),
                5e-4, 4, 5, "result_2d_nio", True, all4, ("fc0.",)),
            "1d_FPE": Experiment("1d_FPE", 1, data.TrajectoryDataset1D,
                                 lambda n, dev: nio.NIOFP(1, 3, 100, 25, 3, 30, 15, 2, dev), 1e-3, 32, 10,
                                 "results_nio", True, all4, ("fc0.",)),
            "1d_GPE": Experiment("1d_GPE", 1, data.ParameterDataset,
                                 lambda n, dev: nio.NIOFP_schrodinger(1, 3, 100, 25, 3, 20, 40, 1, dev), 1e-3,
                                 32, 10, "results_GPE_nio", False, exclude_prefixes=("fc0.",)),
        }
    if model == "unet":
        all4 = ("train_losses", "test_losses", "test_losses_drift", "test_losses_diffusion")
        return {
            "2d_FPE": Experiment("2d_FPE", 2, data.TrajectoryDataset2D,
                                 lambda n, dev: unet.PermInvUNet_attn(1, 2, 1, 4, (n, n)), 5e-4, 4, 5,
                                 "result_unet", True, all4),
            "2d_Non_conservative_FPE": Experiment(
                "2d_Non_conservative_FPE", 2, data.TrajectoryDataset2DForce,
                lambda n, dev: unet.PermInvUNet_attn_NC(1, 2, 1, 5, (n, n)), 5e-4, 4, 5, "result_unet", True),
            "1d_FPE": Experiment("1d_FPE", 1, data.TrajectoryDataset1D,
                                 lambda n, dev: unet.PermInvUNet_attn1D_bag(1, 2, 1, 5, n, device=dev), 1e-3, 32,
                                 10, "results_unet_bag", True, all4),
            "1d_GPE": Experiment("1d_GPE", 1, data.ParameterDataset,
                                 lambda n, dev: unet.PermInvUNet_attn1D_bag_GPE(1, 2, 1, 4, n, device=dev,
                                                                                width=20, modes=40),
                                 1e-3, 32, 10, "results_GPE_unet", False),
        }

    def nio2d(heads):
        return lambda n, dev: nio.NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 32, 2, heads=heads,
                                              branch_last_kernel=Encoder2D.kernel_for_grid(n))
    return {
        "2d_FPE": Experiment("2d_FPE", 2, data.TrajectoryDataset2D, nio2d(("fno_drift", "fno_diffusion")),
                             5e-4, 4, 5, "result_2d_fno", True, all4),
        "2d_Non_conservative_FPE": Experiment("2d_Non_conservative_FPE", 2, data.TrajectoryDataset2DForce,
                                              nio2d(("fno_Fx", "fno_Fy")), 5e-4, 4, 5, "result_2d_fno", True,
                                              all4),
        "1d_FPE": Experiment("1d_FPE", 1, data.TrajectoryDataset1D,
                             lambda n, dev: nio.NIOFP_FNO(3, 30, 15, 2, dev), 1e-3, 32, 10, "results_fno", True,
                             all4),
        "1d_GPE": Experiment("1d_GPE", 1, data.ParameterDataset,
                             lambda n, dev: nio.NIOFP_FNO(3, 20, 40, 1, dev, heads=("fno_V",)), 1e-3, 32, 10,
                             "results_GPE_fno", False),
    }


def split_indices(n: int, seed: int = SPLIT_SEED):
    """``random_split(dataset, [int(0.8 n), n - int(0.8 n)], generator=seeded(seed))``
    (2d_FPE/train_fno.py:67-69)."""
    g = torch.Generator()
    g.manual_seed(seed)
    perm = torch.randperm(n, generator=g).tolist()
    n_train = int(0.8 * n)
    return perm[:n_train], perm[n_train:]


class Trainer:
    def __init__(self, exp: Experiment, data_path: str, outdir: str, device, *, epochs: int,
                 seed: int = 1, split_seed: int = SPLIT_SEED, scheduler_mode: str = "reference",
                 eval_mode: str = "reference", save_interval: Optional[int] = None,
                 batch: Optional[int] = None, lr: Optional[float] = None, log=print):
        from . import data as bdata
        from .train import (DataParallel, FlatAdam, GraphedBagStep, StepLR, grid1d, grid2d,
                            trained_parameters)
        from .nio import draw_bag
        from . import load_library, mse_loss
        load_library()
        self.exp, self.device, self.epochs, self.log = exp, device, epochs, log
        self.seed = seed
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        self.outdir = outdir
        self.save_interval = save_interval or exp.save_interval
        self.B = batch or exp.batch
        self.eval_mode = eval_mode
        self.draw_bag = draw_bag
        self.mse_loss = mse_loss
        ds = exp.dataset(data_path)
        self.dataset = ds
        tr, te = split_indices(len(ds), split_seed)
        self.train_idx, self.test_idx = tr, te
        Xtr, Ytr = bdata.device_tensors(ds, tr, device)
        Xte, Yte = bdata.device_tensors(ds, te, device)
        self.Xtr, self.Ytr, self.Xte, self.Yte = Xtr, Ytr, Xte, Yte
        self.T = Xtr.shape[1]
        n = Xtr.shape[2]
        self.grid = grid2d(n, Xtr.shape[3], device) if exp.dim == 2 else grid1d(n, device)
        # seeds after the split, as the reference (2d_FPE/train_fno.py:78-81)
        np.random.seed(seed + self.rank)
        torch.manual_seed(seed + self.rank)
        self.model = exp.model(n, device).to(device)
        self.opt = FlatAdam(trained_parameters(self.model, exclude_prefixes=exp.exclude_prefixes),
                            lr=lr or exp.lr)
        self.dp = DataParallel(self.opt)
        self.dp.broadcast_parameters(0)
        world_steps = self.world if scheduler_mode == "reference" else 1
        self.sched = StepLR(self.opt, 100, 0.5, world_steps=world_steps)
        self.xb = torch.empty((self.B,) + tuple(Xtr.shape[1:]), device=device)
        self.yb = torch.empty((self.B,) + tuple(Ytr.shape[1:]), device=device)
        self.graphed = GraphedBagStep(self.model, mse_loss, self.opt, self.dp, self.xb, self.yb, self.grid)
        self.loss_sum = torch.zeros((), dtype=torch.float64, device=device)
        self.history = {k: [] for k in exp.loss_files}
        self.best = math.inf
        self.best_path = None
        if self.rank == 0:
            os.makedirs(outdir, exist_ok=True)

    # ------------------------------------------------------------------ training
    def _epoch_batches(self, epoch: int):
        """Shuffled train indices of this epoch split into per-rank batches.  One process: the
        DataLoader's batches, the last one possibly partial.  DDP: every rank gets the same
        number of full batches (accelerate's even_batches wraps the index list)."""
        g = torch.Generator()
        g.manual_seed(1_000_003 * (self.seed + 1) + epoch)     # DataLoader(shuffle=True), seeded
        order = torch.randperm(len(self.train_idx), generator=g)
        if self.world == 1:
            return [order[i:i + self.B] for i in range(0, len(order), self.B)]
        per = self.world * self.B
        steps = -(-len(order) // per)
        order = order.repeat(-(-steps * per // len(order)))[:steps * per]
        return [order[s * per + self.rank * self.B: s * per + (self.rank + 1) * self.B] for s in range(steps)]

    def train_epoch(self, epoch: int) -> float:
        self.model.train()
        self.loss_sum.zero_()
        for ids in self._epoch_batches(epoch):
            ids = ids.to(self.device)
            b = ids.numel()
            _, idx = self.draw_bag(self.T)                # the reference's numpy draw
            if b == self.B:
                torch.index_select(self.Xtr, 0, ids, out=self.xb)
                torch.index_select(self.Ytr, 0, ids, out=self.yb)
                key = self.graphed.step(idx)
                self.loss_sum.add_(self.graphed.loss[key], alpha=float(b))
            else:                                         # partial last batch (one process)
                out = self.model(self.Xtr.index_select(0, ids), self.grid, bag_idx=idx)
                loss = self.mse_loss(out, self.Ytr.index_select(0, ids))
                loss.backward()
                self.dp.step()
                self.opt.zero_grad()
                self.loss_sum.add_(loss.detach(), alpha=float(b))
        self.sched.step()
        return float(self.loss_sum) / len(self.train_idx)

    # ------------------------------------------------------------------ evaluation
    @torch.no_grad()
    def evaluate(self):
        """(test_loss, drift, diffusion) as the reference's eval block computes them."""
        from . import ops
        self.model.eval()
        sums = torch.zeros(2, dtype=torch.float64, device=self.device)
        nb = -(-len(self.test_idx) // self.B)
        for k in range(nb):
            if self.world > 1 and k % self.world != self.rank:
                continue                                  # accelerate shards the test loader
            x = self.Xte[k * self.B:(k + 1) * self.B]
            y = self.Yte[k * self.B:(k + 1) * self.B]
            pred = self.model(x, self.grid)
            if self.exp.two_channel_metric:
                e0, e1 = ops.train_rel_l2_2ch(pred, y)
                sums[0] += e0.sum()
                sums[1] += e1.sum()
            else:
                n = pred[0].numel()
                s = ops.rowsq(pred, y, pred.shape[0], n, 1, 0, 0, 1)
                sums[0] += (s[:, 0].sqrt() / s[:, 1].sqrt()).sum()
        if self.world > 1 and self.eval_mode == "global":
            dist.all_reduce(sums)
        d, f = (float(v) / len(self.test_idx) for v in sums.tolist())
        return d + f, d, f

    # ------------------------------------------------------------------ checkpoints
    def state_dict(self):
        sd = self.model.state_dict()
        if self.world > 1:                                # accelerator.save of the DDP model
            return type(sd)(("module." + k, v) for k, v in sd.items())
        return sd

    def maybe_save_best(self, test_loss: float):
        if self.rank != 0 or not test_loss < self.best:
            return
        self.best = test_loss
        if self.best_path is not None and os.path.exists(self.best_path):
            os.remove(self.best_path)
        self.best_path = os.path.join(self.outdir, f"model_checkpoint_best_{self.best:.6f}.pt")
        torch.save({k: v.detach().cpu() for k, v in self.state_dict().items()}, self.best_path)
        self.log(f"New best model saved with Test Loss {self.best:.6f} ")

    def save_losses(self):
        if self.rank != 0:
            return
        for k, v in self.history.items():
            np.save(os.path.join(self.outdir, k + ".npy"), np.array(v))

    def fit(self):
        for epoch in range(1, self.epochs + 1):
            train_loss = self.train_epoch(epoch)
            self.history["train_losses"].append(train_loss)
            if epoch % self.save_interval == 0:
                test_loss, d, f = self.evaluate()
                self.history["test_losses"].append(test_loss)
                if "test_losses_drift" in self.history:
                    self.history["test_losses_drift"].append(d)
                    self.history["test_losses_diffusion"].append(f)
                if self.rank == 0:
                    msg = f"Epoch {epoch}/{self.epochs}, Train Loss: {train_loss:.6f}, Test Loss: {test_loss:.6f}, "
                    if self.exp.two_channel_metric:
                        msg += f"Test Loss drift: {d:.6f}, Test Loss diffusion: {f:.6f}"
                    self.log(msg)
                self.maybe_save_best(test_loss)
        self.save_losses()
        return self.history


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--experiment", choices=sorted(_experiments()), default="2d_FPE")
    ap.add_argument("--model", choices=["fno", "unet", "nio"], default="fno",
                    help="fno: train_fno*.py (NIO-FNO); unet: train_unet*.py (attention UNet); "
                         "nio: train_nio*.py (DeepONet-branch NIO)")
    ap.add_argument("--data", required=True, help="the experiment's dataset file (npz, or the GPE .npy dict)")
    ap.add_argument("--outdir", default=None, help="result directory (default: the reference's)")
    ap.add_argument("--epochs", type=int, default=400)
    ap.add_argument("--save-interval", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None, help="per-rank batch (default: the reference's)")
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--split-seed", type=int, default=SPLIT_SEED)
    ap.add_argument("--scheduler-mode", choices=["reference", "per-epoch"], default="reference")
    ap.add_argument("--eval-mode", choices=["reference", "global"], default="reference")
    a = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    exp = _experiments(a.model)[a.experiment]
    t = Trainer(exp, a.data, a.outdir or exp.result_dir, torch.device("cuda", local), epochs=a.epochs,
                seed=a.seed, split_seed=a.split_seed, scheduler_mode=a.scheduler_mode,
                eval_mode=a.eval_mode, save_interval=a.save_interval, batch=a.batch, lr=a.lr,
                log=lambda s: print(s, flush=True))
    t.fit()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
