#!/usr/bin/env python3
"""BlinDNO FNO-NIO training throughput on MI355X (BASELINE.json config C).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (one "step"): NIOFP2D_FNO(2,3,100,25,3,12,32,2) train step on a 128x128 grid,
per-GPU batch B=4 snapshot bags of T=100 frames, random bag size L = randint(50, T) with
replacement (numpy RNG seeded 1234+rank), MSE loss, backward, gradient all-reduce over
ranks (N>1), fused Adam (lr 5e-4).  Synthetic standardised bags live in HBM (each rank
owns its shard of a 4096-bag set).  value = world * B * K / max-over-ranks(time of K steps)
snapshot-bags/s.

Extra fields: "roofline" for the dominant kernel (algorithmic bytes or flops per launch /
average launch time, measured with HIP events on the launch stream during the timed
region) and "cpu_baseline" (the float32 CPU oracle timed on this host on a bounded
sample of the same workload, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FP32_PEAK_TFLOPS = 157.3       # fp32 vector = fp32 MFMA dense peak (same table)
BASELINE_METRIC = "snapshot-bags/sec (train step) + rel-L2 drift error, 2D FPE 128\u00b2 @1/2/4/8 GPU"


# BASELINE.json configs (SURVEY.md section 8 "Configs restated")
CONFIGS = {
    "A": dict(desc="1d_FPE train_fno.py NIOFP_FNO(3,30,15,2) on a 64-point grid", dim=1, N=64, T=256, B=32,
              lr=1e-3),
    "B": dict(desc="1d_GPE train_fno_GPE.py NIOFP_FNO(3,20,40,1) head fno_V on a 256-point grid", dim=1,
              N=256, T=101, B=32, lr=1e-3),
    "C": dict(desc="2d_FPE train_fno.py NIOFP2D_FNO(2,3,100,25,3,12,32,2)", dim=2, N=128, T=100, B=4,
              lr=5e-4),
    "D": dict(desc="2d_Non_conservative_FPE train_nio.py NIOFP2D(2,3,100,25,3,12,32,2) heads Fx,Fy", dim=2,
              N=128, T=100, B=4, lr=5e-4),
    "E": dict(desc="2D FNO-NIO NIOFP2D_FNO(2,3,100,25,3,12,32,2) on a 256x256 grid (no 2d_GPE in the "
                   "reference; real-valued synthetic bags)", dim=2, N=256, T=100, B=4, lr=5e-4),
    # the token-attention variant (not a BASELINE.json config; bags drawn without
    # replacement, 2d_FPE/NIOModules.py:344-345)
    "C_attn": dict(desc="2d_FPE NIOFP2D_FNO_attn(2,3,100,25,3,12,32,2,128,128)", dim=2, N=128, T=100,
                   B=4, lr=5e-4),
    # the attention UNet ("BlinDNO") at the reference's own training configurations
    "U": dict(desc="2d_FPE train_unet.py PermInvUNet_attn(1,2,1,4,(61,61))", dim=2, N=61, T=100, B=4,
              lr=5e-4),
    "U_NC": dict(desc="2d_Non_conservative_FPE train_unet.py PermInvUNet_attn(1,2,1,5,(80,80))", dim=2,
                 N=80, T=100, B=4, lr=5e-4),
    "U1": dict(desc="1d_FPE train_unet_bag.py PermInvUNet_attn1D_bag(1,2,1,5,80)", dim=1, N=80, T=256,
               B=32, lr=1e-3),
}


def build_model(cfg_name, N, dev):
    import blindno
    from blindno.train import trained_parameters
    if cfg_name == "A":
        m = blindno.NIOFP_FNO(3, 30, 15, 2, dev)
        return m.to(dev), trained_parameters(m), 2
    if cfg_name == "B":
        m = blindno.NIOFP_FNO(3, 20, 40, 1, dev, heads=("fno_V",))
        return m.to(dev), trained_parameters(m), 1
    if cfg_name in ("U", "U_NC", "U1"):
        from blindno import unet
        if cfg_name == "U":
            m = unet.PermInvUNet_attn(1, 2, 1, 4, (N, N))
        elif cfg_name == "U_NC":
            m = unet.PermInvUNet_attn_NC(1, 2, 1, 5, (N, N))
        else:
            m = unet.PermInvUNet_attn1D_bag(1, 2, 1, 5, N, device=dev)
        m = m.to(dev)
        return m, trained_parameters(m), 2
    if cfg_name == "C_attn":
        m = blindno.NIOFP2D_FNO_attn(2, 3, 100, 25, 3, 12, 32, 2, N, N)
        return m.to(dev), trained_parameters(m), 2
    if cfg_name == "D":
        m = blindno.NIOFP2D(2, 3, 100, 25, 3, 12, 32, 2, heads=("fno_Fx", "fno_Fy"),
                            branch_last_kernel=blindno.Encoder2D.kernel_for_grid(N))
        return m.to(dev), trained_parameters(m, exclude_prefixes=("fc0.",)), 2
    m = blindno.NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 32, 2,
                            branch_last_kernel=blindno.Encoder2D.kernel_for_grid(N))
    return m.to(dev), trained_parameters(m), 2


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--serial-heads", action="store_true", help="run the two heads on one stream")
    ap.add_argument("--forked-heads", action="store_true",
                    help="two heads as two forked launch chains instead of one grouped chain")
    ap.add_argument("--config", default="C", choices=sorted(CONFIGS),
                    help="BASELINE.json config (C = the headline metric)")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--T", type=int, default=None)
    ap.add_argument("--bags", type=int, default=4096, help="dataset size (all ranks)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="cpu baseline budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the GPU-vs-CPU-reference parity leg")
    ap.add_argument("--no-kernel-timer", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of HIP graphs")
    ap.add_argument("--overlap", default="auto", choices=("auto", "on", "off"),
                    help="two-graph step with the heads' gradient all-reduce beside the encoder's "
                         "backward (auto: at N > 1)")
    ap.add_argument("--mix", default=None, choices=("fp32", "fp16"),
                    help="channel-mix operand precision of the 2D spectral layers (default: fp16 "
                         "for config E as BASELINE.json names it, fp32 otherwise)")
    ap.add_argument("--timer-steps", type=int, default=4,
                    help="eager steps after the timed region that time the dominant kernel (graph mode)")
    return ap.parse_args()


def main():
    a = parse()
    import blindno
    from blindno import timing
    from blindno.nio import draw_bag_distinct as draw_distinct
    from blindno.train import (BatchSelect, DataParallel, FlatAdam, GraphedBagStep, grid1d, grid2d,
                               shard_bag_ids, synthetic_bags)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # RCCL ("nccl") across the node's GPUs; BLINDNO_BENCH_BACKEND=gloo rehearses the N > 1
        # path with several ranks on one GPU (RCCL refuses two ranks per device)
        backend = os.environ.get("BLINDNO_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    blindno.load_library()

    seed = 1234
    np.random.seed(seed + rank)
    torch.manual_seed(seed + rank)
    cfg = CONFIGS[a.config]
    if a.serial_heads:
        import blindno.nio
        blindno.nio.HEAD_STREAMS = False
    if a.forked_heads or a.serial_heads:
        from blindno import ops as _ops
        _ops.GROUPED_HEADS = False
    N = a.grid or cfg["N"]
    T = a.T or cfg["T"]
    B = a.batch or cfg["B"]
    mix = a.mix or ("fp16" if a.config == "E" else "fp32")
    blindno.set_mix_precision(mix)
    model, params, out_ch = build_model(a.config, N, dev)
    model.train()
    opt = FlatAdam(params, lr=cfg["lr"])
    dp = DataParallel(opt)
    dp.broadcast_parameters(0)

    # one global bag-keyed dataset of a.bags bags; rank r holds {i : i mod world = r}
    gshape = (N, N) if cfg["dim"] == 2 else (N,)
    my_ids = shard_bag_ids(a.bags, B, rank, world)
    n_local = len(my_ids)
    X, Y = synthetic_bags(n_local, T, gshape, out_ch, seed=seed, device=dev, bag_ids=my_ids)
    grid = grid2d(N, N, dev) if cfg["dim"] == 2 else grid1d(N, dev)
    order = torch.randperm(n_local, device=dev, generator=torch.Generator(device=dev).manual_seed(seed + rank))
    loss_acc = torch.zeros((), device=dev)

    xb = torch.empty((B,) + tuple(X.shape[1:]), device=dev)
    yb = torch.empty((B,) + tuple(Y.shape[1:]), device=dev)
    graphed = None
    # one graph per bag size (device-resident bag indices)
    if not a.no_graph:
        # one HIP graph per bag size L = randint(50, T) (captured here, before the warm-up; the
        # numpy draw below stays the reference's: L and idx are drawn on the host every step)
        graphed = GraphedBagStep(model, blindno.mse_loss, opt, dp, xb, yb, grid, loss_acc,
                                 overlap=None if a.overlap == "auto" else a.overlap == "on")
        torch.index_select(X, 0, order[:B], out=xb)
        torch.index_select(Y, 0, order[:B], out=yb)
        # keys: the bag size L, or with deduplicated bags the number of distinct snapshots
        # (U <= L; a randint(50, T) draw with replacement from T has U >= ~0.3 T in practice)
        for L in range(min(50, T // 5) if graphed.dedup else 50, T):
            graphed.capture(L)
        torch.cuda.synchronize()

    # the batch (bags and targets of the drawn ids) in one blindno_gather_batch launch
    select = BatchSelect([X, Y], [xb, yb])
    hostp = {"batch_select": 0.0, "draw": 0.0, "step": 0.0, "n": 0}

    n_loss = [0]             # steps whose loss went into loss_acc (the kernel-timer steps do not)

    def step(i, eager=False, count_loss=True):
        t0_ = time.perf_counter()
        j = (i * B) % (n_local - B + 1)
        ids = order[j:j + B]
        select(ids)
        if graphed is not None and not eager:
            t1_ = time.perf_counter()
            idx = (draw_distinct if a.config == "C_attn" else blindno.draw_bag)(T)[1]
            t2_ = time.perf_counter()
            graphed.step(idx)
            n_loss[0] += 1
            t3_ = time.perf_counter()
            hostp["batch_select"] += t1_ - t0_
            hostp["draw"] += t2_ - t1_
            hostp["step"] += t3_ - t2_
            hostp["n"] += 1
            return
        out = model(xb, grid)
        loss = blindno.mse_loss(out, yb)
        loss.backward()
        dp.step()
        opt.zero_grad()
        if count_loss:
            loss_acc.add_(loss.detach())
            n_loss[0] += 1

    for i in range(a.warmup):
        tw = time.perf_counter()
        step(i)
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] warmup step {i}: {time.perf_counter() - tw:.3f}s", file=sys.stderr, flush=True)
    timer = None
    if not a.no_kernel_timer:
        # the dominant kernel: the bag-level projection (configs with the fused snapshot encoder);
        # config D: its snapshot CNN's implicit-GEMM convolutions as one family
        timer = timing.KernelTimer("blindno_conv2d" if a.config == "D" else timing.DOMINANT)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if timer and graphed is None:
        timer.start()
    hostp.update(batch_select=0.0, draw=0.0, step=0.0, n=0)
    if graphed is not None:
        graphed.host_times = {}
        if world > 1:
            graphed.ar_events = []
    # per-step GPU time on the main stream (N > 1: per-rank min / max in the line)
    sev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)] if world > 1 else None
    if sev:
        sev[0].record()
    for i in range(a.steps):
        step(a.warmup + i)
        if sev:
            sev[i + 1].record()
    t_enq = time.perf_counter() - t0          # host time to enqueue the K steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if timer and graphed is not None:
        # graph replays cannot be hooked: time the dominant kernel (the identical launches) with
        # HIP events on its stream over a few eager steps right after the timed region
        timer.start()
        for i in range(a.timer_steps):
            step(a.warmup + a.steps + i, eager=True, count_loss=False)
    if timer:
        timer.stop()
    dtt = torch.tensor([dt], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(dtt, op=dist.ReduceOp.MAX)
    dt = float(dtt)
    value = world * B * a.steps / dt
    dist_info = None
    if world > 1:
        # self-validating N > 1 line: who ran, over what, and where the time went per rank
        st = [sev[i].elapsed_time(sev[i + 1]) for i in range(a.steps)]
        ar = graphed.allreduce_ms() if graphed is not None else {}
        mine = torch.tensor([min(st), max(st), sum(st) / len(st), dt * 1e3 / a.steps,
                             sum(ar.values())], device=dev, dtype=torch.float64)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        try:
            rccl = ".".join(str(v) for v in torch.cuda.nccl.version())
        except Exception:  # noqa: BLE001 (gloo rehearsal builds)
            rccl = None
        # DP replicas must stay identical: compare every rank's parameters with rank 0's
        ref_flat = opt.flat.clone()
        dist.broadcast(ref_flat, 0)
        same = torch.tensor([1 if torch.equal(ref_flat, opt.flat) else 0], device=dev, dtype=torch.int32)
        maxdiff = (ref_flat - opt.flat).abs().max().reshape(1).double()
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
        dist.all_reduce(maxdiff, op=dist.ReduceOp.MAX)
        del ref_flat
        ids = torch.tensor([my_ids[0], my_ids[-1], len(my_ids)], device=dev, dtype=torch.int64)
        all_ids = [torch.zeros_like(ids) for _ in range(world)]
        dist.all_gather(all_ids, ids)
        dist_info = {
            "params_identical_across_ranks": bool(int(same) == 1),
            "params_max_abs_diff_vs_rank0": float(maxdiff),
            "bag_ids_per_rank": [{"rank": r, "first": int(t[0]), "last": int(t[1]), "count": int(t[2]),
                                  "rule": "i mod world == rank"} for r, t in enumerate(all_ids)],
            "world_size": dist.get_world_size(), "backend": dist.get_backend(),
            "rccl_version": rccl,
            "per_rank_step_ms": [{"rank": r, "min": round(float(t[0]), 4), "max": round(float(t[1]), 4),
                                  "mean": round(float(t[2]), 4), "wall_mean": round(float(t[3]), 4),
                                  "allreduce_ms": round(float(t[4]), 4)} for r, t in enumerate(allr)],
            "allreduce_bytes_per_step": int(4 * opt.grad.numel()),
            "allreduce_ms_per_step_rank0": {k: round(v, 4) for k, v in ar.items()},
            "allreduce_timing": "HIP events on the issuing stream around each bucketed all_reduce",
        }
    loss_mean = float(loss_acc) / max(1, n_loss[0])      # before the parity leg's replay adds to it

    if rank == 0:
        res = {
            "metric": (BASELINE_METRIC if a.config == "C" else
                       f"snapshot-bags/sec (train step), config {a.config}"),
            "value": round(value, 3),
            "unit": "snapshot-bags/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * dt / a.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if mix == "fp32" else "f32 (fp16 channel-mix operands, fp32 accumulate)",
            "data": "synthetic (standardised N(0,1) bags resident in HBM; reference datasets not shipped)",
            "config": {"workload": f"{cfg['desc']} ({a.config}), grid {'x'.join([str(N)] * cfg['dim'])}",
                       "per_gpu_batch": B, "global_batch": B * world, "T": T,
                       "bag_size": "L=randint(50,T) " + ("without" if a.config == "C_attn" else "with")
                                   + " replacement", "dataset_bags": a.bags,
                       "sharding": "bag i on rank i mod world (bag-keyed synthetic set, same data at any N)",
                       "parallelism": f"dp{world}", "optimizer": f"Adam lr {cfg['lr']} (fused flat)",
                       "launch": ("eager" if not graphed else
                                  "hip-graph per bag size L (all kernels replayed each step)" +
                                  ("; two graphs per step, heads' gradient all-reduce overlapped "
                                   "with the encoder backward" if graphed.overlap else ""))},
        }
        if dist_info is not None:
            res["dist"] = dist_info
        if timer:
            # the limiter: the bag-level projection is fp32 VALU-issue-bound (PMC valu_issue_util);
            # the conv family runs on the fp32 matrix cores
            # PMC records of this config's shapes (profiles/pmc_traffic.json: config C unprefixed,
            # config E as "E:<entry>", tools/pmc_traffic.py --prefix)
            pre = {"C": "", "E": "E:"}.get(a.config)
            res["roofline"] = timer.roofline(HBM_PEAK_GBS, FP32_PEAK_TFLOPS,
                                             bound="valu" if timer.name == timing.DOMINANT else None,
                                             traffic_per_point=timing.pmc_traffic(ROOT, pre + timing.DOMINANT)
                                             if pre is not None else None)
            rec = timing.pmc_record(ROOT, pre + timing.DOMINANT) if pre is not None else None
            if res["roofline"] and rec and "valu_issue_util" in rec:
                # the limiter of this kernel (profiles/pmc_traffic.json, tools/pmc_traffic.py)
                res["roofline"]["valu_issue_util"] = rec["valu_issue_util"]
                res["roofline"]["valu_issue_util_source"] = (
                    "PMC SQ_INSTS_VALU / _TRANS_F32 / _MFMA, GRBM_GUI_ACTIVE clock, kbench Bn=300: " +
                    rec["source"])
            pb = os.path.join(ROOT, "profiles", "pmc_benched_step.json")
            if res["roofline"] and a.config == "C" and os.path.exists(pb):
                # the same utilisation over the benched step's own dispatches (graph replays,
                # drawn bag sizes; tools/pmc_bench.sh + tools/pmc_bench.py)
                sb = json.load(open(pb))
                if "valu_issue_util" in sb:
                    res["roofline"]["valu_issue_util_benched_step"] = sb["valu_issue_util"]
                    res["roofline"]["valu_issue_util_benched_step_source"] = sb.get("source")
            if a.config in ("C", "E"):
                res["roofline_spectral"] = spectral_roofline(model, grid, B, T, N, dev, pmc_prefix=pre)
        if world == 1 and a.config in ("A", "B", "C", "D", "E"):
            # the reference's CPU path on the same weights / inputs: accuracy parity of the
            # benched step (the "rel-L2 drift error" half of BASELINE's metric), then its timing
            if not a.no_parity:
                res["parity"] = parity_check(a.config, model, graphed, opt, xb, yb, grid, T, mix=mix)
            if a.config == "C" and not a.no_cpu:
                res["cpu_baseline"] = cpu_baseline(a.config, model, xb, yb, grid, T, budget=a.cpu_seconds)
        res["loss_mean"] = loss_mean
        res["host_enqueue_ms_per_step"] = round(1000.0 * t_enq / a.steps, 4)
        if hostp["n"]:
            hb = {k: round(1e6 * hostp[k] / hostp["n"], 1) for k in ("batch_select", "draw", "step")}
            for k, v in (getattr(graphed, "host_times", None) or {}).items():
                hb["step." + k] = round(1e6 * v / hostp["n"], 1)
            res["host_us_per_step"] = hb
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


# the chained FNO_input layer's kernels as tools/pmc_traffic.py names them in
# profiles/pmc_traffic.json (the fused column pass since round 4, the row inverse with the next
# layer's row DFT)
SPECTRAL_PMC_KERNELS = ("colfuse (blindno_colpass, FNO_input)", "blindno_rowidft_epi_rd")
# ... and of the layer with the column pass folded into the row kernels (csrc/colspec.h)
SPECTRAL_PMC_KERNELS_FOLDED = ("blindno_colmix", "blindno_rowidft_epi_zc")


def spectral_roofline(model, grid, B, T, N, dev, pmc_prefix=""):
    """HBM roofline of one FNO_input spectral layer (the north star's 'spectral-conv kernel') at
    the mean bag size (L = 75), timed with HIP events on the launch stream; algorithmic bytes per
    SURVEY.md 8d: 4 Bn Ci P^2 (read x) + 4 Bn Co P^2 (write y) + 16 Ci Co m1 m2 (weights).

    Headline form = the layer as the step chains it.  With the folded column pass (ops.COLSPEC,
    csrc/colspec.h): blindno_colmix (the previous kernel's column-DFT partials summed, Xs and the
    mixed spectrum Y) + the row inverse that rebuilds its row coefficients from Y, applies the
    conv / bias / GELU epilogue and leaves the NEXT layer's column-DFT partials
    (blindno_rowidft_epi_zc).  Reported beside it: the chain through the column pass (column pass
    + row inverse with the next row DFT, round 4's headline) and the unchained layer (row DFT +
    column pass + row inverse, three passes over the field's spectra, x read twice)."""
    from blindno import ops
    from blindno._lib import call, ptr, stream_ptr
    fno = model.FNO_input
    C, m = fno.width, fno.modes1
    P = N + ops.pad_amount(N)
    Bn = B * 75
    x = torch.randn(Bn, C, P, P, device=dev)
    s0 = fno.spectral_list[1]
    w1, w2 = s0._real_view()
    cw, cb = fno.conv_list[1].weight.detach(), fno.conv_list[1].bias.detach()
    sh = ops.SpecShape(Bn, C, C, P, P, m, m, 2)
    Wt = ops.pack_weights((w1.detach(), w2.detach()), P, 2)
    At = ops.k_rowdft(x, Bn, C, P, P, m, 1)

    def colpass_chained():
        _, Z = ops.k_colpass(At, Wt, Bn, C, C, P, m, m, P, 0)
        return ops.k_rowidft_epi_rd(Z, x, cw, cb, Bn, C, P, P, m, 1, 1)

    def unchained():
        _, Z = ops.spec_forward(x, 1, Wt, sh)
        return ops.k_rowidft_epi(Z, x, cw, cb, Bn, C, P, P, m, 1)

    folded = None
    if ops.colspec_ok(Bn, C, P, P, m, m):
        cs = ops._ColSpec(Bn, C, P, P, m, m, dev)
        p_in, p_out = cs.part(C, x), cs.part(C, x)
        z = torch.empty_like(x)
        # the incoming partials (what the previous layer's row inverse leaves)
        call("blindno_rowdft_cd", ptr(x), ptr(p_in), ptr(cs.Tp), ptr(cs.tab), Bn, C, P, P, m, 1, P, P,
             stream_ptr())

        def folded():
            _, Y = cs.mix(p_in, cs.nb, Wt, 0)
            call("blindno_rowidft_epi_zc", ptr(Y), ptr(x), ptr(cw), ptr(cb), ptr(z), ptr(cs.tb), ptr(cs.tab),
                 ptr(p_out), ptr(cs.Tp), Bn, C, P, P, m, m, 1, 1, P, P, stream_ptr())

        # the same layer's adjoint as the step chains it: colmix (direction 1) + the adjoint row
        # inverse with GELU' of the layer input, the 1x1-conv weight gradient and the previous
        # layer's column-DFT partials (blindno_rowidft_bwd_zc); dz given as a field
        dzt, dxt = torch.randn_like(x), torch.empty_like(x)
        pa_in, pa_out = cs.part(C, x), cs.part(C, x)
        call("blindno_rowdft_cd", ptr(dzt), ptr(pa_in), ptr(cs.Tp), ptr(cs.tab), Bn, C, P, P, m, 0, P, P,
             stream_ptr())
        pw = torch.empty(ops.query("blindno_colspec_bwd_nchunk", Bn, P), C * C + C, device=dev)

        def adjoint():
            _, Yb = cs.mix(pa_in, cs.nb, Wt, 1)
            call("blindno_rowidft_bwd_zc", ptr(Yb), ptr(dzt), ptr(cw), ptr(x), ptr(dxt), ptr(cs.tb), ptr(cs.tab),
                 ptr(pa_out), ptr(cs.Tp), ptr(pw), Bn, C, P, P, m, m, 1, P, P, stream_ptr())

    trials = {}

    def timed(layer, name=None):
        # the best of five 10-launch trials, with min / median / max kept for the line: one trial
        # of a round-5 run read 2x the others (gpurun_out/bench_r05z_C.json)
        for _ in range(3):
            layer()
        ts = []
        for _ in range(5):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            ev0.record()
            for _ in range(reps):
                layer()
            ev1.record()
            torch.cuda.synchronize()
            ts.append(ev0.elapsed_time(ev1) / reps)
        if name is not None:
            trials[name] = {"min": round(min(ts), 4), "median": round(sorted(ts)[len(ts) // 2], 4),
                            "max": round(max(ts), 4)}
        return min(ts)

    nbytes = 4 * Bn * C * P * P * 2 + 16 * C * C * m * m
    gb = lambda ms: nbytes / (ms * 1e-3) / 1e9
    ms_c, ms_u = timed(colpass_chained, "column_pass_chained"), timed(unchained, "unchained")
    side = {"column_pass_chained": {"kernels": "blindno_colpass + blindno_rowidft_epi_rd",
                                    "achieved": round(gb(ms_c), 1), "frac": round(gb(ms_c) / HBM_PEAK_GBS, 4),
                                    "ms_per_layer": round(ms_c, 4)},
            "unchained": {"kernels": "blindno_rowdft + blindno_colpass + blindno_rowidft_epi",
                          "achieved": round(gb(ms_u), 1), "frac": round(gb(ms_u) / HBM_PEAK_GBS, 4),
                          "ms_per_layer": round(ms_u, 4)}}
    adj = None
    if folded is not None:
        ms = timed(folded, "forward")
        ms_a = timed(adjoint, "adjoint")
        ab = 4 * Bn * C * P * P * 3 + 16 * C * C * m * m      # read dz, x; write dx
        adj = {"kernels": "blindno_colmix (direction 1) + blindno_rowidft_bwd_zc", "bytes": int(ab),
               "achieved": round(ab / (ms_a * 1e-3) / 1e9, 1),
               "frac": round(ab / (ms_a * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "ms_per_layer": round(ms_a, 4)}
        kern = ("blindno_colmix + blindno_rowidft_epi_zc (one chained FNO_input layer with the column pass "
                "folded into the row kernels: the mixed spectrum in, the next layer's column-DFT partials out)")
        pmc_keys = SPECTRAL_PMC_KERNELS_FOLDED
    else:
        ms = ms_c
        kern = ("blindno_colpass + blindno_rowidft_epi_rd (one chained FNO_input layer: the next layer's row "
                "DFT taken in the row-inverse pass)")
        pmc_keys = SPECTRAL_PMC_KERNELS
        side.pop("column_pass_chained")
    res = {"kernels": kern, "bound": "hbm", "achieved": round(gb(ms), 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(gb(ms) / HBM_PEAK_GBS, 4), "ms_per_layer": round(ms, 4),
           "algorithmic_bytes": int(nbytes), "snapshots": Bn, "traffic": None, **side}
    if adj is not None:
        res["adjoint"] = adj
    res["trials_ms"] = trials
    # measured HBM bytes of the same layer shape (Bn = 300: tools/kbench.py "[input]" under
    # tools/pmc_kbench.sh -> profiles/pmc_traffic.json)
    from blindno import timing
    parts = {k: timing.pmc_record(ROOT, pmc_prefix + k) for k in pmc_keys}
    # only records of this very shape: Bn = 300 snapshots at this grid (a record without "N" is
    # from the 128^2 runs of rounds 4-5)
    if Bn == 300 and all(v is not None and v.get("N", 128) == N for v in parts.values()):
        res["traffic"] = int(sum(v["hbm_bytes_per_dispatch"] for v in parts.values()))
        res["traffic_by_kernel"] = {k: v["hbm_bytes_per_dispatch"] for k, v in parts.items()}
        res["traffic_source"] = sorted({v.get("source") for v in parts.values()})
    return res


def _cpu_params(model):
    """CPU fp32 leaves of the model's current weights (the reference's state_dict keys)."""
    p = {}
    for k, v in model.state_dict().items():
        if k.startswith("branch.") or not (v.is_floating_point() or v.is_complex()):
            continue
        p[k] = v.detach().cpu().clone().requires_grad_(True)
    return p


def _cpu_step(cfg_name, p, x, y, grid, idx):
    """The reference's train step in fp32 on the host (oracle.cpu_ref: rfft2/irfft2, F.gelu,
    F.linear -- the reference's own CPU execution), forward + MSE + backward."""
    from oracle import cpu_ref
    if cfg_name in ("A", "B"):
        heads = ("fno_V",) if cfg_name == "B" else ("fno_drift", "fno_diffusion")
        out = cpu_ref.niofp_fno_fft(p, x, grid, idx=list(idx), heads=heads)
    else:
        out = cpu_ref.niofp2d_fno_fft(p, x, grid, idx=list(idx))
    loss = ((out - y) ** 2).mean()
    loss.backward()
    return out.detach(), loss.detach()


# separately stated tolerance of the fp16 channel mix (config E): fp16 operands carry a unit
# roundoff of 2^-11 = 4.9e-4, so the spectral branch of every layer is ~1e-3 off fp32
MIX16_TOL = {"fields": 5e-3, "grads": 2e-2}


def parity_check(cfg_name, model, graphed, opt, xb, yb, grid, T, seed=4321, mix="fp32"):
    """Accuracy of the benched GPU step (graph replay: deduplicated bag, grouped heads) on one
    recorded bag draw, against (1) the reference's fp32 CPU step (oracle.cpu_ref: pocketfft,
    F.gelu, F.linear -- how the reference computes) and (2) the same step in float64 (same
    code, plain torch fp64 ops on the GPU) as the arbiter, on the same weights and inputs.
    Reported: rel-L2 of the output fields (drift = channel 0, diffusion = channel 1), the loss,
    and the worst per-tensor gradient rel-L2; also the reference fp32 path's own distance to
    fp64 (its conditioning floor).  Pass: GPU vs fp64 within SURVEY.md 8c (fields 1e-5,
    gradients 1e-4) and GPU vs the reference's fp32 fields within 1e-5."""
    if cfg_name == "D":
        return parity_check_nio(model, graphed, opt, xb, yb, grid, T, seed)
    rs = np.random.RandomState(seed)
    L = rs.randint(50, T)
    idx = rs.choice(T, L)
    if graphed is not None:
        key = graphed.replay(idx)
        out_gpu, loss_gpu = graphed.out[key], graphed.loss[key]
    else:
        import blindno
        opt.zero_grad()
        out_gpu = model(xb, grid, bag_idx=idx)
        loss = blindno.mse_loss(out_gpu, yb)
        loss.backward()
        opt.gather_grads()
        out_gpu, loss_gpu = out_gpu.detach(), loss.detach()
        key = L
    torch.cuda.synchronize()
    grads_gpu = {}
    names = {id(q): k for k, q in model.named_parameters()}
    for prm, off, sz in zip(opt.params, opt.offsets, opt.sizes):
        grads_gpu[names[id(prm)]] = opt.grad[off:off + sz].detach().clone()
    out_gpu, loss_gpu = out_gpu.clone(), loss_gpu.clone()
    if graphed is not None:
        graphed.release()            # the timed region is over: free the graph pool for fp64
    p32 = _cpu_params(model)
    out32, loss32 = _cpu_step(cfg_name, p32, xb.cpu(), yb.cpu(), grid.cpu(), idx)
    p64 = {k: v.detach().to(xb.device, torch.complex128 if v.is_complex() else torch.float64)
           .requires_grad_(True) for k, v in p32.items()}
    out64, loss64 = _cpu_step(cfg_name, p64, xb.double(), yb.double(), grid.double(), idx)

    def rel(a, b):
        a, b = a.double().cpu(), b.double().cpu()
        return float((a - b).norm() / b.norm().clamp_min(1e-30))

    def g(p, k):
        t = p[k].grad
        return torch.view_as_real(t) if t.is_complex() else t

    def fields(out, ref):
        r = {"fwd": rel(out, ref), "drift": rel(out[..., 0], ref[..., 0])}
        if ref.shape[-1] > 1:
            r["diffusion"] = rel(out[..., 1], ref[..., 1])
        return r

    def worst(get):
        w = max(((rel(get(k), g(p64, k)), k) for k in grads_gpu), key=lambda t: t[0])
        return w

    gw, gk = worst(lambda k: grads_gpu[k].view(g(p64, k).shape))
    rw, rk = worst(lambda k: g(p32, k))
    gpu64 = fields(out_gpu, out64)
    ref64 = fields(out32, out64)
    gpu32 = fields(out_gpu, out32)
    fmt = lambda d: {k: float(f"{v:.3e}") for k, v in d.items()}
    res = {"bag": {"L": int(L), "distinct": int(len(np.unique(idx))), "graph_key": int(key)},
           "reference": "the reference's fp32 CPU step (oracle.cpu_ref: rfft2/irfft2, F.gelu, F.linear) "
                        "and the same step in fp64 as arbiter, same weights / inputs / bag",
           "drift_rel_l2": float(f"{gpu32['drift']:.3e}"),
           "gpu_vs_ref_fp32": fmt(gpu32),
           "gpu_vs_fp64": dict(fmt(gpu64), grad_max=float(f"{gw:.3e}"), grad_worst=gk,
                               loss=float(f"{abs(float(loss_gpu) - float(loss64)) / abs(float(loss64)):.3e}")),
           "ref_fp32_vs_fp64": dict(fmt(ref64), grad_max=float(f"{rw:.3e}"), grad_worst=rk),
           }
    tf, tg = (1e-5, 1e-4) if mix == "fp32" else (MIX16_TOL["fields"], MIX16_TOL["grads"])
    res["pass"], res["tolerance"], res["checks"] = _field_verdict(gpu64, gpu32, ref64, tf, tg, gw)
    if mix != "fp32":
        res["tolerance"]["mix"] = "fp16"
    return res


def _field_verdict(gpu64, gpu32, ref64, tf, tg, gw, extra=()):
    """Per-channel pass rule of the parity legs (the reference reports drift and diffusion
    separately, 2d_FPE/train_fno.py:160-168).  Every output channel (and the whole output):
      GPU vs fp64            <= tf                                   
      GPU vs reference fp32  <= max(tf, 2 * ref_fp32_vs_fp64[channel]) -- two correct fp32 paths
                                 sit on either side of the fp64 value, so their distance is bounded
                                 by the sum of their distances to it; the bar is that sum with the
                                 GPU's own at most the reference's
    and the worst parameter gradient vs fp64 <= tg.  Returns (pass, tolerance, per-check list)."""
    checks = []
    for ch in gpu64:
        checks.append({"check": f"gpu_vs_fp64.{ch}", "value": float(f"{gpu64[ch]:.3e}"), "bar": tf})
        bar32 = max(tf, 2.0 * ref64[ch])
        checks.append({"check": f"gpu_vs_ref_fp32.{ch}", "value": float(f"{gpu32[ch]:.3e}"),
                       "bar": float(f"{bar32:.3e}")})
    checks.append({"check": "gpu_vs_fp64.grad_max", "value": float(f"{gw:.3e}"), "bar": tg})
    checks.extend(extra)
    for c in checks:
        c["pass"] = bool(c["value"] <= c["bar"])
    tol = {"fields_vs_fp64": tf, "grads_vs_fp64": tg,
           "fields_vs_ref_fp32": f"per channel max({tf:g}, 2 x ref_fp32_vs_fp64[channel])"}
    return all(c["pass"] for c in checks), tol, checks


def parity_check_nio(model, graphed, opt, xb, yb, grid, T, seed):
    """Config D's parity leg: the benched NIOFP2D step (a HIP graph per drawn L, train-mode
    BatchNorm inside it) on one recorded draw vs (1) the reference's fp32 CPU step
    (oracle.cpu_ref.niofp2d_fft: F.conv2d / F.batch_norm / addmm, its own LeakyReLU branches)
    and (2) the same step in fp64 on the GPU as the arbiter.  The Encoder2D branch is piecewise
    linear: a pre-activation within fp32 rounding of 0 may take either LeakyReLU branch in two
    correct evaluations, so the fp64 arbiter takes the branches the REPLAY took (comparisons
    captured into a fresh graph of the same step, tests/test_gpu_configs.py::
    test_config_d_graphed_niofp2d_nc_128) and the count of branches an unconditioned fp64 forward
    takes differently is reported (bar 1e-5 of all).  Pass: GPU vs fp64 fields 1e-5 and every
    gradient 1e-4 (conv biases ahead of batch-statistics BatchNorm, whose true gradient is 0,
    excluded), dL/dbasis (the trunk's upstream gradient) vs fp64 1e-5, GPU vs the reference's fp32
    fields 1e-5, flips within the bar.  The full-chain errors of the worst gradients are reported beside
    the reference fp32 step's own."""
    import blindno
    from oracle import cpu_ref, fno_ref
    from blindno.train import DataParallel, GraphedBagStep
    rs = np.random.RandomState(seed)
    L = rs.randint(50, T)
    idx = rs.choice(T, L)
    if graphed is not None:
        graphed.release()            # the timed region is over: free the graph pool
    rec = []
    names = ("convblock1", "convblock2_1", "convblock2_2", "convblock3_1", "convblock3_2", "convblock4_1",
             "convblock4_2", "convblock7_1", "convblock7_2", "convblock7_3")
    hooks = [getattr(model.branch, n).register_forward_hook(lambda mod, i, o: rec.append(o.detach() > 0))
             for n in names]
    # the trunk's upstream gradient dL/dbasis as the replay computes it (a copy captured into the
    # graph, like the branch masks)
    rec_db = []
    hooks.append(model.trunk.register_full_backward_hook(
        lambda mod, gi, go: rec_db.append(go[0].detach().clone())))
    gs = GraphedBagStep(model, blindno.mse_loss, opt, DataParallel(opt), xb, yb, grid)
    key = gs.replay(idx)
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    masks = rec[-10:]
    dbasis_gpu = rec_db[-1].clone()
    out_gpu, loss_gpu = gs.out[key].clone(), gs.loss[key].clone()
    pnames = {id(q): k for k, q in model.named_parameters()}
    grads_gpu = {pnames[id(prm)]: opt.grad[off:off + sz].detach().clone()
                 for prm, off, sz in zip(opt.params, opt.offsets, opt.sizes)}
    gs.release()
    heads = tuple(model._heads)
    sd = {k: v.detach() for k, v in model.state_dict().items()
          if v.is_floating_point() and not k.endswith(("running_mean", "running_var"))}
    p32 = {k: v.cpu().clone().requires_grad_(True) for k, v in sd.items()}
    out32 = cpu_ref.niofp2d_fft(p32, xb.cpu(), grid.cpu(), idx=list(idx), heads=heads)
    ((out32 - yb.cpu()) ** 2).mean().backward()
    # the trunk's LeakyReLU branches as the GPU takes them (the same kernels as the replay's trunk,
    # on the same weights): a trunk pre-activation within fp32 rounding of 0 flips between two
    # correct evaluations, and one flip moves the trunk's gradients by ~1e-3
    model.trunk.record_branches = []
    # a train-mode forward advances the trunk's BatchNorm1d running statistics and
    # num_batches_tracked: keep the benched model's buffers as the replay left them
    saved = {k: b.clone() for k, b in model.trunk.named_buffers()}
    with torch.no_grad():
        model.trunk(grid.reshape(-1, 2))
        for k, b in model.trunk.named_buffers():
            b.copy_(saved[k])
    del saved
    tmasks = model.trunk.record_branches
    model.trunk.record_branches = None
    p64 = {k: v.double().requires_grad_(True) for k, v in sd.items()}
    own = []
    with torch.no_grad():
        fno_ref.encoder2d(fno_ref.sub_params({k: v.detach() for k, v in p64.items()}, "branch"),
                          xb.double()[:, list(idx)].unsqueeze(2), record=own)
    flips = sum(int((a != b).sum()) for a, b in zip(masks, own))
    total = sum(a.numel() for a in masks)
    del own
    taps = {}
    with torch.no_grad():
        t_own = []
        h = grid.double().reshape(-1, 2)
        pt0 = fno_ref.sub_params({k: v.detach() for k, v in p64.items()}, "trunk")
        z = h @ pt0["input_layer.weight"].T + pt0["input_layer.bias"]
        t_own.append(z > 0)
        h = torch.nn.functional.leaky_relu(z, 0.01)
        for k in range(2):
            z = h @ pt0[f"hidden_layers.{k}.weight"].T + pt0[f"hidden_layers.{k}.bias"]
            t_own.append(z > 0)
            h = torch.nn.functional.batch_norm(torch.nn.functional.leaky_relu(z, 0.01), None, None,
                                               pt0[f"batch_layers.{k}.weight"], pt0[f"batch_layers.{k}.bias"],
                                               training=True, eps=1e-5)
        tflips = sum(int((a != b).sum()) for a, b in zip(tmasks, t_own))
        ttotal = sum(a.numel() for a in tmasks)
    out64 = cpu_ref.niofp2d_fft(p64, xb.double(), grid.double(), idx=list(idx), heads=heads, branch_masks=masks,
                                taps=taps, trunk_masks=tmasks)
    loss64 = ((out64 - yb.double()) ** 2).mean()
    loss64.backward()
    dbasis64 = taps.pop("basis").grad.detach()
    # the trunk as a stage as well: dL/dbasis vs fp64, and the trunk's gradients vs the fp64 trunk
    # given the replay's dL/dbasis.  Its BatchNorm1d over the 16384 grid points sees a nearly
    # constant upstream gradient (rank B = 4): fp32 batch sums there cost 1e-3 of the trunk's
    # gradients (torch's GPU BatchNorm too; its CPU one sums in fp64), csrc/batchnorm.hip sums in fp64
    pt = {k[len("trunk."):]: v.detach().clone().requires_grad_(True) for k, v in p64.items()
          if k.startswith("trunk.")}
    cpu_ref._ffn(pt, grid.double().reshape(-1, 2), 3, tmasks).backward(dbasis_gpu.double())

    def rel(a, b):
        a, b = a.double().cpu(), b.double().cpu()
        return float((a - b).norm() / b.norm().clamp_min(1e-30))

    def fields(o, r):
        return {"fwd": rel(o, r), "Fx": rel(o[..., 0], r[..., 0]), "Fy": rel(o[..., 1], r[..., 1])}

    # the branch ConvBlocks' conv biases feed batch-statistics BatchNorms (true gradient 0); the
    # trunk's hidden_layers.0.bias / batch_layers.0.bias are checked like every other gradient
    keys = [k for k in grads_gpu if not (k.startswith("branch.") and k.endswith(".layers.0.bias"))]
    eg = {k: rel(grads_gpu[k].view(p64[k].shape), p64[k].grad) for k in keys}
    er = {k: rel(p32[k].grad, p64[k].grad) for k in keys}
    es = {k: rel(grads_gpu[k].view(p64[k].shape), pt[k[len("trunk."):]].grad) for k in keys
          if k.startswith("trunk.")}
    e_db = rel(dbasis_gpu, dbasis64)
    gw, gk = max((v, k) for k, v in eg.items())
    rw, rk = max((v, k) for k, v in er.items())
    top = sorted(keys, key=lambda k: -eg[k])[:6]
    gpu64, gpu32, ref64 = fields(out_gpu, out64.detach()), fields(out_gpu, out32.detach()), \
        fields(out32.detach(), out64.detach())
    fmt = lambda d: {k: float(f"{v:.3e}") for k, v in d.items()}
    res = {"bag": {"L": int(L), "distinct": int(len(np.unique(idx))), "graph_key": int(key)},
           "reference": "the reference's fp32 CPU step (oracle.cpu_ref.niofp2d_fft: F.conv2d, F.batch_norm, "
                        "addmm, rfft2/irfft2) and the same step in fp64 on the GPU as arbiter (LeakyReLU "
                        "branches of the replay), same weights / inputs / bag",
           "drift_rel_l2": float(f"{gpu32['Fx']:.3e}"),
           "gpu_vs_ref_fp32": fmt(gpu32),
           "gpu_vs_fp64": dict(fmt(gpu64), grad_max=float(f"{gw:.3e}"), grad_worst=gk,
                               loss=float(f"{abs(float(loss_gpu) - float(loss64)) / abs(float(loss64)):.3e}")),
           "ref_fp32_vs_fp64": dict(fmt(ref64), grad_max=float(f"{rw:.3e}"), grad_worst=rk,
                                    note="the fp32 reference takes its own LeakyReLU branches"),
           "grads_worst": {k: {"gpu": float(f"{eg[k]:.3e}"), "ref_fp32": float(f"{er[k]:.3e}")}
                                      for k in top},
           "trunk_stage": {"dbasis": float(f"{e_db:.3e}"),
                           "grad_max": float(f"{max(es.values()):.3e}"),
                           "note": "trunk gradients vs the fp64 trunk given the replay's dL/dbasis"},
           "branch_flips": {"count": int(flips), "of": int(total), "bar": "1e-5 of all"},
           "trunk_branch_flips": {"count": int(tflips), "of": int(ttotal), "bar": "1e-5 of all",
                                  "note": "the fp64 arbiter takes the trunk's fp32 GPU branches too"},
           "grads_excluded": "branch.*.layers.0.bias: the branch conv biases ahead of batch-statistics "
                             "BatchNorm (true gradient 0)"}
    extra = [{"check": "trunk_stage.dbasis", "value": float(f"{e_db:.3e}"), "bar": 1e-5},
             {"check": "branch_flips", "value": int(flips), "bar": 1e-5 * total},
             {"check": "trunk_branch_flips", "value": int(tflips), "bar": 1e-5 * ttotal}]
    res["pass"], res["tolerance"], res["checks"] = _field_verdict(gpu64, gpu32, ref64, 1e-5, 1e-4, gw, extra)
    return res


def _cpu_share():
    """Threads for the CPU baseline: the CPUs this process may run on (affinity mask), capped by
    the cgroup's CPU quota when one is set (a container's share of a larger host, where the
    affinity mask still lists every CPU)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    threads = min(aff, quota) if quota else aff
    return threads, {"affinity_cpus": aff, "cgroup_quota_cpus": quota, "os_cpu_count": os.cpu_count()}


def _cpu_model():
    """The host CPU's model name (lscpu's 'Model name', read from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or None


def cpu_baseline(cfg_name, model, xb, yb, grid, T, budget):
    """The reference's fp32 CPU train step (oracle.cpu_ref, the reference's own execution:
    pocketfft rfft2/irfft2, fused GELU, addmm linears) timed on this host's cores at the
    benched batch (B bags, L = randint(50, T) with replacement, a fresh draw per step), on the
    model's current weights, until ~``budget`` s."""
    # every core this process may run on (the box's CPU share: its affinity mask, not the whole
    # machine's os.cpu_count())
    threads, share = _cpu_share()
    torch.set_num_threads(threads)
    p = _cpu_params(model)
    x, y, g = xb.cpu(), yb.cpu(), grid.cpu()
    rs = np.random.RandomState(99)
    _cpu_step(cfg_name, p, x, y, g, rs.choice(T, 60))          # warm-up (allocator, fft plans)
    n, Ls, t0 = 0, [], time.perf_counter()
    while True:
        for v in p.values():
            v.grad = None
        L = rs.randint(50, T)
        _cpu_step(cfg_name, p, x, y, g, rs.choice(T, L))
        Ls.append(int(L))
        n += 1
        el = time.perf_counter() - t0
        if (el >= budget and n >= 10) or n >= 200:
            break
    B = x.shape[0]
    return {"value": round(n * B / el, 4), "unit": "snapshot-bags/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "cpu_share": share,
            "sample": f"{n} train steps x B={B} bags (L={Ls} with replacement, fp32 forward+MSE+backward, "
                      f"no optimizer) in {el:.1f}s",
            # the reference itself cannot travel to the GPU box; its own CPU step was timed in the
            # build container
            "reference_measured": {"value": 1.29, "unit": "snapshot-bags/s", "cores": 8,
                                   "where": "the reference's own CPU step (torch 2.10 CPU, 8 threads) in the "
                                            "build container, BASELINE.md; the port above runs ~25 % slower "
                                            "per core"}}


if __name__ == "__main__":
    main()
