"""Diagnostic: per-level activations and gradients of the HIP PermInvUNet_attn vs the fp64
oracle (and the oracle in fp32 as the conditioning yardstick), on a golden case."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"),
                os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import numpy as np
import torch
import oracle
from conftest import load_golden, rel_l2
from test_oracle_golden import unet_recipe_params
from test_gpu_unet import _model

case = sys.argv[1] if len(sys.argv) > 1 else "unet2d_train"
m, g = _model(case)
m.train()
m._taps = []
x = torch.from_numpy(g["in.x"]).cuda()
dim = 1 if case.startswith("unet1d") else 2
idx = g["idx"].tolist() if "idx" in g else None
y = m(x, bag_idx=idx)
(y * torch.from_numpy(g["cot"]).cuda()).sum().backward()
hip = {k: (t.detach().double().cpu(), t.grad.double().cpu()) for k, t in m._taps}
res = {}
for prec, dt in (("fp64", torch.float64), ("fp32", torch.float32)):
    oracle.set_precision(prec)
    st = unet_recipe_params(g)
    p = {k: torch.from_numpy(np.asarray(v)).to(dt).requires_grad_(True) for k, v in st.items()
         if np.asarray(v).dtype.kind == "f"}
    p.update({k: torch.from_numpy(np.asarray(v)) for k, v in st.items() if np.asarray(v).dtype.kind != "f"})
    taps = []
    yo = oracle.unet_ref.perminv_unet_attn(p, torch.from_numpy(g["in.x"]).to(dt), int(g["depth"]), dim,
                                           idx=idx, taps=taps, variant="nc" if case.startswith("nc_") else "fpe")
    (yo * torch.from_numpy(g["cot"]).to(dt)).sum().backward()
    res[prec] = ({k: (t.detach().double(), t.grad.double()) for k, t in taps},
                 {k: v.grad.double() for k, v in p.items() if getattr(v, "grad", None) is not None})
oracle.set_precision("fp64")
for k in hip:
    a, ga = hip[k]
    r, gr = res["fp64"][0][k]
    r32, gr32 = res["fp32"][0][k]
    print(f"{k:8s} act hip {rel_l2(a, r):.2e} fp32 {rel_l2(r32, r):.2e} | grad hip {rel_l2(ga, gr):.2e} "
          f"fp32 {rel_l2(gr32, gr):.2e}")
for k, prm in m.named_parameters():
    if k in res["fp64"][1] and (".0.bias" in k or "norm.bias" in k):
        a = prm.grad.double().cpu()
        r = res["fp64"][1][k]
        print(f"{k:34s} hip {rel_l2(a, r):.2e} fp32 {rel_l2(res['fp32'][1][k], r):.2e} ref {rel_l2(g['g.' + k], r):.2e}")
