"""The per-experiment drop-in shims (dropin/<experiment>/*.py, dropin/run.py) expose the
reference's names with the reference's state_dict layouts (CPU only: construction, imports,
launcher)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import GOLDEN, ROOT

DROPIN = os.path.join(ROOT, "dropin")

# (experiment, constructor expression, layouts.json key or None)
CASES = [
    ("2d_FPE", "NIOFP2D_FNO(2,3,100,25,3,12,32,2)", "2d_FPE.NIOFP2D_FNO(2,3,100,25,3,12,32,2)"),
    ("2d_FPE", "NIOFP2D(2,3,100,25,3,12,32,2)", "2d_FPE.NIOFP2D(2,3,100,25,3,12,32,2)"),
    ("2d_Non_conservative_FPE", "NIOFP2D_FNO(2,3,100,25,3,12,32,2)", "2d_NC.NIOFP2D_FNO(2,3,100,25,3,12,32,2)"),
    ("2d_Non_conservative_FPE", "NIOFP2D(2,3,100,25,3,12,32,2)", "2d_NC.NIOFP2D(2,3,100,25,3,12,32,2)"),
    ("1d_FPE", "NIOFP_FNO(3,30,15,2,'cpu')", "1d_FPE.NIOFP_FNO(3,30,15,2)"),
    ("1d_GPE", "NIOFP_FNO(3,20,40,1,'cpu')", "1d_GPE.NIOFP_FNO(3,20,40,1)"),
    # the attention UNet ("BlinDNO"): each experiment's own copy
    ("2d_FPE", "PermInvUNet_attn(in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=(61, 61))",
     "2d.PermInvUNet_attn(1,2,1,4,(61,61))"),
    ("2d_Non_conservative_FPE", "PermInvUNet_attn(in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=(61, 61))",
     "2d_NC.PermInvUNet_attn(1,2,1,4,(61,61))"),
    ("1d_FPE", "PermInvUNet_attn1D_bag(in_ch=1, out_ch=2, base_ch=1, depth=5, input_size=80, device='cpu')",
     "1d.PermInvUNet_attn1D_bag(1,2,1,5,80)"),
    ("1d_FPE", "PermInvUNet_attn1D(in_ch=1, out_ch=2, base_ch=1, depth=6, input_size=80, device='cpu')",
     "1d.PermInvUNet_attn1D(1,2,1,6,80)"),
    ("1d_GPE", "PermInvUNet_attn1D_bag(in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=128, device='cpu')",
     "1d_GPE.PermInvUNet_attn1D_bag(1,2,1,4,128)"),
    ("1d_GPE", "PermInvUNet_attn1D_bag_GPE(in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=128, device='cpu', "
     "width=20, modes=40)", "1d_GPE.PermInvUNet_attn1D_bag_GPE(1,2,1,4,128,20,40)"),
]

IMPORTS = {
    "2d_FPE": "from NIOModules import NIOFP2D, NIOFP2D_FNO, NIOFP2D_FNO_attn",
    "2d_Non_conservative_FPE": "from NIOModules import PermInvUNet_attn, NIOFP2D, NIOFP2D_FNO",
    "1d_FPE": "from NIOModules import NIOFP, NIOFP_FNO, PermInvUNet_attn1D, PermInvUNet_attn1D_bag",
    "1d_GPE": "from NIOModules import NIOFP_schrodinger, NIOFP_FNO, PermInvUNet_attn1D_bag_GPE",
}


def _run(code, exp):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    return subprocess.run([sys.executable, "-c", f"import sys; sys.path.insert(0, {os.path.join(DROPIN, exp)!r})\n" + code],
                          capture_output=True, text=True, env=env, timeout=240)


@pytest.mark.parametrize("exp,ctor,key", CASES)
def test_dropin_layout(exp, ctor, key):
    code = ("import json, torch\nfrom NIOModules import *\nfrom FNOModules import FNO2d, FNO1d, SpectralConv2d\n"
            "from DeepONetModules import FFN, DeepOnetNoBiasOrg\nfrom Baselines import Encoder2D, Encoder\n"
            f"m = {ctor}\n"
            "print(json.dumps([[k, list(v.shape), str(v.dtype).replace('torch.', '')] for k, v in m.state_dict().items()]))\n")
    r = _run(code, exp)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout.strip().splitlines()[-1])
    lay = json.load(open(os.path.join(GOLDEN, "layouts.json")))
    assert got == lay[key]


@pytest.mark.parametrize("exp", sorted(IMPORTS))
def test_reference_import_lines_work(exp):
    # the exact import lines of the reference scripts (train_fno.py:8, eval_fno.py:7, ...)
    r = _run(IMPORTS[exp] + "\nprint('ok')", exp)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr


def test_out_of_scope_classes_raise():
    r = _run("from NIOModules import NIOFP2D_Trans_attn\ntry:\n    NIOFP2D_Trans_attn(2,3,100,25,3,12,32,2)\n"
             "except NotImplementedError as e:\n    print('raised', 'SURVEY' in str(e))\n", "2d_FPE")
    assert r.stdout.strip() == "raised True", r.stderr


def test_attention_variant_is_served():
    r = _run("from NIOModules import NIOFP2D_FNO_attn\n"
             "m = NIOFP2D_FNO_attn(2,3,100,25,3,12,32,2,64,64)\n"
             "print(type(m).__mro__[1].__name__, sorted(n for n, _ in m.named_children()))\n",
             "2d_Non_conservative_FPE")
    assert r.stdout.strip() == "NIOFP2D_FNO_attn ['FNO_input', 'fc0', 'fno_Fx', 'fno_Fy']", r.stderr


def test_launcher_runs_script_with_shims(tmp_path):
    # a stand-in "experiment directory" holding its own (different) NIOModules.py, as the
    # reference does: the launcher must make the script see the drop-in instead
    d = tmp_path / "2d_FPE"
    d.mkdir()
    (d / "NIOModules.py").write_text("raise ImportError('reference module must be shadowed')\n")
    (d / "train_fno.py").write_text(
        "import os\nfrom NIOModules import NIOFP2D_FNO\nimport NIOModules\n"
        "print(NIOFP2D_FNO.__mro__[1].__module__, os.getcwd() == os.path.dirname(os.path.abspath(__file__)))\n")
    r = subprocess.run([sys.executable, os.path.join(DROPIN, "run.py"), "2d_FPE", str(d / "train_fno.py")],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "blindno.nio True"


def test_fplanck_shim_names():
    # compute_time_error.py's `from fplanck import fokker_planck, boundary, gaussian_pdf`
    r = _run("from fplanck import fokker_planck, boundary, gaussian_pdf, potential_from_data\n"
             "s = fokker_planck(temperature=300, drag=1e-9, extent=[100e-9, 80e-9], resolution=10e-9,\n"
             "                  force=lambda x, y: [0 * x, 0 * y], boundary=boundary.reflecting)\n"
             "print(s.grid.shape)\n", "2d_Non_conservative_FPE")
    assert r.stdout.strip() == "(2, 10, 8)", r.stderr


# the fplanck import lines of the reference scripts, per experiment (1d_FPE/compute_time_error.py:8-15,
# dataset_1d_drift_diffusion.py:3, cal_trajectory*.py:3; 2d_FPE/test_datagen.py:3, cal_traj.py:3;
# 2d_Non_conservative_FPE/compute_time_error.py:44, testdata_gen.py:3)
FPLANCK_IMPORTS = {
    "1d_FPE": "from fplanck import fokker_planck, boundary, gaussian_pdf, combine, gaussian_potential, "
              "potential_from_data",
    "2d_FPE": "from fplanck import fokker_planck, boundary, gaussian_pdf, combine, gaussian_potential",
    "2d_Non_conservative_FPE": "from fplanck import fokker_planck, boundary, gaussian_pdf",
}


@pytest.mark.parametrize("exp", sorted(FPLANCK_IMPORTS))
def test_fplanck_shim_serves_every_reference_import(exp):
    r = _run(FPLANCK_IMPORTS[exp] + "\nimport fplanck\n"
             "U = fplanck.combine(fplanck.gaussian_potential(0.0, 1.0, 2.0), fplanck.gaussian_potential(1.0, 1.0, 1.0))\n"
             "print(sorted(fplanck.__all__), float(U(0.0)) < 0)\n", exp)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == ("['boundary', 'combine', 'fokker_planck', 'gaussian_pdf', 'gaussian_potential', "
                                "'potential_from_data'] True"), r.stdout
