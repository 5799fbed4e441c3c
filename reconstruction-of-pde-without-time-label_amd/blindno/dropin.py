"""Per-experiment module namespaces with the reference's exact class names and constructor
signatures, for the shims under ``dropin/<experiment>/``.

The reference keeps one copy of ``FNOModules`` / ``NIOModules`` / ``DeepONetModules`` /
``Baselines`` per experiment directory; the copies differ only in head names, grid-specific
encoder kernels and the 1D GPE head layout:

  2d_FPE                    NIOFP2D / NIOFP2D_FNO heads fno_drift, fno_diffusion; Encoder2D (2,1)
                            (2d_FPE/NIOModules.py:14-83,508-581; 2d_FPE/Baselines.py:200)
  2d_Non_conservative_FPE   heads fno_Fx, fno_Fy; Encoder2D (3,2)
                            (2d_Non_conservative_FPE/NIOModules.py:13-82,503-577; Baselines.py:200)
  1d_FPE                    NIOFP / NIOFP_FNO heads fno_drift, fno_diffusion; Encoder (5,4,15)
                            (1d_FPE/NIOModules.py:15-155; 1d_FPE/Baselines.py:254-287)
  1d_GPE                    NIOFP_schrodinger / NIOFP_FNO head fno_V; Encoder (5,7,4) + conv4
                            (1d_GPE/NIOModules.py:160-289; 1d_GPE/Baselines.py:254-290)

The attention UNet ("BlinDNO") maps to blindno.unet: PermInvUNet_attn (2d_FPE),
its ConvBlock copy PermInvUNet_attn_NC (2d_Non_conservative_FPE), PermInvUNet_attn1D(_bag)
(1d_FPE) and the one-head 1d_GPE copies.  Classes outside the hot-path scope (Transolver /
plain-UNet / 3D / ODE variants) are importable -- the
reference scripts import them next to the in-scope ones -- but raise NotImplementedError when
constructed.
"""
from __future__ import annotations

import types

from . import deeponet as _don
from . import encoders as _enc
from . import fno as _fno
from . import nio as _nio
from . import unet as _unet


def _out_of_scope(name: str, where: str):
    def __init__(self, *a, **k):
        raise NotImplementedError(
            f"{name} ({where}) is outside the MI355X hot-path scope (SURVEY.md section 2); "
            "only the FNO/NIO models are implemented")
    return type(name, (object,), {"__init__": __init__, "__doc__": f"Out of scope: {where}."})


# ------------------------------------------------------------------------------- 2D FPE
class _NIOFP2D_FNO_2d(_nio.NIOFP2D_FNO):
    def __init__(self, input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                 width, modes, output_dim):
        super().__init__(input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                         width, modes, output_dim, heads=("fno_drift", "fno_diffusion"),
                         branch_last_kernel=(2, 1))


class _NIOFP2D_2d(_nio.NIOFP2D):
    def __init__(self, input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                 width, modes, output_dim):
        super().__init__(input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                         width, modes, output_dim, heads=("fno_drift", "fno_diffusion"),
                         branch_last_kernel=(2, 1))


class _NIOFP2D_FNO_nc(_nio.NIOFP2D_FNO):
    def __init__(self, input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                 width, modes, output_dim):
        super().__init__(input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                         width, modes, output_dim, heads=("fno_Fx", "fno_Fy"),
                         branch_last_kernel=(3, 2))


class _NIOFP2D_nc(_nio.NIOFP2D):
    def __init__(self, input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                 width, modes, output_dim):
        super().__init__(input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                         width, modes, output_dim, heads=("fno_Fx", "fno_Fy"),
                         branch_last_kernel=(3, 2))


class _NIOFP2D_FNO_attn_2d(_nio.NIOFP2D_FNO_attn):
    def __init__(self, input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                 width, modes, output_dim, nx, ny):
        super().__init__(input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                         width, modes, output_dim, nx, ny, heads=("fno_drift", "fno_diffusion"))


class _NIOFP2D_FNO_attn_nc(_nio.NIOFP2D_FNO_attn):
    def __init__(self, input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                 width, modes, output_dim, nx, ny):
        super().__init__(input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                         width, modes, output_dim, nx, ny, heads=("fno_Fx", "fno_Fy"))


# ------------------------------------------------------------------------------- 1D
class _NIOFP_FNO_1d(_nio.NIOFP_FNO):
    def __init__(self, fno_layers, width, modes, output_dim, device):
        super().__init__(fno_layers, width, modes, output_dim, device,
                         heads=("fno_drift", "fno_diffusion"))


class _NIOFP_1d(_nio.NIOFP):
    def __init__(self, input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                 width, modes, output_dim, device):
        super().__init__(input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                         width, modes, output_dim, device, heads=("fno_drift", "fno_diffusion"),
                         encoder_kernels=(5, 4, 15), encoder_conv4=False)


class _NIOFP_FNO_gpe(_nio.NIOFP_FNO):
    def __init__(self, fno_layers, width, modes, output_dim, device):
        super().__init__(fno_layers, width, modes, output_dim, device, heads=("fno_V",))


_COMMON_FNO = dict(SpectralConv1d=_fno.SpectralConv1d, SpectralConv2d=_fno.SpectralConv2d,
                   SpectralConv3d=_fno.SpectralConv3d, FNO1d=_fno.FNO1d, FNO2d=_fno.FNO2d,
                   FNO3d=_fno.FNO3d, MLP=_fno.MLP)
_COMMON_DON = dict(FFN=_don.FFN, DeepOnetNoBiasOrg=_don.DeepOnetNoBiasOrg,
                   FeedForwardNN=_don.FeedForwardNN, FourierFeatures=_don.FourierFeatures,
                   Swish=_don.Swish, Sin=_don.Sin, activation=_don.activation,
                   kaiming_init=_don.kaiming_init, init_xavier=_don.init_xavier)
_COMMON_BASE = dict(ConvBlock=_enc.ConvBlock, Encoder2D=_enc.Encoder2D, Encoder=_enc.Encoder)


def _oos(where, *names):
    return {n: _out_of_scope(n, where) for n in names}


_2D_OOS = ("NIOFP2D_Trans", "NIOFP2D_Trans_attn", "NIOFP2D_attn",
           "NIOFP_ode", "NIOFP3D", "PermInvUNet")

EXPERIMENTS = {
    "2d_FPE": dict(
        NIOModules=dict(NIOFP2D=_NIOFP2D_2d, NIOFP2D_FNO=_NIOFP2D_FNO_2d, NIOFP=_NIOFP_1d,
                        NIOFP2D_FNO_attn=_NIOFP2D_FNO_attn_2d,
                        PermInvUNet_attn=_unet.PermInvUNet_attn, ConvNeXtBlock=_unet.ConvNeXtBlock,
                        TemporalSelfAttention=_unet.TemporalSelfAttention,
                        draw_bag=_nio.draw_bag, **_oos("2d_FPE/NIOModules.py", *_2D_OOS)),
    ),
    "2d_Non_conservative_FPE": dict(
        NIOModules=dict(NIOFP2D=_NIOFP2D_nc, NIOFP2D_FNO=_NIOFP2D_FNO_nc, NIOFP=_NIOFP_1d,
                        NIOFP2D_FNO_attn=_NIOFP2D_FNO_attn_nc,
                        PermInvUNet_attn=_unet.PermInvUNet_attn_NC,
                        TemporalSelfAttention=_unet.TemporalSelfAttention,
                        draw_bag=_nio.draw_bag,
                        **_oos("2d_Non_conservative_FPE/NIOModules.py", *_2D_OOS)),
    ),
    "1d_FPE": dict(
        NIOModules=dict(NIOFP=_NIOFP_1d, NIOFP_FNO=_NIOFP_FNO_1d, draw_bag=_nio.draw_bag,
                        ConvNeXtBlock1D=_unet.ConvNeXtBlock1D,
                        TemporalSelfAttention1D=_unet.TemporalSelfAttention1D,
                        PermInvUNet_attn1D=_unet.PermInvUNet_attn1D,
                        PermInvUNet_attn1D_bag=_unet.PermInvUNet_attn1D_bag),
    ),
    "1d_GPE": dict(
        NIOModules=dict(NIOFP_schrodinger=_nio.NIOFP_schrodinger, NIOFP_FNO=_NIOFP_FNO_gpe,
                        draw_bag=_nio.draw_bag,
                        ConvNeXtBlock1D=_unet.ConvNeXtBlock1D,
                        TemporalSelfAttention1D=_unet.TemporalSelfAttention1D,
                        PermInvUNet_attn1D_bag=_unet.PermInvUNet_attn1D_bag_V,
                        PermInvUNet_attn1D_bag_GPE=_unet.PermInvUNet_attn1D_bag_GPE,
                        **_oos("1d_GPE/NIOModules.py", "NIOFP2D", "NIOFP")),
    ),
}
for _exp in EXPERIMENTS.values():
    _exp["FNOModules"] = dict(_COMMON_FNO)
    _exp["DeepONetModules"] = dict(_COMMON_DON)
    _exp["Baselines"] = dict(_COMMON_BASE)


def module(experiment: str, name: str) -> types.ModuleType:
    """A module object holding the reference names of ``<experiment>/<name>.py``."""
    try:
        ns = EXPERIMENTS[experiment][name]
    except KeyError:
        raise KeyError(f"no drop-in for {experiment}/{name}.py; known: "
                       f"{ {e: sorted(v) for e, v in EXPERIMENTS.items()} }") from None
    m = types.ModuleType(name, f"blindno drop-in for {experiment}/{name}.py")
    m.__dict__.update(ns)
    m.__all__ = sorted(ns)
    return m


def install(experiment: str, target_globals: dict, name: str) -> None:
    """Populate a shim module's globals with the reference names (used by dropin/*/*.py)."""
    m = module(experiment, name)
    target_globals.update({k: getattr(m, k) for k in m.__all__})
    target_globals["__all__"] = m.__all__
