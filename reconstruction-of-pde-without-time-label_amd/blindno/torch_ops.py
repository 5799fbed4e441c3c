"""The hot-path operations registered as torch operators (namespace ``blindno``):
``torch.ops.blindno.<name>`` -- visible to the profiler, torch.compile (fake-tensor shape
functions) and the dispatcher, with autograd formulas registered through torch.library.

    spectral_conv2d(x, w1, w2) -> (y, spectrum)       SpectralConv2d, 2d_FPE/FNOModules.py:156-178
    spectral_conv1d(x, w) -> (y, spectrum)            SpectralConv1d, 1d_FPE/FNOModules.py:47-59
    fno2d(inp, params, n_layers, modes1, modes2)      FNO2d.forward,  2d_FPE/FNOModules.py:218-240
    fno1d(inp, params, n_layers, modes)               FNO1d.forward,  1d_FPE/FNOModules.py:99-122
    project_mlp(z, w1, b1, w2, b2, Ho, Wo)            crop -> fc1 -> GELU -> fc2, FNOModules.py:234-239
    bag_mean(u, grid, w, b)                           2d_FPE/NIOModules.py:565-575
    conv2d(x, w, b, stride, padding)                  the NIO encoders' nn.Conv2d, Baselines.py:40-52
    mse_loss(pred, target)                            nn.MSELoss, 2d_FPE/train_fno.py:116,142
    time_averaged_relative_l2(pt_pred, pt_ref)        2d_Non_conservative_FPE/compute_time_error.py:321-333
  attention UNet ("BlinDNO"; blindno.unet):
    depthwise_conv(x, w, b)                           ConvNeXtBlock.dwconv, 2d_FPE/NIOModules.py:1047
    convnext_pointwise(xd, sc, lw, lb, w1, b1, w2, b2)  LN -> Linear -> GELU -> Linear -> + x, :1053-1062
    max_pool(x, kh, kw) -> (y, arg)                   MaxPool2d(2) / MaxPool1d(2), :1115
    conv_transpose(x, w, b, Ho, Wo)                   ConvTranspose2d(k = s = 2, output_padding), :1130-1134
    temporal_attention_mean(X, lw, lb, eps) -> (Y, state)  TemporalSelfAttention + bag mean, :1065-1083

Every operator runs only libblindno kernels (the same launch sequences as blindno.ops' autograd
Functions, which the models use on their fast path).  The spectral operators also return the
kept-mode spectrum of x (the tensor their backward needs) as a second, non-differentiable
output; ``fno2d`` / ``fno1d`` recompute their activations in the backward (one extra forward)
so the operator's outputs stay the reference's.  ``params`` lists an FNO's parameters in
``blindno.fno.fno_params`` order (2D spectral weights as their real (..., 2) views).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch.library import custom_op

from . import ops
from ._lib import call, ptr, query, stream_ptr

F32 = torch.float32


def _immediate(bwd):
    """Autograd formula wrapper: the operator's backward runs with reduction deferral
    suspended (ops.deferred_reductions, which GraphedBagStep wraps around backward(), would
    otherwise hand back unwritten reduction buffers that the backward clones or slices)."""
    def run(ctx, *grads):
        with ops.immediate_reductions():
            return bwd(ctx, *grads)
    return run


# ---------------------------------------------------------------------------- spectral conv 2D
def _spec2d_geom(x, w1):
    Bn, Ci, P1, P2 = x.shape
    Co, m1, m2 = w1.shape[1], w1.shape[2], w1.shape[3]
    return ops.SpecShape(Bn, Ci, Co, P1, P2, m1, m2, 2)


@custom_op("blindno::spectral_conv2d", mutates_args=())
def spectral_conv2d(x: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    ops.require_device(x, w1, w2)
    x, w1, w2 = ops._c(x), ops._c(w1), ops._c(w2)
    sh = _spec2d_geom(x, w1)
    Wt = ops.pack_weights((w1, w2), sh.P1, 2)
    X, Z = ops.spec_forward(x, 0, Wt, sh)
    y = ops.k_rowidft_epi(Z, None, None, None, sh.Bn, sh.Co, sh.P1, sh.P2, sh.m2, 0)
    return y, X


@spectral_conv2d.register_fake
def _(x, w1, w2):
    Bn, Ci, P1, P2 = x.shape
    Co, m1, m2 = w1.shape[1], w1.shape[2], w1.shape[3]
    K1 = ops.kept_rows_count(m1, P1)
    return x.new_empty(Bn, Co, P1, P2), x.new_empty(Bn, m2, Ci, K1, 2)


@custom_op("blindno::spectral_conv2d_backward", mutates_args=())
def spectral_conv2d_backward(dy: torch.Tensor, X: torch.Tensor, x: torch.Tensor, w1: torch.Tensor,
                             w2: torch.Tensor, need_dx: bool) -> List[torch.Tensor]:
    sh = _spec2d_geom(x, w1)
    Wt = ops.pack_weights((ops._c(w1), ops._c(w2)), sh.P1, 2)
    dWt, GZ = ops.spec_backward(ops._c(dy), X, Wt, sh)
    dw1, dw2 = ops.unpack_weights(dWt, (w1, w2), sh.P1, 2)
    dx = (ops.k_rowidft_bwd(GZ, None, None, None, sh.Bn, sh.Ci, sh.P1, sh.P2, sh.m2, 0)[0]
          if need_dx else torch.zeros_like(x))
    return [dx, dw1, dw2]


@spectral_conv2d_backward.register_fake
def _(dy, X, x, w1, w2, need_dx):
    return [torch.empty_like(x), torch.empty_like(w1), torch.empty_like(w2)]


def _spec2d_setup(ctx, inputs, output):
    x, w1, w2 = inputs
    ctx.save_for_backward(output[1], x, w1, w2)


def _spec2d_bwd(ctx, gy, gX):
    X, x, w1, w2 = ctx.saved_tensors
    dx, dw1, dw2 = torch.ops.blindno.spectral_conv2d_backward(gy, X, x, w1, w2,
                                                               bool(ctx.needs_input_grad[0]))
    return dx, dw1, dw2


spectral_conv2d.register_autograd(_immediate(_spec2d_bwd), setup_context=_spec2d_setup)


# ---------------------------------------------------------------------------- spectral conv 1D
@custom_op("blindno::spectral_conv1d", mutates_args=())
def spectral_conv1d(x: torch.Tensor, w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    ops.require_device(x, w)
    x = ops._c(x)
    Bn, Ci, P2 = x.shape
    Co, m = w.shape[1], w.shape[2]
    sh = ops.SpecShape(Bn, Ci, Co, 1, P2, 1, m, 1)
    Wt = ops.pack_weights((w.contiguous(),), 1, 1)
    X, Z = ops.spec_forward(x, 0, Wt, sh)
    y = ops.k_rowidft_epi(Z, None, None, None, Bn, Co, 1, P2, m, 0).view(Bn, Co, P2)
    return y, X


@spectral_conv1d.register_fake
def _(x, w):
    Bn, Ci, P2 = x.shape
    return (x.new_empty(Bn, w.shape[1], P2),
            x.new_empty(Bn, w.shape[2], Ci, 1, 2, dtype=torch.float32))


@custom_op("blindno::spectral_conv1d_backward", mutates_args=())
def spectral_conv1d_backward(dy: torch.Tensor, X: torch.Tensor, x: torch.Tensor, w: torch.Tensor,
                             need_dx: bool) -> List[torch.Tensor]:
    Bn, Ci, P2 = x.shape
    Co, m = w.shape[1], w.shape[2]
    sh = ops.SpecShape(Bn, Ci, Co, 1, P2, 1, m, 1)
    Wt = ops.pack_weights((w.contiguous(),), 1, 1)
    dWt, GZ = ops.spec_backward(ops._c(dy), X, Wt, sh)
    (dw,) = ops.unpack_weights(dWt, (w,), 1, 1)
    dx = (ops.k_rowidft_bwd(GZ, None, None, None, Bn, Ci, 1, P2, m, 0)[0].view(Bn, Ci, P2)
          if need_dx else torch.zeros_like(x))
    return [dx, dw]


@spectral_conv1d_backward.register_fake
def _(dy, X, x, w, need_dx):
    return [torch.empty_like(x), torch.empty_like(w)]


def _spec1d_setup(ctx, inputs, output):
    x, w = inputs
    ctx.save_for_backward(output[1], x, w)


def _spec1d_bwd(ctx, gy, gX):
    X, x, w = ctx.saved_tensors
    dx, dw = torch.ops.blindno.spectral_conv1d_backward(gy, X, x, w, bool(ctx.needs_input_grad[0]))
    return dx, dw


spectral_conv1d.register_autograd(_immediate(_spec1d_bwd), setup_context=_spec1d_setup)


# ---------------------------------------------------------------------------- FNO bodies
def _fno_meta(inp, params, dim, n_layers, m1, m2):
    nw = 2 if dim == 2 else 1
    width = params[0].shape[0]
    off = 2 + n_layers * (nw + 2)
    hidden, cout = params[off].shape[0], params[off + 2].shape[0]
    return ops.FNOMeta(dim, n_layers, width, m1, m2, hidden, cout, inp.shape[-1])


def _fno_fwd(inp, params, dim, n_layers, m1, m2):
    ops.require_device(inp, *params)
    meta = _fno_meta(inp, params, dim, n_layers, m1, m2)
    out, _ = ops.fno_forward(meta, ops._c(inp), [ops._c(p) for p in params], save=False)
    return out


def _fno_bwd(gout, inp, params, dim, n_layers, m1, m2, need_inp):
    meta = _fno_meta(inp, params, dim, n_layers, m1, m2)
    inp = ops._c(inp)
    prm = [ops._c(p) for p in params]
    _, saved = ops.fno_forward(meta, inp, prm, save=True)      # activations recomputed
    d_inp, grads = ops.fno_backward(meta, inp, prm, saved, gout, need_inp)
    # the small-parameter gradients are slices of one reduced buffer: outputs must not alias
    return [d_inp if d_inp is not None else torch.zeros_like(inp)] + [
        g.reshape(p.shape).clone() if g._base is not None else g.reshape(p.shape) for g, p in zip(grads, params)]


def _fno_out_shape(inp, params, dim, n_layers):
    """The reference's crop x[..., :-x1_padding, :-x2_padding] (pad names swapped,
    2d_FPE/FNOModules.py:234): (Bn, P1 - pW, P2 - pH, cout) -- not the input grid when N1 != N2."""
    meta = _fno_meta(inp, params, dim, n_layers, 1, 1)
    Bn, _, _, _, _, _, Ho, Wo = ops._fno_geometry(inp, meta)
    return (Bn, Ho, Wo, meta.cout) if dim == 2 else (Bn, Wo, meta.cout)


@custom_op("blindno::fno2d", mutates_args=())
def fno2d(inp: torch.Tensor, params: List[torch.Tensor], n_layers: int, modes1: int,
          modes2: int) -> torch.Tensor:
    return _fno_fwd(inp, params, 2, n_layers, modes1, modes2)


@fno2d.register_fake
def _(inp, params, n_layers, modes1, modes2):
    return inp.new_empty(_fno_out_shape(inp, params, 2, n_layers))


@custom_op("blindno::fno2d_backward", mutates_args=())
def fno2d_backward(gout: torch.Tensor, inp: torch.Tensor, params: List[torch.Tensor], n_layers: int,
                   modes1: int, modes2: int, need_inp: bool) -> List[torch.Tensor]:
    return _fno_bwd(gout, inp, params, 2, n_layers, modes1, modes2, need_inp)


@fno2d_backward.register_fake
def _(gout, inp, params, n_layers, modes1, modes2, need_inp):
    return [torch.empty_like(inp)] + [torch.empty_like(p) for p in params]


def _fno2d_setup(ctx, inputs, output):
    inp, params, n_layers, m1, m2 = inputs
    ctx.save_for_backward(inp, *params)
    ctx.cfg = (n_layers, m1, m2)


def _fno2d_grad(ctx, gout):
    inp, *params = ctx.saved_tensors
    n_layers, m1, m2 = ctx.cfg
    g = torch.ops.blindno.fno2d_backward(gout, inp, params, n_layers, m1, m2, bool(ctx.needs_input_grad[0]))
    return g[0], list(g[1:]), None, None, None


fno2d.register_autograd(_immediate(_fno2d_grad), setup_context=_fno2d_setup)


@custom_op("blindno::fno1d", mutates_args=())
def fno1d(inp: torch.Tensor, params: List[torch.Tensor], n_layers: int, modes: int) -> torch.Tensor:
    return _fno_fwd(inp, params, 1, n_layers, 1, modes)


@fno1d.register_fake
def _(inp, params, n_layers, modes):
    return inp.new_empty(_fno_out_shape(inp, params, 1, n_layers))


@custom_op("blindno::fno1d_backward", mutates_args=())
def fno1d_backward(gout: torch.Tensor, inp: torch.Tensor, params: List[torch.Tensor], n_layers: int,
                   modes: int, need_inp: bool) -> List[torch.Tensor]:
    return _fno_bwd(gout, inp, params, 1, n_layers, 1, modes, need_inp)


@fno1d_backward.register_fake
def _(gout, inp, params, n_layers, modes, need_inp):
    return [torch.empty_like(inp)] + [torch.empty_like(p) for p in params]


def _fno1d_setup(ctx, inputs, output):
    inp, params, n_layers, m = inputs
    ctx.save_for_backward(inp, *params)
    ctx.cfg = (n_layers, m)


def _fno1d_grad(ctx, gout):
    inp, *params = ctx.saved_tensors
    n_layers, m = ctx.cfg
    g = torch.ops.blindno.fno1d_backward(gout, inp, params, n_layers, m, bool(ctx.needs_input_grad[0]))
    return g[0], list(g[1:]), None, None


fno1d.register_autograd(_immediate(_fno1d_grad), setup_context=_fno1d_setup)


# ---------------------------------------------------------------------------- projection MLP
@custom_op("blindno::project_mlp", mutates_args=())
def project_mlp(z: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor,
                Ho: int, Wo: int) -> torch.Tensor:
    ops.require_device(z, w1, b1, w2, b2)
    z = ops._c(z)
    Bn, C, P1, P2 = z.shape
    Hd, Cout = w1.shape[0], w2.shape[0]
    out = ops._empty(Bn, Ho, Wo, Cout, like=z)
    call("blindno_project_fwd", ptr(z), ptr(ops._c(w1)), ptr(ops._c(b1)), ptr(ops._c(w2)), ptr(ops._c(b2)),
         ptr(out), Bn, C, P1, P2, Ho, Wo, Hd, Cout, Cout, 0, stream_ptr())
    return out


@project_mlp.register_fake
def _(z, w1, b1, w2, b2, Ho, Wo):
    return z.new_empty(z.shape[0], Ho, Wo, w2.shape[0])


@custom_op("blindno::project_mlp_backward", mutates_args=())
def project_mlp_backward(gout: torch.Tensor, z: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor,
                         w2: torch.Tensor, Ho: int, Wo: int) -> List[torch.Tensor]:
    z = ops._c(z)
    Bn, C, P1, P2 = z.shape
    Hd, Cout = w1.shape[0], w2.shape[0]
    dz = torch.zeros_like(z)
    npar = Hd * C + Hd + Cout * Hd + Cout
    nchunk = query("blindno_project_bwd_nchunk", Bn, Ho, Wo)
    partial = ops._empty(nchunk, npar, like=z)
    call("blindno_project_bwd", ptr(z), ptr(ops._c(w1)), ptr(ops._c(b1)), ptr(ops._c(w2)), ptr(ops._c(gout)),
         ptr(dz), ptr(partial), nchunk, Bn, C, P1, P2, Ho, Wo, Hd, Cout, Cout, 0, 1, stream_ptr())
    g = ops.reduce_partials(partial, nchunk, npar)
    o = Hd * C
    return [dz, g[:o].view(Hd, C).clone(), g[o:o + Hd].clone(), g[o + Hd:o + Hd + Cout * Hd].view(Cout, Hd).clone(),
            g[o + Hd + Cout * Hd:].clone()]


@project_mlp_backward.register_fake
def _(gout, z, w1, b1, w2, Ho, Wo):
    return [torch.empty_like(z), torch.empty_like(w1), torch.empty_like(b1), torch.empty_like(w2),
            w2.new_empty(w2.shape[0])]


def _proj_setup(ctx, inputs, output):
    z, w1, b1, w2, b2, Ho, Wo = inputs
    ctx.save_for_backward(z, w1, b1, w2)
    ctx.hw = (Ho, Wo)


def _proj_grad(ctx, gout):
    z, w1, b1, w2 = ctx.saved_tensors
    dz, dw1, db1, dw2, db2 = torch.ops.blindno.project_mlp_backward(gout, z, w1, b1, w2, *ctx.hw)
    return dz, dw1, db1, dw2, db2, None, None


project_mlp.register_autograd(_immediate(_proj_grad), setup_context=_proj_setup)


# ---------------------------------------------------------------------------- bag mean, conv, loss
@custom_op("blindno::bag_mean", mutates_args=())
def bag_mean(u: torch.Tensor, grid: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    with torch.no_grad():
        return ops.BagMeanFn.apply(u, grid, w, b)


@bag_mean.register_fake
def _(u, grid, w, b):
    return u.new_empty(u.shape[0], u.shape[2], w.shape[0])


@custom_op("blindno::bag_mean_backward", mutates_args=())
def bag_mean_backward(gy: torch.Tensor, w: torch.Tensor, L: int, d: int) -> torch.Tensor:
    B, S, width = gy.shape
    s = ops._empty(B, S, like=gy)
    call("blindno_bagmean_bwd", ptr(ops._c(gy)), ptr(ops._c(w)), ptr(s), B, S, d, width, L, stream_ptr())
    return s.unsqueeze(1).expand(B, L, S).contiguous()


@bag_mean_backward.register_fake
def _(gy, w, L, d):
    return gy.new_empty(gy.shape[0], L, gy.shape[1])


def _bag_setup(ctx, inputs, output):
    u, grid, w, b = inputs
    ctx.save_for_backward(w)
    ctx.Ld = (u.shape[1], grid.shape[1])


def _bag_grad(ctx, gy):
    (w,) = ctx.saved_tensors
    return torch.ops.blindno.bag_mean_backward(gy, w.detach(), *ctx.Ld), None, None, None


bag_mean.register_autograd(_immediate(_bag_grad), setup_context=_bag_setup)


@custom_op("blindno::conv2d", mutates_args=())
def conv2d(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], stride: List[int],
           padding: List[int]) -> torch.Tensor:
    with torch.no_grad():
        return ops.Conv2dFn.apply(x, w, b, tuple(stride), tuple(padding))


@conv2d.register_fake
def _(x, w, b, stride, padding):
    N, _, H, W = x.shape
    Co, _, KH, KW = w.shape
    return x.new_empty(N, Co, (H + 2 * padding[0] - KH) // stride[0] + 1, (W + 2 * padding[1] - KW) // stride[1] + 1)


@custom_op("blindno::conv2d_backward", mutates_args=())
def conv2d_backward(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride: List[int],
                    padding: List[int]) -> List[torch.Tensor]:
    N, Ci, Hi, Wi = x.shape
    Co, _, KH, KW = w.shape
    g = (N, Ci, Hi, Wi, Co, KH, KW, stride[0], stride[1], padding[0], padding[1])
    dy, x, w = ops._c(dy), ops._c(x), ops._c(w)
    dx = ops.k_conv2d_bwd_data(dy, w, g)
    ncol = Ci * KH * KW + 1
    ns = query("blindno_conv2d_wgrad_nsplit", *g)
    dwb = ops._empty(Co, ncol, like=dy)
    part = ops._empty(ns, Co * ncol, like=dy) if ns > 1 else None
    call("blindno_conv2d_bwd_weight", ptr(dy), ptr(x), ptr(dwb), ptr(part), ns, *g, stream_ptr())
    return [dx, dwb[:, :-1].reshape(Co, Ci, KH, KW).contiguous(), dwb[:, -1].contiguous()]


@conv2d_backward.register_fake
def _(dy, x, w, stride, padding):
    return [torch.empty_like(x), torch.empty_like(w), w.new_empty(w.shape[0])]


def _conv_setup(ctx, inputs, output):
    x, w, b, stride, padding = inputs
    ctx.save_for_backward(x, w)
    ctx.cfg = (list(stride), list(padding), b is not None)


def _conv_grad(ctx, dy):
    x, w = ctx.saved_tensors
    stride, padding, has_b = ctx.cfg
    dx, dw, db = torch.ops.blindno.conv2d_backward(dy, x, w, stride, padding)
    return dx, dw, (db if has_b else None), None, None


conv2d.register_autograd(_immediate(_conv_grad), setup_context=_conv_setup)


@custom_op("blindno::mse_loss", mutates_args=())
def mse_loss(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    with torch.no_grad():
        return ops.MSEFn.apply(pred, target)


@mse_loss.register_fake
def _(pred, target):
    return pred.new_empty(())


@custom_op("blindno::mse_loss_backward", mutates_args=())
def mse_loss_backward(g: torch.Tensor, pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    pred, target = ops._c(pred), ops._c(target)
    n = pred.numel()
    nblk = ops._mse_blocks(n)
    partial = ops._empty(nblk, like=pred)
    grad = torch.empty_like(pred)
    call("blindno_mse", ptr(pred), ptr(target), ptr(partial), ptr(grad), n, nblk, ptr(ops._c(g.reshape(1))),
         stream_ptr())
    return grad


@mse_loss_backward.register_fake
def _(g, pred, target):
    return torch.empty_like(pred)


def _mse_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _mse_grad(ctx, g):
    pred, target = ctx.saved_tensors
    return torch.ops.blindno.mse_loss_backward(g, pred, target), None


mse_loss.register_autograd(_immediate(_mse_grad), setup_context=_mse_setup)


@custom_op("blindno::time_averaged_relative_l2", mutates_args=())
def time_averaged_relative_l2(pt_pred: torch.Tensor, pt_ref: torch.Tensor) -> torch.Tensor:
    return torch.tensor(ops.time_averaged_relative_l2(pt_pred, pt_ref), dtype=torch.float64,
                        device=pt_pred.device)


@time_averaged_relative_l2.register_fake
def _(pt_pred, pt_ref):
    return pt_pred.new_empty((), dtype=torch.float64)


# ---------------------------------------------------------------------------- attention UNet
def _unet():
    from . import unet
    return unet


@custom_op("blindno::depthwise_conv", mutates_args=())
def depthwise_conv(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return _unet().dwconv_fwd(x, w, b)


@depthwise_conv.register_fake
def _(x, w, b):
    return torch.empty_like(x)


@custom_op("blindno::depthwise_conv_backward", mutates_args=())
def depthwise_conv_backward(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor) -> List[torch.Tensor]:
    return list(_unet().dwconv_bwd(dy, x, w))


@depthwise_conv_backward.register_fake
def _(dy, x, w):
    return [torch.empty_like(x), torch.empty_like(w), w.new_empty(w.shape[0])]


def _dw_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0], inputs[1])


def _dw_grad(ctx, gy):
    x, w = ctx.saved_tensors
    dx, dw, db = torch.ops.blindno.depthwise_conv_backward(gy, x, w)
    return dx, dw, db


depthwise_conv.register_autograd(_immediate(_dw_grad), setup_context=_dw_setup)


@custom_op("blindno::convnext_pointwise", mutates_args=())
def convnext_pointwise(xd: torch.Tensor, sc: torch.Tensor, lw: torch.Tensor, lb: torch.Tensor, w1: torch.Tensor,
                       b1: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor) -> torch.Tensor:
    return _unet().cnx_pw_fwd(xd, sc, lw, lb, w1, b1, w2, b2)


@convnext_pointwise.register_fake
def _(xd, sc, lw, lb, w1, b1, w2, b2):
    return torch.empty_like(xd)


@custom_op("blindno::convnext_pointwise_backward", mutates_args=())
def convnext_pointwise_backward(dy: torch.Tensor, xd: torch.Tensor, lw: torch.Tensor, lb: torch.Tensor,
                                w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor) -> List[torch.Tensor]:
    return [t.clone() if t.storage_offset() else t for t in _unet().cnx_pw_bwd(dy, xd, lw, lb, w1, b1, w2)]


@convnext_pointwise_backward.register_fake
def _(dy, xd, lw, lb, w1, b1, w2):
    C = xd.shape[1]
    return [torch.empty_like(xd), lw.new_empty(C), lw.new_empty(C), torch.empty_like(w1), b1.new_empty(4 * C),
            torch.empty_like(w2), lw.new_empty(C)]


def _cnx_setup(ctx, inputs, output):
    xd, sc, lw, lb, w1, b1, w2, b2 = inputs
    ctx.save_for_backward(xd, lw, lb, w1, b1, w2)


def _cnx_grad(ctx, gy):
    xd, lw, lb, w1, b1, w2 = ctx.saved_tensors
    dxd, dlw, dlb, dw1, db1, dw2, db2 = torch.ops.blindno.convnext_pointwise_backward(gy, xd, lw, lb, w1, b1, w2)
    return dxd, gy, dlw, dlb, dw1, db1, dw2, db2


convnext_pointwise.register_autograd(_immediate(_cnx_grad), setup_context=_cnx_setup)


@custom_op("blindno::max_pool", mutates_args=())
def max_pool(x: torch.Tensor, kh: int, kw: int) -> Tuple[torch.Tensor, torch.Tensor]:
    return _unet().maxpool_fwd(x, kh, kw)


@max_pool.register_fake
def _(x, kh, kw):
    N, C, H, W = x.shape
    return x.new_empty(N, C, H // kh, W // kw), x.new_empty(N, C, H // kh, W // kw, dtype=torch.uint8)


@custom_op("blindno::max_pool_backward", mutates_args=())
def max_pool_backward(dy: torch.Tensor, arg: torch.Tensor, H: int, W: int, kh: int, kw: int) -> torch.Tensor:
    return _unet().maxpool_bwd(dy, arg, H, W, kh, kw)


@max_pool_backward.register_fake
def _(dy, arg, H, W, kh, kw):
    return dy.new_empty(dy.shape[0], dy.shape[1], H, W)


def _mp_setup(ctx, inputs, output):
    x, kh, kw = inputs
    ctx.save_for_backward(output[1])
    ctx.geom = (x.shape[2], x.shape[3], kh, kw)


def _mp_grad(ctx, gy, garg):
    (arg,) = ctx.saved_tensors
    return torch.ops.blindno.max_pool_backward(gy, arg, *ctx.geom), None, None


max_pool.register_autograd(_immediate(_mp_grad), setup_context=_mp_setup)


@custom_op("blindno::conv_transpose", mutates_args=())
def conv_transpose(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, Ho: int, Wo: int) -> torch.Tensor:
    return _unet().convt_fwd(x, w, b, Ho, Wo)


@conv_transpose.register_fake
def _(x, w, b, Ho, Wo):
    return x.new_empty(x.shape[0], w.shape[1], Ho, Wo)


@custom_op("blindno::conv_transpose_backward", mutates_args=())
def conv_transpose_backward(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor) -> List[torch.Tensor]:
    return [t.clone() if t.storage_offset() else t for t in _unet().convt_bwd(dy, x, w)]


@conv_transpose_backward.register_fake
def _(dy, x, w):
    return [torch.empty_like(x), torch.empty_like(w), w.new_empty(w.shape[1])]


def _ct_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0], inputs[1])


def _ct_grad(ctx, gy):
    x, w = ctx.saved_tensors
    dx, dw, db = torch.ops.blindno.conv_transpose_backward(gy, x, w)
    return dx, dw, db, None, None


conv_transpose.register_autograd(_immediate(_ct_grad), setup_context=_ct_setup)


@custom_op("blindno::temporal_attention_mean", mutates_args=())
def temporal_attention_mean(X: torch.Tensor, lw: torch.Tensor, lb: torch.Tensor,
                            eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    return _unet().tok_attn_fwd(X, lw, lb, eps)


@temporal_attention_mean.register_fake
def _(X, lw, lb, eps):
    B, L, D = X.shape
    n = 4 * B * L + B * L + 2 * B * L * L + B + B * D
    return X.new_empty(B, D), X.new_empty(n)


@custom_op("blindno::temporal_attention_mean_backward", mutates_args=())
def temporal_attention_mean_backward(dY: torch.Tensor, X: torch.Tensor, lw: torch.Tensor,
                                     state: torch.Tensor) -> List[torch.Tensor]:
    return list(_unet().tok_attn_bwd(dY, X, lw, state))


@temporal_attention_mean_backward.register_fake
def _(dY, X, lw, state):
    return [torch.empty_like(X), torch.empty_like(lw), torch.empty_like(lw)]


def _ta_setup(ctx, inputs, output):
    X, lw, lb, eps = inputs
    ctx.save_for_backward(X, lw, output[1])


def _ta_grad(ctx, gY, gstate):
    X, lw, state = ctx.saved_tensors
    dX, dlw, dlb = torch.ops.blindno.temporal_attention_mean_backward(gY, X, lw, state)
    return dX, dlw, dlb, None


temporal_attention_mean.register_autograd(_immediate(_ta_grad), setup_context=_ta_setup)


REGISTERED = ("spectral_conv2d", "spectral_conv1d", "fno2d", "fno1d", "project_mlp", "bag_mean", "conv2d",
              "mse_loss", "time_averaged_relative_l2", "depthwise_conv", "convnext_pointwise", "max_pool",
              "conv_transpose", "temporal_attention_mean")
