"""Fused conv + frozen-BN + ReLU + residual ops for the pre-activation ResNet trunk.

Reference unit (`rcnn/resnet.py:5-64`): ``bn1 -> relu -> conv1 -> bn2 -> relu -> conv2 -> bn3 ->
relu -> conv3 (+ shortcut)``, stages 1-3 with ``use_global_stats=True``.  A frozen BN is a
per-channel affine, so it (and the ReLU, and the residual add, and the NEXT unit's bn1) ride
in the implicit-GEMM conv epilogue (csrc/hip/conv_igemm.hip ``ConvEpi``):

* ``conv_bn_relu``      a = relu(bn(conv(x)))          -- one kernel instead of two
* ``conv_add``          y = conv(x) + r                 -- no separate add kernel
* ``conv_add_bn_relu``  y = conv(x) + r, a = relu(bn'(y)) -- unit output AND next unit's act1

The raw conv output y is kept (bf16) for the BN backward, which runs the existing fused
BN-ReLU backward kernel (ops/bn.py) with gamma/beta gradients delivered straight into the flat
gradient buffers; for ``conv_add_bn_relu`` that kernel also adds the residual-path gradient
(``dres``), replacing autograd's gradient-accumulation add.  Numerics equal the unfused
sequence: the BN reads the bf16-rounded conv output, exactly like the separate kernels.
"""
import torch

from . import grad_sink
from ._ext import need_ext
from .conv import conv_backward


def _bn_args(bn):
    return (bn.gamma, bn.beta, bn.moving_mean, bn.moving_var)


def _bn_backward(ctx, y, d_act, gamma, beta, mean, var, gi, dres=None):
    """BN-ReLU backward on the saved raw conv output.  gi: index of gamma in needs_input_grad.
    Returns (d_y, dgamma, dbeta) with the parameter grads None when delivered directly."""
    need_g = ctx.needs_input_grad[gi] and not ctx.fix_gamma
    need_b = ctx.needs_input_grad[gi + 1]
    tg = grad_sink.target(ctx.bn_params[0]) if need_g else None
    tb = grad_sink.target(ctx.bn_params[1]) if need_b else None
    direct = (tg is not None or not need_g) and (tb is not None or not need_b) and (need_g or need_b)
    direct = direct and tg is not None and tb is not None and tg.dtype == torch.float32
    d_act = d_act.contiguous(memory_format=torch.channels_last).to(y.dtype)
    dy, dg, db = need_ext().bn_relu_bwd(y, d_act, gamma.float().contiguous(), beta.float().contiguous(),
                                       mean.float().contiguous(), var.float().contiguous(), float(ctx.eps),
                                       bool(ctx.fix_gamma), True, True, bool(need_g or need_b),
                                       tg if direct else None, tb if direct else None, dres)
    if direct:
        return dy, None, None
    dg = dg.to(gamma.dtype) if (need_g and dg is not None) else None
    db = db.to(beta.dtype) if (need_b and db is not None) else None
    return dy, dg, db


class _ConvBnRelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, gamma, beta, mean, var, stride, pad, eps, fix_gamma):
        x = x.contiguous(memory_format=torch.channels_last)
        y, a = need_ext().conv_igemm_fwd(x, w, None, stride, pad, False, 0, 0, None, [gamma, beta, mean, var],
                                         eps, fix_gamma, True)
        ctx.save_for_backward(x, w, y, gamma, beta, mean, var)
        ctx.param = w if w.is_leaf else None
        ctx.bn_params = (gamma if gamma.is_leaf else None, beta if beta.is_leaf else None)
        ctx.stride, ctx.pad, ctx.eps, ctx.fix_gamma = stride, pad, eps, fix_gamma
        return a

    @staticmethod
    def backward(ctx, d_act):
        x, w, y, gamma, beta, mean, var = ctx.saved_tensors
        dy, dg, db = _bn_backward(ctx, y, d_act, gamma, beta, mean, var, 2)
        dx, dw, _ = conv_backward(x, w, ctx.param, dy, ctx.stride, ctx.pad, False, ctx.needs_input_grad[0],
                                  ctx.needs_input_grad[1], False)
        return dx, dw, dg, db, None, None, None, None, None, None


class _ConvAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, res, stride, pad):
        x = x.contiguous(memory_format=torch.channels_last)
        res = res.contiguous(memory_format=torch.channels_last)
        y = need_ext().conv_igemm_fwd(x, w, None, stride, pad, False, 0, 0, res)[0]
        ctx.save_for_backward(x, w)
        ctx.param = w if w.is_leaf else None
        ctx.stride, ctx.pad = stride, pad
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx, dw, _ = conv_backward(x, w, ctx.param, dy, ctx.stride, ctx.pad, False, ctx.needs_input_grad[0],
                                  ctx.needs_input_grad[1], False)
        return dx, dw, (dy if ctx.needs_input_grad[2] else None), None, None


class _ConvAddBnRelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, res, gamma, beta, mean, var, stride, pad, eps, fix_gamma):
        x = x.contiguous(memory_format=torch.channels_last)
        res = res.contiguous(memory_format=torch.channels_last)
        y, a = need_ext().conv_igemm_fwd(x, w, None, stride, pad, False, 0, 0, res, [gamma, beta, mean, var],
                                         eps, fix_gamma, True)
        ctx.save_for_backward(x, w, y, gamma, beta, mean, var)
        ctx.param = w if w.is_leaf else None
        ctx.bn_params = (gamma if gamma.is_leaf else None, beta if beta.is_leaf else None)
        ctx.stride, ctx.pad, ctx.eps, ctx.fix_gamma = stride, pad, eps, fix_gamma
        return y, a

    @staticmethod
    def backward(ctx, d_out, d_act):
        x, w, y, gamma, beta, mean, var = ctx.saved_tensors
        d_out = d_out.contiguous(memory_format=torch.channels_last).to(y.dtype)
        # d_total = d_out + d(bn_relu)/dy * d_act, one kernel
        dt, dg, db = _bn_backward(ctx, y, d_act, gamma, beta, mean, var, 3, dres=d_out)
        dx, dw, _ = conv_backward(x, w, ctx.param, dt, ctx.stride, ctx.pad, False, ctx.needs_input_grad[0],
                                  ctx.needs_input_grad[1], False)
        return dx, dw, (dt if ctx.needs_input_grad[2] else None), dg, db, None, None, None, None, None, None


def conv_bn_relu(x, conv, bn):
    """relu(bn(conv(x))) with a frozen BN, one kernel (conv: layers.Conv without bias)."""
    return _ConvBnRelu.apply(x, conv.weight, *_bn_args(bn), int(conv.stride), int(conv.pad), float(bn.eps),
                             bool(bn.fix_gamma))


def conv_add(x, conv, res):
    return _ConvAdd.apply(x, conv.weight, res, int(conv.stride), int(conv.pad))


def conv_add_bn_relu(x, conv, res, bn):
    """(y, relu(bn(y))) with y = conv(x) + res."""
    return _ConvAddBnRelu.apply(x, conv.weight, res, *_bn_args(bn), int(conv.stride), int(conv.pad),
                                float(bn.eps), bool(bn.fix_gamma))
