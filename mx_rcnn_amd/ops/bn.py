"""Frozen BatchNorm (use_global_stats=True) + ReLU as one op (reference
pre-activation units `rcnn/resnet.py:27-54`, eps 2e-5, ``fix_gamma`` for bn_data).

Gradients flow to x and, when they require grad, to gamma/beta (MXNet keeps the affine
parameters of global-stats BN trainable); the running statistics are constants.
"""
import torch

from . import grad_sink
from . import precision
from ._ext import ext_available, need_ext


class _FrozenBnRelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, mean, var, eps, fix_gamma, relu):
        ctx.eps, ctx.fix_gamma, ctx.relu = eps, fix_gamma, relu
        ctx.x2 = precision.is_pair(x)  # fp32-class pairs (ops/precision.py)
        if x.is_cuda:
            ext = need_ext()
            xc = x.contiguous(memory_format=torch.channels_last)
            y = ext.bn_relu_fwd(xc, gamma.float().contiguous(), beta.float().contiguous(), mean.float().contiguous(),
                                var.float().contiguous(), float(eps), bool(fix_gamma), bool(relu), ctx.x2)
            ctx.save_for_backward(xc, gamma, beta, mean, var)
            ctx.params = (gamma if gamma.is_leaf else None, beta if beta.is_leaf else None)
            return y
        ctx.save_for_backward(x, gamma, beta, mean, var)
        if ext_available() and x.dim() == 4:  # C++ twin (host_ops.h): one fused pass
            return need_ext().bn_relu_fwd_cpu(x.detach(), gamma.detach(), beta.detach(), mean, var, float(eps),
                                              bool(fix_gamma), bool(relu)).to(x.dtype)
        g = torch.ones_like(gamma) if fix_gamma else gamma
        s = g.float() * torch.rsqrt(var.float() + eps)
        t = beta.float() - mean.float() * s
        y = x.float() * s[None, :, None, None] + t[None, :, None, None]
        if relu:
            y = torch.relu(y)
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, mean, var = ctx.saved_tensors
        need_dx = ctx.needs_input_grad[0]
        need_p = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        if x.is_cuda:
            ext = need_ext()
            tg = grad_sink.target(ctx.params[0]) if ctx.needs_input_grad[1] and not ctx.fix_gamma else None
            tb = grad_sink.target(ctx.params[1]) if ctx.needs_input_grad[2] else None
            direct = tg is not None and tb is not None and tg.dtype == torch.float32 and tb.dtype == torch.float32
            dx, dg, db = ext.bn_relu_bwd(x, dy.to(x.dtype), gamma.float().contiguous(), beta.float().contiguous(),
                                         mean.float().contiguous(), var.float().contiguous(), float(ctx.eps),
                                         bool(ctx.fix_gamma), bool(ctx.relu), bool(need_dx), bool(need_p),
                                         tg if direct else None, tb if direct else None, None, ctx.x2)
            dx = dx if need_dx else None
            if direct:  # accumulated straight into the flat gradient buffers
                return dx, None, None, None, None, None, None, None
        else:
            g = torch.ones_like(gamma) if ctx.fix_gamma else gamma
            inv = torch.rsqrt(var.float() + ctx.eps)
            s = g.float() * inv
            t = beta.float() - mean.float() * s
            pre = x.float() * s[None, :, None, None] + t[None, :, None, None]
            gm = dy.float() * (pre > 0).float() if ctx.relu else dy.float()
            dx = (gm * s[None, :, None, None]).to(x.dtype) if need_dx else None
            xhat = (x.float() - mean.float()[None, :, None, None]) * inv[None, :, None, None]
            dg = (gm * xhat).sum(dim=(0, 2, 3))
            db = gm.sum(dim=(0, 2, 3))
        if ctx.fix_gamma or not ctx.needs_input_grad[1]:
            dg = None
        if not ctx.needs_input_grad[2]:
            db = None
        if dg is not None:
            dg = dg.to(gamma.dtype)
        if db is not None:
            db = db.to(beta.dtype)
        return dx, dg, db, None, None, None, None, None


def frozen_bn_relu(x, gamma, beta, mean, var, eps=2e-5, fix_gamma=False, relu=True):
    return _FrozenBnRelu.apply(x, gamma, beta, mean, var, float(eps), bool(fix_gamma), bool(relu))


class _TrainBnRelu(torch.autograd.Function):
    """Batch-statistics BN (+ReLU) of the ResNet head (csrc/hip/bn_train.hip); the running stats
    are updated in the forward kernel with MXNet's momentum convention."""

    @staticmethod
    def forward(ctx, x, gamma, beta, rmean, rvar, momentum, eps, fix_gamma, relu, parts=None):
        xc = x.contiguous(memory_format=torch.channels_last)
        ctx.x2 = x2 = precision.is_pair(x)
        if parts is not None:  # statistics partials from the producing conv's epilogue
            y, save = need_ext().bn_train_apply(xc, parts, gamma, beta, rmean, rvar, float(momentum), float(eps),
                                                bool(fix_gamma), bool(relu), x2)
        else:
            y, save = need_ext().bn_train_fwd(xc, gamma, beta, rmean, rvar, float(momentum), float(eps),
                                              bool(fix_gamma), bool(relu), x2)
        sm, si = save[0], save[1]
        ctx.save_for_backward(xc, gamma, beta, sm, si)
        ctx.params = (gamma if gamma.is_leaf else None, beta if beta.is_leaf else None)
        ctx.fix_gamma, ctx.relu = fix_gamma, relu
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, sm, si = ctx.saved_tensors
        need_g = ctx.needs_input_grad[1] and not ctx.fix_gamma
        need_b = ctx.needs_input_grad[2]
        tg = grad_sink.target(ctx.params[0]) if need_g else None
        tb = grad_sink.target(ctx.params[1]) if need_b else None
        direct = tg is not None and tb is not None and tg.dtype == torch.float32 and tb.dtype == torch.float32
        dx, dg, db = need_ext().bn_train_bwd(x, dy.contiguous(memory_format=torch.channels_last), gamma, beta, sm,
                                             si, bool(ctx.fix_gamma), bool(ctx.relu),
                                             bool(ctx.needs_input_grad[0]), tg if direct else None,
                                             tb if direct else None, ctx.x2)
        dx = dx if ctx.needs_input_grad[0] else None
        if direct:
            return dx, None, None, None, None, None, None, None, None, None
        dg = dg.to(gamma.dtype) if need_g else None
        db = db.to(beta.dtype) if need_b else None
        return dx, dg, db, None, None, None, None, None, None, None


def train_bn_relu(x, gamma, beta, rmean, rvar, momentum=0.9, eps=2e-5, fix_gamma=False, relu=True, parts=None):
    """parts: the (2 * nparts + 1, C) statistics partials of x from its conv's epilogue
    (conv_igemm_fwd(..., stat_shift=rmean)), which replace the statistics pass."""
    return _TrainBnRelu.apply(x, gamma, beta, rmean, rvar, float(momentum), float(eps), bool(fix_gamma), bool(relu),
                              parts)


def train_bn_eligible(x):
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 64 == 0 and
            x.is_contiguous(memory_format=torch.channels_last))
