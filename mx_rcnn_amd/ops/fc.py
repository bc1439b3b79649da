"""FullyConnected (+bias, +ReLU, +inverted dropout) on the MFMA implicit-GEMM kernel.

MXNet ``FullyConnected`` is ``y = x W^T + b`` with W stored (out, in) -- exactly the (Cout, K)
K-contiguous operand layout of the conv kernel, so an FC over M rows is the 1x1 convolution of
an (M, K, 1, 1) map: no separate GEMM kernel, and the conv epilogue fuses bias, ReLU and the
head's Dropout (`rcnn/symbol.py:96-107`: fc6 -> relu6 -> drop6 -> fc7 -> relu7 -> drop7).

Dropout is counter-based (Philox-4x32-10 of (seed, step, element), csrc/hip/common.h): the step
lives in a device tensor the trainer advances each update, so a replayed hipGraph draws a new
mask every step and no mask is stored.  With ReLU before dropout the backward needs no mask at
all: the output is positive exactly where ReLU passed AND the element was kept, so
``d pre = dy * (y > 0) / (1 - p)``.

Backward: the data gradient runs the same kernel on ``dy`` with the TRANSPOSED weight (kept by
the FlatParamStore's filter cache, refreshed after every update; ``W^T`` of fc6 is 205 MB bf16,
nothing on 288 GB), the weight gradient runs the MFMA wgrad kernel straight into the flat
gradient buffer (ops/grad_sink.py).  Small outputs (the cls / bbox predictors, N = 21..324) fall
back to torch matmuls for the parts the kernels do not tile.
"""
import os
import zlib

import torch
import torch.nn.functional as F

from . import grad_sink
from ._ext import need_ext
from .conv import LOWP, cached_dgrad_weight, wgrad_enabled


def layer_seed(name, base=None):
    """32-bit dropout key of a layer: the process seed mixed with a hash of the layer name."""
    if base is None:
        base = torch.initial_seed()
    return (int(base) ^ zlib.crc32(name.encode())) & 0x7FFFFFFF


def fc_eligible(x, w):
    if os.environ.get('MXR_FC_KERNEL', '1') == '0':
        return False
    return (x.is_cuda and x.dtype in LOWP and w.dtype == x.dtype and x.dim() == 2 and
            x.shape[1] % 64 == 0)


def _as_map(t):
    """(M, K) row-major -> (M, K, 1, 1), which is channels_last contiguous."""
    return t.contiguous().view(t.shape[0], t.shape[1], 1, 1)


class _FC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu, drop_p, seed, step):
        ext = need_ext()
        y = ext.conv_igemm_fwd(_as_map(x), _as_map(w), b, 1, 0, relu, 0, 0, None, None, 2e-5, False, True, None,
                               None, None, None, float(drop_p), int(seed), step)[0]
        y = y.view(x.shape[0], w.shape[0])
        ctx.save_for_backward(x, w, y if (relu or drop_p > 0) else None)
        ctx.param = w if w.is_leaf else None
        ctx.relu, ctx.drop_p, ctx.has_bias = relu, drop_p, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dy = dy.contiguous()
        if y is not None:
            dy = dy * (y > 0)
            if ctx.drop_p > 0:
                dy = dy * (1.0 / (1.0 - ctx.drop_p))
        ext = need_ext()
        dx = dw = db = None
        M, K = x.shape
        N = w.shape[0]
        if ctx.needs_input_grad[0]:
            wt = cached_dgrad_weight(ctx.param)
            if wt is not None and N % 64 == 0:
                dx = ext.conv_igemm_fwd(_as_map(dy), wt, None, 1, 0, False)[0].view(M, K)
            else:
                dx = dy.mm(w)
        if ctx.needs_input_grad[1]:
            tgt = grad_sink.target(ctx.param)
            if wgrad_enabled() and N % 8 == 0:
                if tgt is not None and tgt.is_contiguous():
                    ext.conv_wgrad(_as_map(dy), _as_map(x), 1, 1, 1, 0, 0, tgt.view(N, K, 1, 1))
                else:
                    dw = ext.conv_wgrad(_as_map(dy), _as_map(x), 1, 1, 1, 0).view(N, K)
            else:
                dw = dy.t().mm(x)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.float().sum(0).to(dy.dtype)
        return dx, dw, db, None, None, None, None


def fully_connected(x, w, b=None, relu=False, drop_p=0.0, seed=0, step=None, training=False):
    """FC on (M, K) activations; ``drop_p`` applies inverted dropout after the (optional) ReLU
    when ``training``.  GPU bf16 -> the HIP kernel (dropout needs ``step``, an int64 device
    tensor); otherwise the PyTorch ops."""
    p = float(drop_p) if training else 0.0
    if fc_eligible(x, w) and (p == 0.0 or (relu and step is not None)):
        return _FC.apply(x, w, b, bool(relu), p, int(seed), step)
    y = F.linear(x, w, b)
    if relu:
        y = F.relu(y)
    if p > 0:
        y = F.dropout(y, p, True)
    return y
