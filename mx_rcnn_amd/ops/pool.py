"""Max / global-average pooling on NHWC bf16 activations (csrc/hip/pool.hip).

MXNet ``Pooling(pool_type='max', kernel, stride, pad)`` with the default "valid" (floor)
convention: VGG pool1..4 2x2/2 (`rcnn/symbol.py:19,28,40,52`), ResNet pool0 3x3/2 pad 1
(`rcnn/resnet.py:150`); ``Pooling(global_pool=True, pool_type='avg')`` before the ResNet
predictors (`rcnn/resnet.py:167`).  GPU bf16 channels_last tensors run the HIP kernels (the
backward gathers through the recorded winning taps, no atomics); anything else runs torch.
"""
import os

import torch
import torch.nn.functional as F

from . import precision
from ._ext import need_ext


def _eligible(x):
    if os.environ.get('MXR_POOL_KERNEL', '1') == '0':
        return False
    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and x.dim() == 4 and x.shape[1] % 8 == 0 and
            x.is_contiguous(memory_format=torch.channels_last))


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        ctx.x2 = x2 = precision.is_pair(x)  # fp32-class pairs (ops/precision.py)
        y, arg = need_ext().maxpool_fwd(x, k, s, p, x2)
        ctx.save_for_backward(arg)
        ctx.geo = (x.shape[2], x.shape[3], k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        arg, = ctx.saved_tensors
        H, W, k, s, p = ctx.geo
        dx = need_ext().maxpool_bwd(dy.contiguous(memory_format=torch.channels_last), arg, H, W, k, s, p, ctx.x2)
        return dx, None, None, None


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        ctx.x2 = x2 = precision.is_pair(x)
        return need_ext().avgpool_fwd(x, x2)

    @staticmethod
    def backward(ctx, dy):
        return need_ext().avgpool_bwd(dy.contiguous(), ctx.hw[0], ctx.hw[1], ctx.x2)


def max_pool2d(x, k, s, p=0):
    if _eligible(x) or precision.is_pair(x):
        return _MaxPool.apply(x, int(k), int(s), int(p))
    return F.max_pool2d(x, kernel_size=k, stride=s, padding=p)


def global_avg_pool(x):
    """(N, C, H, W) -> (N, C)."""
    if _eligible(x) or precision.is_pair(x):
        return _AvgPool.apply(x)
    return torch.mean(x, dim=(2, 3))
