"""Max / global-average pooling on NHWC bf16 activations (csrc/hip/pool.hip).

MXNet ``Pooling(pool_type='max', kernel, stride, pad)`` with the default "valid" (floor)
convention: VGG pool1..4 2x2/2 (`rcnn/symbol.py:19,28,40,52`), ResNet pool0 3x3/2 pad 1
(`rcnn/resnet.py:150`); ``Pooling(global_pool=True, pool_type='avg')`` before the ResNet
predictors (`rcnn/resnet.py:167`).  GPU bf16 channels_last tensors run the HIP kernels (the
backward gathers through the recorded winning taps, no atomics); anything else runs torch.

Inference: a pooling whose output only feeds a frozen BN + ReLU (ResNet pool0 -> stage1_unit1_bn1,
RoI pooling -> stage4_unit1_bn1: pre-activation projection units read nothing but bn1's output)
writes relu(bn(pool)) straight from the pooling kernel -- no separate BN pass over the map, and no
tap / argmax map (``max_pool_bn_relu``, ops/roi_pool.py ``roi_pool_bn_relu``).
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


def post_bn_ok(bn):
    """The frozen BN + ReLU ``bn`` may be applied in a pooling kernel's store: no gradient is being
    recorded, BN uses its moving statistics (not calibrating them), ReLU follows."""
    if os.environ.get('MXR_POOL_POST_BN', '1') == '0' or torch.is_grad_enabled():
        return False
    return bool(bn.relu) and (bn.use_global_stats or not bn.training) and not getattr(bn, '_calibrate', False)


def kernel_path(x):
    """x takes the HIP pooling kernels (16-bit channels_last or fp32-class planes)."""
    return _eligible(x) or bool(precision.is_pair(x))


def post_bn_params(bn):
    """-> the (2, C) fp32 [scale; shift] of frozen ``bn`` for the pooling kernels (ext.bn_affine: the
    arithmetic of bn_relu_fwd, so the fused output is the same bits), cached on the module and
    rebuilt when a parameter / statistic moves (version counters, reload epochs, the training
    generation: SGD and the batch-statistics kernels update in place)."""
    prm = [bn.gamma, bn.beta, bn.moving_mean, bn.moving_var]
    key = (float(bn.eps), bool(bn.fix_gamma), precision.train_generation(*prm)) + tuple(
        (t.data_ptr(), t._version, precision.weight_epoch(t)) for t in prm)
    hit = bn.__dict__.get('_mxr_post_bn')
    if hit is None or hit[0] != key:
        with torch.no_grad():
            aff = need_ext().bn_affine(*[t.detach().float().contiguous() for t in prm], float(bn.eps),
                                       bool(bn.fix_gamma))
        hit = (key, aff)
        bn.__dict__['_mxr_post_bn'] = hit
    return hit[1]


def max_pool_bn_relu(x, k, s, p, bn):
    """relu(bn(max_pool(x))) for a frozen ``bn``: one kernel on the HIP path (post_bn_ok), else the
    two ops."""
    if post_bn_ok(bn) and kernel_path(x):
        return need_ext().maxpool_fwd(x, int(k), int(s), int(p), precision.is_pair(x), False, post_bn_params(bn))[0]
    return bn(max_pool2d(x, k, s, p))


def max_pool2d(x, k, s, p=0):
    if _eligible(x) or precision.is_pair(x):
        return _MaxPool.apply(x, int(k), int(s), int(p))
    return F.max_pool2d(x, kernel_size=k, stride=s, padding=p)


def global_avg_pool(x):
    """(N, C, H, W) -> (N, C)."""
    if _eligible(x) or precision.is_pair(x):
        return _AvgPool.apply(x)
    return torch.mean(x, dim=(2, 3))
