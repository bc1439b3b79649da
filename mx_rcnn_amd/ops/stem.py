"""Fused stem convolution: the trunk's 3-channel first layer in one HIP launch (csrc/hip/stem.hip).

ResNet (`rcnn/resnet.py:146-150`): bn_data (frozen, fix_gamma) -> conv0 7x7/2 pad 3 -> bn0
(frozen) -> relu.  VGG16 (`rcnn/symbol.py:11-13`): conv1_1 3x3/1 pad 1 + bias -> relu.  The
unfused path is three launches (input BN, a vendor conv -- the MFMA implicit-GEMM kernels need
64-channel K blocks -- and BN+ReLU) with two full-resolution round trips through HBM.

Forward-only: used when nothing upstream of the stem output needs a gradient (the reference
freezes conv0 / bn_data / bn0 and conv1_x: FIXED_PARAMS, `rcnn/config.py`), i.e. in training with
those parameters fixed and at test time.  The kernel folds the BN affines from the BN
parameters / moving statistics in-kernel (no derived copy to invalidate: the graph warm-up's
state restore rewrites those buffers), and reads the filter from a packed (64, KP) copy cached
on the parameter itself and rebuilt when its version counter or reload epoch moves.  A
captured step contains the conv launch only.
"""
import os

import torch
import torch.nn.functional as F

from . import precision
from ._ext import need_ext


def _packed_filter(w, dtype):
    """dtype torch.float32 (the multi-plane modes): the packed filter's bf16 planes in the kernel's
    LOGICAL order -- (128, KP) = (hi, lo) for bf16x3, (192, KP) = (hi, mid, lo) for fp32.

    The packing lives ON the weight tensor (``w._mxr_stem``), so it dies with the parameter and can
    never be served to a later tensor that reuses the same ``id`` / address (the round-4 stale-filter
    bug of an ``id()``-keyed cache).  It is rebuilt when the tensor's version counter, storage or
    reload epoch (``precision.forget_weight``: ``.data`` writes do not move the version counter)
    changes -- IN PLACE when the shape allows, so a captured hipGraph keeps reading live values --
    and, for a trainable filter, when a training step ran since (``precision.train_generation``)."""
    planes = precision.nplanes() if dtype == torch.float32 else 0
    slot = (dtype, planes)
    ver = (w.data_ptr(), w._version, tuple(w.shape), precision.weight_epoch(w), precision.train_generation(w))
    cache = w.__dict__.get('_mxr_stem')
    if cache is None:
        cache = w.__dict__['_mxr_stem'] = {}
    hit = cache.get(slot)
    if hit is None or hit[0] != ver:
        if dtype == torch.float32:
            pf = precision.split(pack_filter(w, torch.float32), planes or 2)
            if planes == 3:  # memory order (mid, hi, lo) -> logical (hi, mid, lo)
                pf = torch.cat([pf[64:128], pf[:64], pf[128:]], 0).contiguous()
        else:
            pf = pack_filter(w, dtype)
        if hit is not None and hit[1].shape == pf.shape:
            hit[1].copy_(pf)
            pf = hit[1]
        hit = (ver, pf)
        cache[slot] = hit
    return hit[1]


def stem_fusable(x, *params):
    """True when the fused stem kernel can replace the unfused layers for input ``x``."""
    if os.environ.get('MXR_STEM', '1') == '0':
        return False
    ok_dtype = (torch.float32,) if precision.x2_enabled() else (torch.bfloat16, torch.float16)
    if not (x.is_cuda and x.dtype in ok_dtype and x.dim() == 4 and x.shape[1] == 3):
        return False
    if torch.is_grad_enabled() and (x.requires_grad or any(p is not None and p.requires_grad for p in params)):
        return False
    return True


def pack_filter(w, dtype):
    """(64, 3, KH, KW) filter -> contiguous (64, KP) in ``dtype``, k = (fr*KW + fc)*3 + c,
    zero-padded to a multiple of 32 (the MFMA K step): the kernel's B operand."""
    co, ci, kh, kw = w.shape
    k = kh * kw * ci
    kp = (k + 31) // 32 * 32
    wp = w.detach().to(dtype).permute(0, 2, 3, 1).reshape(co, k)
    return F.pad(wp, (0, kp - k)).contiguous()


def bn_affine(bn):
    """Frozen BatchNorm as y = x*scale + shift (fp32), MXNet fix_gamma semantics."""
    g = torch.ones_like(bn.gamma, dtype=torch.float32) if bn.fix_gamma else bn.gamma.detach().float()
    scale = g * torch.rsqrt(bn.moving_var.float() + bn.eps)
    shift = bn.beta.detach().float() - bn.moving_mean.float() * scale
    return scale.contiguous(), shift.contiguous()


def _bn_args(bn):
    if bn is None:
        return [], 0.0, False
    ts = [bn.gamma.detach(), bn.beta.detach(), bn.moving_mean, bn.moving_var]
    ts = [t if (t.dtype == torch.float32 and t.is_contiguous()) else t.float().contiguous() for t in ts]
    return ts, float(bn.eps), bool(bn.fix_gamma)


def stem_conv(x, weight, stride, pad, in_bn=None, out_bn=None, bias=None, relu=True):
    """relu?(conv(in_bn(x), weight) -> out_bn or + bias), x (N,3,H,W) channels_last 16-bit (or the fp32
    image in the fp32-class mode, whose output is a (2N, 64, Ho, Wo) pair)."""
    co, ci, kh, kw = weight.shape
    assert co == 64 and ci == 3, 'stem_conv: 3 -> 64 channels'
    wp = _packed_filter(weight, x.dtype)
    ib, ieps, ifix = _bn_args(in_bn)
    ob, oeps, ofix = _bn_args(out_bn)
    b = bias.detach() if (bias is not None and out_bn is None) else None
    xc = x.contiguous(memory_format=torch.channels_last)
    return need_ext().stem_conv(xc, wp, ib, ieps, ifix, ob, oeps, ofix, b, kh, kw, int(stride), int(pad), bool(relu))


def stem_conv_reference(x, weight, stride, pad, in_bn=None, out_bn=None, bias=None, relu=True):
    """fp32 PyTorch oracle of stem_conv (same rounding points: the normalised input is stored in
    the activation dtype before the conv, as the unfused path does)."""
    xf = x.float()
    if in_bn is not None:
        s, t = bn_affine(in_bn)
        xf = (xf * s.view(1, -1, 1, 1) + t.view(1, -1, 1, 1)).to(x.dtype).float()
    y = F.conv2d(xf, weight.detach().to(x.dtype).float(), None, stride=stride, padding=pad)
    if out_bn is not None:
        s, t = bn_affine(out_bn)
        y = y * s.view(1, -1, 1, 1) + t.view(1, -1, 1, 1)
    elif bias is not None:
        y = y + bias.detach().float().view(1, -1, 1, 1)
    return torch.relu(y) if relu else y
