"""RoI max pooling (MXNet `ROIPooling` as called at `rcnn/symbol.py:356`,
`rcnn/resnet.py:111`) as an autograd op.  GPU: HIP NHWC kernels (csrc/hip/roi_pool.hip);
the feature map is used in channels_last memory format, which is the framework's native
activation layout.  CPU: reference loops (test oracle)."""
import math

import numpy as np
import torch

from . import precision
from ._ext import ext_available, need_ext


def _bins(roi, PH, PW, H, W, scale):
    """Bin edges with MXNet's float32 arithmetic (static_cast<float>(ph) * bin_size)."""
    f = np.float32
    sc = f(scale)
    x1 = int(_round(float(f(roi[1]) * sc))); y1 = int(_round(float(f(roi[2]) * sc)))
    x2 = int(_round(float(f(roi[3]) * sc))); y2 = int(_round(float(f(roi[4]) * sc)))
    rw = max(x2 - x1 + 1, 1); rh = max(y2 - y1 + 1, 1)
    bh = f(rh) / f(PH); bw = f(rw) / f(PW)
    for ph in range(PH):
        hs = min(max(int(math.floor(f(ph) * bh)) + y1, 0), H)
        he = min(max(int(math.ceil(f(ph + 1) * bh)) + y1, 0), H)
        for pw in range(PW):
            ws = min(max(int(math.floor(f(pw) * bw)) + x1, 0), W)
            we = min(max(int(math.ceil(f(pw + 1) * bw)) + x1, 0), W)
            yield ph, pw, hs, he, ws, we


def _round(v):
    # C roundf: half away from zero
    return math.floor(v + 0.5) if v >= 0 else -math.floor(-v + 0.5)


def roi_pool_ref(feat, rois, PH, PW, scale):
    """fp32 reference: returns (out (R, C, PH, PW), argmax (R, C, PH, PW) of h*W + w or -1)."""
    B, C, H, W = feat.shape
    R = rois.shape[0]
    out = torch.zeros(R, C, PH, PW, dtype=torch.float32)
    arg = torch.full((R, C, PH, PW), -1, dtype=torch.int32)
    f = feat.float()
    for r in range(R):
        b = int(rois[r, 0])
        if b < 0 or b >= B:
            continue
        for ph, pw, hs, he, ws, we in _bins(rois[r], PH, PW, H, W, scale):
            if he <= hs or we <= ws:
                continue
            reg = f[b, :, hs:he, ws:we].reshape(C, -1)
            mx, am = reg.max(dim=1)
            # first max in row-major order
            am = (reg == mx[:, None]).float().argmax(dim=1)
            out[r, :, ph, pw] = mx
            hh = hs + am // (we - ws)
            ww = ws + am % (we - ws)
            arg[r, :, ph, pw] = (hh * W + ww).to(torch.int32)
    return out.to(feat.dtype), arg


class _RoIPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feat, rois, PH, PW, scale, grad_add=None):
        B, C, H, W = feat.shape
        ctx.grad_add = grad_add
        rois = rois.float().contiguous()
        ctx.x2 = x2 = precision.is_pair(feat)
        if x2:
            B = B // x2  # (P*B, C, H, W) planes
        if feat.is_cuda:
            ext = need_ext()
            # the argmax map only feeds the backward: inference (no grad) skips writing it
            out, arg = ext.roi_pool_fwd(feat.contiguous(memory_format=torch.channels_last), rois, PH, PW, float(scale),
                                        x2, bool(ctx.needs_input_grad[0]))
        else:
            if ext_available():  # C++ twin (the loop reference below is the test oracle)
                out, arg = need_ext().roi_pool_fwd_cpu(feat, rois, PH, PW, float(scale))
                out = out.to(feat.dtype)
            else:
                out, arg = roi_pool_ref(feat, rois, PH, PW, scale)
        ctx.save_for_backward(arg, rois)
        ctx.shape = (B, C, H, W)
        return out

    @staticmethod
    def backward(ctx, gout):
        arg, rois = ctx.saved_tensors
        B, C, H, W = ctx.shape
        ga = ctx.grad_add
        if gout.is_cuda:
            ext = need_ext()
            if ga is not None:
                ga = ga.to(gout.dtype).contiguous(memory_format=torch.channels_last)
            gin = ext.roi_pool_bwd(gout.contiguous(memory_format=torch.channels_last), arg, rois, B, H, W, ga, ctx.x2)
            ga = None  # added in the kernel
        elif ext_available():  # C++ twin: channel-parallel scatter, deterministic sum order
            gin = need_ext().roi_pool_bwd_cpu(gout, arg, rois, B, H, W).to(gout.dtype)
        else:
            gin = torch.zeros(B, C * H * W, dtype=torch.float32)
            R = gout.shape[0]
            g = gout.float().reshape(R, C, -1)
            a = arg.reshape(R, C, -1).long()
            for r in range(R):
                b = int(rois[r, 0])
                if b < 0 or b >= B:
                    continue
                m = a[r] >= 0
                flat = (torch.arange(C)[:, None] * H * W + a[r].clamp_min(0))[m]
                gin[b].index_add_(0, flat, g[r][m])
            gin = gin.reshape(B, C, H, W).to(gout.dtype)
        if ga is not None:
            gin = gin + ga.to(gin.dtype)
        ctx.grad_add = None
        return gin, None, None, None, None, None


def roi_pool(feat, rois, pooled_size=(7, 7), spatial_scale=0.0625, grad_add=None):
    """feat (B, C, H, W), rois (R, 5) -> (R, C, PH, PW) (channels_last on GPU).  grad_add: a
    gradient of ``feat`` from elsewhere (B, C, H, W), added to the pooling's input gradient in
    the backward kernel -- the early RPN-head backward's (models/faster_rcnn.py)."""
    return _RoIPool.apply(feat, rois, int(pooled_size[0]), int(pooled_size[1]), float(spatial_scale), grad_add)


def roi_pool_bn_relu(feat, rois, pooled_size, spatial_scale, bn):
    """relu(bn(roi_pool(feat, rois))) for a frozen ``bn`` (inference: stage4_unit1_bn1 of the ResNet
    head): the BN + ReLU in the pooling kernel's store, no argmax map (ops/pool.py post_bn_ok)."""
    from .pool import post_bn_ok, post_bn_params
    if feat.is_cuda and post_bn_ok(bn):
        return need_ext().roi_pool_fwd(feat.contiguous(memory_format=torch.channels_last), rois.float().contiguous(),
                                       int(pooled_size[0]), int(pooled_size[1]), float(spatial_scale),
                                       precision.is_pair(feat), False, post_bn_params(bn))[0]
    return bn(roi_pool(feat, rois, pooled_size, spatial_scale))
