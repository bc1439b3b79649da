"""Convolution dispatch for channels_last bf16 activations on MI355X.

* k x k, Cin % 64 == 0: hand-written MFMA implicit-GEMM forward (csrc/hip/conv_igemm.hip),
  fused bias + ReLU epilogue.  Backward: the stride-1 data gradient is the same kernel run
  on dY with the flipped/transposed filter (pad' = k-1-pad); the weight gradient is the MFMA
  wgrad kernel (csrc/hip/conv_wgrad.hip, transposed LDS reads); strided dgrad still uses
  ``aten.convolution_backward`` (MIOpen).  ``MXR_CONV_WGRAD=0`` restores MIOpen wgrad.
* 1x1: one GEMM over the NHWC matrix view (layers.conv1x1_nhwc).
* Anything else (the 3-channel stem convs): MIOpen.

``MXR_CONV_IGEMM=0`` disables the custom kernel (A/B switch for profiling).
"""
import os

import torch
import torch.nn.functional as F

from ._ext import need_ext


def igemm_enabled():
    return os.environ.get('MXR_CONV_IGEMM', '1') != '0'


def wgrad_enabled():
    return os.environ.get('MXR_CONV_WGRAD', '1') != '0'


def _flip_t(w):
    """(O, I, kh, kw) -> (I, O, kh, kw) spatially flipped, channels_last memory."""
    return w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)


class _ConvIgemm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, relu):
        ext = need_ext()
        x = x.contiguous(memory_format=torch.channels_last)
        wc = w.contiguous(memory_format=torch.channels_last)
        y = ext.conv_igemm_fwd(x, wc, b, stride, pad, relu)
        ctx.save_for_backward(x, wc, y if relu else None)
        ctx.stride, ctx.pad, ctx.relu, ctx.has_bias = stride, pad, relu, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        if ctx.relu:
            dy = dy * (y > 0)
        kh = w.shape[2]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if ctx.stride == 1 and w.shape[0] % 64 == 0 and 2 * ctx.pad == kh - 1:
                dx = need_ext().conv_igemm_fwd(dy, _flip_t(w), None, 1, kh - 1 - ctx.pad, False)
            else:
                dx = torch.ops.aten.convolution_backward(
                    dy, x, w, None, [ctx.stride] * 2, [ctx.pad] * 2, [1, 1], False, [0, 0], 1,
                    [True, False, False])[0]
        need_w = ctx.needs_input_grad[1]
        need_b = ctx.has_bias and ctx.needs_input_grad[2]
        if need_w and wgrad_enabled() and w.shape[0] % 8 == 0:
            dw = need_ext().conv_wgrad(dy, x, w.shape[2], w.shape[3], ctx.stride, ctx.pad)
            if need_b:
                db = dy.sum(dim=(0, 2, 3)).to(w.dtype)
        elif need_w or need_b:
            _, dw, db = torch.ops.aten.convolution_backward(
                dy, x, w, [w.shape[0]] if ctx.has_bias else None, [ctx.stride] * 2, [ctx.pad] * 2, [1, 1], False,
                [0, 0], 1, [False, bool(ctx.needs_input_grad[1]), bool(ctx.has_bias and ctx.needs_input_grad[2])])
        return dx, dw, db, None, None, None


def conv2d(x, w, b=None, stride=1, pad=0, relu=False):
    """Conv (+bias, +optional fused ReLU) on NCHW-logical / channels_last tensors."""
    if (x.is_cuda and igemm_enabled() and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and
            x.shape[1] % 64 == 0 and w.shape[2] > 1):
        return _ConvIgemm.apply(x, w, b, int(stride), int(pad), bool(relu))
    y = F.conv2d(x, w, b, stride=stride, padding=pad)
    return F.relu(y, inplace=True) if relu else y
