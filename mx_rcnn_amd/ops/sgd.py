"""Fused SGD-momentum over flat buffers (MXNet SGD with clip_gradient,
rescale_grad and weight decay, `train_end2end.py:98-105`)."""
import torch

from ._ext import ext_available, need_ext


def sgd_momentum_(w, mom, grad, lr, momentum=0.9, wd=0.0, rescale=1.0, clip=-1.0, w_bf16=None, planes=1, zero=None,
                  plane_stride=0):
    """In-place update of flat fp32 ``w``/``mom`` from ``grad`` (fp32 or bf16).

    ``lr`` is a 1-element fp32 device tensor (read in-kernel: graph-replay safe).
    ``w_bf16`` (optional) receives the bf16 copy of the updated weights, or with ``planes`` 2 / 3
    their bf16x3 pair / fp32 triple (ops/precision.py), planes ``w_bf16.numel() // planes`` apart.
    ``zero`` (optional, fp32 or bf16, w's size; may be ``grad`` itself): cleared after it is read,
    so the next step's gradient writers start from zero without a separate fill.
    ``plane_stride`` (GPU): ``w_bf16`` is a view into a store's shadow whose planes sit
    ``plane_stride`` elements apart (a bucket slice of a multi-plane group).
    """
    if w.is_cuda:
        need_ext().sgd_momentum(w, mom, grad, lr, float(momentum), float(wd), float(rescale), float(clip), w_bf16,
                                int(planes), zero, int(plane_stride))
        return
    assert not plane_stride, 'plane_stride: GPU only'
    try:
        _sgd_host(w, mom, grad, lr, momentum, wd, rescale, clip, w_bf16, planes)
    finally:
        if zero is not None:
            zero.zero_()


def _sgd_host(w, mom, grad, lr, momentum, wd, rescale, clip, w_bf16, planes):
    if ext_available() and w.dtype == torch.float32 and w.is_contiguous() and mom.is_contiguous():
        # C++ twin (host_ops.h): one fused, thread-parallel pass instead of five tensor ops
        need_ext().sgd_momentum_cpu(w, mom, grad, float(lr), float(momentum), float(wd), float(rescale), float(clip))
        if w_bf16 is not None:
            _write_shadow(w_bf16, w, planes)
        return
    g = grad.float() * rescale
    if clip > 0:
        g = g.clamp(-clip, clip)
    mom.mul_(momentum).sub_(lr.float() * (g + wd * w))
    w.add_(mom)
    if w_bf16 is not None:
        _write_shadow(w_bf16, w, planes)


def _write_shadow(w_bf16, w, planes):
    if planes <= 1:
        w_bf16.copy_(w.to(torch.bfloat16))
        return
    from . import precision
    parts, n, pl = precision.split(w, planes), w.numel(), w_bf16.numel() // planes
    for k in range(planes):
        w_bf16[k * pl:k * pl + n].copy_(parts[k * n:(k + 1) * n])
