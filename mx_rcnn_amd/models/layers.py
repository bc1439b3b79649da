"""Building blocks with MXNet parameter names.

Every layer knows its MXNet name (``mx_name``) so ``arg_params()`` / ``aux_params()``
reproduce the reference's ``.params`` keys (`conv1_1_weight`, `stage3_unit2_bn1_gamma`,
`bn1_moving_mean`, ...).  Activations are NCHW-logical tensors in channels_last memory on
the GPU (the native layout of the HIP kernels); weights are cast to the activation dtype
only when they differ (mixed precision installs bf16 weight views, see
:mod:`mx_rcnn_amd.core.params`).
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.bn import frozen_bn_relu, train_bn_eligible, train_bn_relu
from ..ops.conv import conv2d
from ..ops.fc import fully_connected, layer_seed
from ..ops.pool import max_pool2d


class MxLayer(nn.Module):
    """Base: maps torch parameter names to MXNet argument/aux names."""
    mx_name = ''

    def mx_args(self):
        return {'%s_%s' % (self.mx_name, k): v for k, v in self._parameters.items() if v is not None}

    def mx_aux(self):
        return {}

    def mx_arg_shapes(self):
        """MXNet shapes of the arguments (checkpoint / converter layout; a parameter may be held in
        another logical shape of the same elements, e.g. Linear(in_shape=...))."""
        return {k: tuple(v.shape) for k, v in self.mx_args().items()}


def _w(t, ref):
    from ..ops import precision
    if precision.x2_enabled():  # the fp32 parameter: the ops take its pair from the store
        return t
    return t if t.dtype == ref.dtype else t.to(ref.dtype)


class Conv(MxLayer):
    def __init__(self, name, cin, cout, k, stride=1, pad=0, bias=True):
        super().__init__()
        self.mx_name = name
        self.stride, self.pad = stride, pad
        self.weight = nn.Parameter(torch.empty(cout, cin, k, k))
        self.bias = nn.Parameter(torch.zeros(cout)) if bias else None
        nn.init.normal_(self.weight, 0, 0.01)

    def forward(self, x, relu=False):
        b = None if self.bias is None else _w(self.bias, x)
        return conv2d(x, _w(self.weight, x), b, self.stride, self.pad, relu)


class Linear(MxLayer):
    """MXNet FullyConnected: flattens all but dim 0, y = x W^T + b; optionally fused with the
    following ReLU and Dropout (ops/fc.py).  ``rng_step`` (an int64 device tensor set by the
    Trainer and advanced every update) drives the counter-based dropout mask."""

    def __init__(self, name, cin, cout, bias=True, in_shape=None):
        super().__init__()
        self.mx_name = name
        # in_shape (C, H, W): the layer flattens a (C, H, W) map (VGG fc6 on the 7x7 pooled RoIs).
        # Its weight is then held as the (cout, C, H, W) filter of the same elements -- stored
        # channels_last by the parameter store, i.e. in (h, w, c) column order, which is the order of
        # the pooled map's channels_last rows: the GEMM reads both as plain row-major matrices with no
        # flatten copy of the activations or their gradient (checkpoints keep (cout, cin))
        self.in_shape = tuple(in_shape) if in_shape is not None else None
        if self.in_shape is not None:
            assert cin == self.in_shape[0] * self.in_shape[1] * self.in_shape[2]
            self.weight = nn.Parameter(torch.empty(cout, *self.in_shape))
        else:
            self.weight = nn.Parameter(torch.empty(cout, cin))
        self.cin, self.cout = cin, cout
        self.bias = nn.Parameter(torch.zeros(cout)) if bias else None
        nn.init.normal_(self.weight, 0, 0.01)
        self.rng_step = None
        self._seed = None

    def mx_arg_shapes(self):
        out = super().mx_arg_shapes()
        out['%s_weight' % self.mx_name] = (self.cout, self.cin)
        return out

    def forward(self, x, relu=False, drop_p=0.0):
        if self.in_shape is not None:
            # (h, w, c) columns on both sides: the channels_last filter's rows are a free view, and
            # the activation (MXNet Flatten (c, h, w) rows, or the map itself) is the one permuted
            # -- a copy of R x 25088 activations, never of the 100M-element weight
            if x.dim() != 4:
                x = x.reshape(x.shape[0], *self.in_shape)
            x = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)
        else:
            x = x.reshape(x.shape[0], -1)
        b = None if self.bias is None else _w(self.bias, x)
        if drop_p and self.training and self._seed is None:
            self._seed = layer_seed(self.mx_name)
        w = _w(self.weight, x)
        if w.dim() != 2:
            w = w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
        return fully_connected(x, w, b, relu, drop_p, self._seed or 0, self.rng_step, self.training)


class BatchNorm(MxLayer):
    """MXNet BatchNorm (eps 2e-5) optionally fused with the following ReLU.

    ``use_global_stats=True`` (ResNet stages 1-3): frozen statistics, HIP fused BN+ReLU kernel,
    gamma/beta still trainable unless frozen by prefix.  ``False`` (stage 4 / bn1, SURVEY
    §2.6): batch statistics over the RoI batch, moving averages with MXNet momentum.
    """

    def __init__(self, name, c, eps=2e-5, momentum=0.9, fix_gamma=False, use_global_stats=True, relu=True):
        super().__init__()
        self.mx_name = name
        self.eps, self.momentum, self.fix_gamma = eps, momentum, fix_gamma
        self.use_global_stats, self.relu = use_global_stats, relu
        self.gamma = nn.Parameter(torch.ones(c))
        self.beta = nn.Parameter(torch.zeros(c))
        self.register_buffer('moving_mean', torch.zeros(c))
        self.register_buffer('moving_var', torch.ones(c))

    def mx_aux(self):
        return {'%s_moving_mean' % self.mx_name: self.moving_mean, '%s_moving_var' % self.mx_name: self.moving_var}

    def forward(self, x, parts=None):
        """parts: statistics partials of x produced by its conv's epilogue (train mode only)."""
        if getattr(self, '_calibrate', False):
            # data-dependent init: moving stats := statistics of this batch (stand-in for the
            # ImageNet statistics a pretrained checkpoint carries)
            xf = x.float()
            with torch.no_grad():
                self.moving_mean.copy_(xf.mean(dim=(0, 2, 3)))
                self.moving_var.copy_(xf.var(dim=(0, 2, 3), unbiased=False))
            g = torch.ones_like(self.gamma) if self.fix_gamma else self.gamma
            y = F.batch_norm(xf, self.moving_mean, self.moving_var, g.float(), self.beta.float(), training=False,
                             eps=self.eps).to(x.dtype)
            return F.relu(y) if self.relu else y
        if self.use_global_stats or not self.training:
            return frozen_bn_relu(x, self.gamma, self.beta, self.moving_mean, self.moving_var, self.eps,
                                  self.fix_gamma, self.relu)
        if train_bn_eligible(x) and os.environ.get('MXR_BN_TRAIN_KERNEL', '1') != '0':
            return train_bn_relu(x, self.gamma, self.beta, self.moving_mean, self.moving_var, self.momentum,
                                 self.eps, self.fix_gamma, self.relu, parts=parts)
        g = torch.ones_like(self.gamma) if self.fix_gamma else self.gamma
        # torch running = (1-m)*running + m*batch  <=>  MXNet moving = mom*moving + (1-mom)*batch
        y = F.batch_norm(x, self.moving_mean, self.moving_var, g.to(x.dtype) if x.dtype != torch.float32 else g,
                         self.beta.to(x.dtype) if x.dtype != torch.float32 else self.beta, training=True,
                         momentum=1.0 - self.momentum, eps=self.eps)
        return F.relu(y) if self.relu else y


def max_pool(x, k, s, p=0):
    return max_pool2d(x, k, s, p)
