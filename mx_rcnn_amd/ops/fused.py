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
import os

import torch

from . import grad_sink
from . import precision
from ._ext import need_ext
from .conv import conv_backward, pair_args


def _wargs(w):
    """(filter for the kernel, extra conv kwargs): in the fp32 (x2) mode the store's pair of the
    fp32 parameter ``w``; otherwise ``w`` itself."""
    if precision.x2_enabled():
        wh, wpl = precision.weight_pair(w)
        return wh, {'x2': precision.x2_enabled(), 'w_plane': wpl}
    return w, {}


def _rows(t):
    """Logical rows (N*H*W) of an activation (pairs: half the tensor)."""
    n = t.numel() // t.shape[1]
    return precision.logical(n)


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
                                       tg if direct else None, tb if direct else None, dres, precision.x2_enabled())
    if direct:
        return dy, None, None
    dg = dg.to(gamma.dtype) if (need_g and dg is not None) else None
    db = db.to(beta.dtype) if (need_b and db is not None) else None
    return dy, dg, db


class _ConvBnRelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, gamma, beta, mean, var, stride, pad, eps, fix_gamma):
        x = x.contiguous(memory_format=torch.channels_last)
        wk, kw = _wargs(w)
        y, a = need_ext().conv_igemm_fwd(x, wk, None, stride, pad, False, 0, 0, None, [gamma, beta, mean, var],
                                         eps, fix_gamma, True, **kw)
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
        wk, kw = _wargs(w)
        y = need_ext().conv_igemm_fwd(x, wk, None, stride, pad, False, 0, 0, res, **kw)[0]
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
        wk, kw = _wargs(w)
        y, a = need_ext().conv_igemm_fwd(x, wk, None, stride, pad, False, 0, 0, res, [gamma, beta, mean, var],
                                         eps, fix_gamma, True, **kw)
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


# ---------------------------------------------------------------------------------------------
# Whole-unit op: forward = the fused epilogues above; backward = a hand-scheduled kernel
# sequence in which every frozen BN-ReLU backward rides in the epilogue of the data-gradient
# conv that produces its input gradient (csrc/hip/conv_igemm.hip BN-backward mode):
#
#   wgrad3(a3, dOut)                      dY2 = dgrad3(dOut) o bn3'   (+ dgamma3/dbeta3)
#   wgrad2(a2, dY2)                       dY1 = dgrad2(dY2)  o bn2'   (+ dgamma2/dbeta2)
#   wgrad1(act1, dY1)  [wgrad_sc, dgrad_sc]
#   dX = dgrad1(dY1) (+ dgrad_sc) o bn1' + dOut (identity shortcut)   (+ dgamma1/dbeta1)
#
# Parameter gradients go straight into the flat gradient buffers (ops/grad_sink.py) when the
# parameters are store-managed; otherwise they are returned through autograd.  The unit's
# second output (next unit's act1, produced in conv3's epilogue) is non-differentiable: its
# gradient is handled inside the next unit, whose bn1 it is.
# ---------------------------------------------------------------------------------------------
def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


_SIDE = {}


# Cross-unit deferral of the last grouped weight-gradient reduce of each unit into the NEXT unit's
# first grouped launch.  Only inside ``defer_reduces()`` (the trainer's backward when no gradient
# hook reads the flat buffers mid-backward, i.e. no overlapped all-reduce / optimizer), which
# flushes whatever is still pending on exit.
# across-unit deferral inside one backward pass (no gradient hook reads the flat buffers mid-backward):
# 'pending' a grouped launch's split-K weight-gradient reduce, 'folds' the deterministic frozen-BN
# gamma / beta folds (run together at the end: a few launches instead of one per BN)
_XUNIT = {'on': False, 'pending': None, 'folds': []}


class defer_reduces(object):
    def __init__(self, enabled=True):
        self.enabled = enabled

    def __enter__(self):
        _XUNIT['on'] = bool(self.enabled)
        return self

    def __exit__(self, *a):
        _XUNIT['on'] = False
        flush_deferred()
        return False


def flush_deferred():
    p = _XUNIT['pending']
    if p is not None:
        need_ext().wgrad_reduce_run(*p)
        _XUNIT['pending'] = None
    if _XUNIT['folds']:
        need_ext().bnb_part_fold_multi(_XUNIT['folds'])
        _XUNIT['folds'] = []


def grouped_enabled():
    """One launch per conv for data + weight gradient in the fused units (MXR_GROUPED_BWD=0: the
    weight gradient on the side stream instead)."""
    import os
    return os.environ.get('MXR_GROUPED_BWD', '1') != '0'


def _side_stream(device):
    """Per-device side stream for the weight-gradient kernels (MXR_WGRAD_STREAM=0 disables)."""
    import os
    if os.environ.get('MXR_WGRAD_STREAM', '1') == '0':
        return None
    s = _SIDE.get(device.index)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _SIDE[device.index] = s
    return s


class _nullctx(object):
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class _Unit(object):
    """Static description of a residual unit for the fused op."""

    def __init__(self, u, next_bn, train=False):
        self.bottle = u.bottle_neck
        self.dim_match = u.dim_match
        self.stride = int((u.conv2 if u.bottle_neck else u.conv1).stride)
        self.bns = [u.bn1, u.bn2] + ([u.bn3] if u.bottle_neck else [])
        self.next_bn = next_bn
        self.eps = [float(b.eps) for b in self.bns]
        self.fix = [bool(b.fix_gamma) for b in self.bns]
        # batch-statistics BNs (the RoI head, stage 4): conv epilogues produce the statistics
        # partials, a normalisation kernel applies them; next_bn (if any) is also batch-statistics
        self.train = bool(train)
        self.mom = [float(b.momentum) for b in self.bns]


def _bnp(bn):
    return [bn.gamma, bn.beta, bn.moving_mean, bn.moving_var]


# Inference: a bottleneck's conv -> frozen BN -> ReLU is ONE conv with the BN folded in (the scale
# into a cached copy of the filter, the shift as an fp32 bias) and a ReLU epilogue, on our kernels,
# writing only the activation the next conv reads.  The training form also stores the pre-BN output
# for the backward -- dead at test time.  Round 5 routed the 1x1 reduce of batch-sized maps to
# hipBLASLt's bias / ReLU GEMM instead (test FPS 735 at batch 8); round 6 folds both the reduce and
# the 3x3 for every inference shape and runs them on the implicit-GEMM kernels (the large-M reduce on
# conv_big's 160x256 tile).  MXR_INFER_FOLD=0: the training-form epilogues (both outputs).
def _infer_fold(x, spec):
    return (spec.bottle and getattr(spec, 'infer', False) and not precision.x2_enabled() and x.is_cuda and
            x.dtype in (torch.bfloat16, torch.float16) and os.environ.get('MXR_INFER_FOLD', '1') != '0')


def _folded(w, bnp, eps, fix_gamma, dtype):
    """(filter * BN scale) in ``dtype`` (channels_last) and the BN shift as an fp32 bias, cached on
    the filter and rebuilt when the filter or the BN parameters change (version counters, reload
    epochs, the training generation: SGD rewrites trainable weights in place)."""
    gamma, beta, mean, var = bnp
    key = (w.data_ptr(), w._version, precision.weight_epoch(w), precision.train_generation(w, *bnp), dtype,
           float(eps), bool(fix_gamma)) + tuple((p.data_ptr(), p._version, precision.weight_epoch(p)) for p in bnp)
    hit = w.__dict__.get('_mxr_bn_fold')
    if hit is None or hit[0] != key:
        with torch.no_grad():
            sc = (torch.ones_like(var.float()) if fix_gamma else gamma.float()) * torch.rsqrt(var.float() + eps)
            wf = (w.detach().float() * sc[:, None, None, None]).to(dtype).contiguous(memory_format=torch.channels_last)
            bf = (beta.float() - mean.float() * sc).contiguous()
        hit = (key, wf, bf)
        w.__dict__['_mxr_bn_fold'] = hit
    return hit[1], hit[2]


class _FusedUnitFn(torch.autograd.Function):
    @staticmethod
    def _forward_train(ctx, spec, x, parts1, t, nconv, ws, bnps, nxt):
        """Batch-statistics unit: every conv's epilogue also writes the statistics partials of its
        output for the BN that consumes it (ConvEpi::st_part), so each BN is ONE normalisation pass
        (bn_train_apply); the unit's input BN uses the partials the previous unit's last conv
        produced (parts1) or a statistics pass.  Saved per BN: [mean, invstd, var+eps, 0, 0] --
        the zero rows are the backward's column-sum accumulators."""
        ext = need_ext()
        x = _cl(x)
        x2 = precision.x2_enabled()

        def norm(inp, parts, i):
            g, b, rm, rv = bnps[i]
            if parts is None:
                return ext.bn_train_fwd(inp, g, b, rm, rv, spec.mom[i], spec.eps[i], spec.fix[i], True, x2)
            return ext.bn_train_apply(inp, parts, g, b, rm, rv, spec.mom[i], spec.eps[i], spec.fix[i], True, x2)

        wa = [_wargs(w) for w in ws]
        act1, sv1 = norm(x, parts1, 0)
        s1 = 1 if spec.bottle else spec.stride
        p1 = 0 if spec.bottle else 1
        y1, pt = ext.conv_igemm_fwd(act1, wa[0][0], None, s1, p1, False, stat_shift=bnps[1][2], **wa[0][1])
        a2, sv2 = norm(y1, pt, 1)
        saves = [sv1, sv2]
        if spec.bottle:
            y2, pt = ext.conv_igemm_fwd(a2, wa[1][0], None, spec.stride, 1, False, stat_shift=bnps[2][2], **wa[1][1])
            a3, sv3 = norm(y2, pt, 2)
            saves.append(sv3)
            last_in, w_last = a3, wa[2]
        else:
            y2, a3 = None, None
            last_in, w_last = a2, wa[1]
        res = x if spec.dim_match else ext.conv_igemm_fwd(act1, wa[-1][0], None, spec.stride, 0, False,
                                                          **wa[-1][1])[0]
        pl = 0 if spec.bottle else 1
        if nxt is not None:
            out, parts_n = ext.conv_igemm_fwd(last_in, w_last[0], None, 1, pl, False, 0, 0, res,
                                              stat_shift=nxt[2].float().contiguous(), **w_last[1])
        else:
            out, parts_n = ext.conv_igemm_fwd(last_in, w_last[0], None, 1, pl, False, 0, 0, res, **w_last[1])[0], None
        ctx.spec = spec
        ctx.nconv = nconv
        ctx.set_materialize_grads(False)
        ctx.params = [p if p.is_leaf else None for p in t]
        ctx.saves = saves
        ctx.save_for_backward(x, act1, y1, a2, y2, a3, None, *t)
        if parts_n is None:
            return out, out.new_empty(0)
        ctx.mark_non_differentiable(parts_n)
        return out, parts_n

    @staticmethod
    def forward(ctx, spec, x, act1, *t):
        # t = W1, W2, [W3], [Wsc], bn1(4), bn2(4), [bn3(4)], [next_bn(4)]
        ext = need_ext()
        if spec.train:
            nconv = (3 if spec.bottle else 2) + (0 if spec.dim_match else 1)
            nb = len(spec.bns)
            bnps = [list(t[nconv + 4 * i:nconv + 4 * i + 4]) for i in range(nb)]
            nxt = list(t[nconv + 4 * nb:nconv + 4 * nb + 4]) if spec.next_bn is not None else None
            return _FusedUnitFn._forward_train(ctx, spec, x, act1, t, nconv, list(t[:nconv]), bnps, nxt)
        nconv = (3 if spec.bottle else 2) + (0 if spec.dim_match else 1)
        ws = list(t[:nconv])
        nb = len(spec.bns)
        bnps = [list(t[nconv + 4 * i:nconv + 4 * i + 4]) for i in range(nb)]
        nxt = list(t[nconv + 4 * nb:nconv + 4 * nb + 4]) if spec.next_bn is not None else None
        x = _cl(x)
        bn1 = bnps[0]
        x2 = precision.x2_enabled()
        wa = [_wargs(w) for w in ws]
        if act1 is None:
            act1 = ext.bn_relu_fwd(x, *[p.float().contiguous() for p in bn1], spec.eps[0], spec.fix[0], True, x2)
        # conv1 (stride 1 for bottleneck; 3x3 stride s for basic) -> bn2
        s1 = 1 if spec.bottle else spec.stride
        p1 = 0 if spec.bottle else 1
        fold = _infer_fold(act1, spec)
        if fold:
            # inference: reduce + bn2 + ReLU as one conv with the BN folded in; only a2 is written
            wf, bf = _folded(ws[0], bnps[1], spec.eps[1], spec.fix[1], act1.dtype)
            y1, a2 = None, ext.conv_igemm_fwd(act1, wf, bf, s1, p1, True)[0]
        else:
            y1, a2 = ext.conv_igemm_fwd(act1, wa[0][0], None, s1, p1, False, 0, 0, None, bnps[1], spec.eps[1],
                                        spec.fix[1], True, **wa[0][1])
        if spec.bottle and fold:  # the 3x3 + bn3 + ReLU the same way (its pre-BN output is dead too)
            wf, bf = _folded(ws[1], bnps[2], spec.eps[2], spec.fix[2], a2.dtype)
            y2, a3 = None, ext.conv_igemm_fwd(a2, wf, bf, spec.stride, 1, True)[0]
            last_in, w_last = a3, wa[2]
        elif spec.bottle:
            y2, a3 = ext.conv_igemm_fwd(a2, wa[1][0], None, spec.stride, 1, False, 0, 0, None, bnps[2], spec.eps[2],
                                        spec.fix[2], True, **wa[1][1])
            last_in, w_last = a3, wa[2]
        else:
            y2, a3 = None, None
            last_in, w_last = a2, wa[1]
        sc_in = None
        if spec.dim_match:
            res = x
        else:
            # strided 1x1 projection read straight from act1 by the kernel (no subsampled copy)
            res = ext.conv_igemm_fwd(act1, wa[-1][0], None, spec.stride, 0, False, **wa[-1][1])[0]
        if nxt is not None:
            out, act1n = ext.conv_igemm_fwd(last_in, w_last[0], None, 1, 0 if spec.bottle else 1, False, 0, 0, res,
                                            nxt, float(spec.next_bn.eps), bool(spec.next_bn.fix_gamma), True,
                                            **w_last[1])
        else:
            out = ext.conv_igemm_fwd(last_in, w_last[0], None, 1, 0 if spec.bottle else 1, False, 0, 0, res,
                                     **w_last[1])[0]
            act1n = None
        ctx.spec = spec
        ctx.nconv = nconv
        ctx.set_materialize_grads(False)  # the act1n output never receives a gradient
        ctx.params = [p if p.is_leaf else None for p in t]
        ctx.save_for_backward(x, act1, y1, a2, y2, a3, sc_in, *t)
        if act1n is None:
            return out, out.new_empty(0)  # placeholder output: no fill kernel
        ctx.mark_non_differentiable(act1n)
        return out, act1n

    @staticmethod
    def backward(ctx, d_out, _d_act1n):
        ext = need_ext()
        spec, nconv = ctx.spec, ctx.nconv
        saved = ctx.saved_tensors
        x, act1, y1, a2, y2, a3, sc_in = saved[:7]
        t = saved[7:]
        ws = list(t[:nconv])
        nb = len(spec.bns)
        bnps = [list(t[nconv + 4 * i:nconv + 4 * i + 4]) for i in range(nb)]
        need = ctx.needs_input_grad[3:]  # per tensor in t
        grads = [None] * len(t)
        d_out = _cl(d_out).to(x.dtype)
        # BN parameters of the BN-backward epilogues.  Batch-statistics BNs: (effective gamma, beta,
        # batch mean, var + eps) with eps 0 reproduce the forward's invstd exactly; the epilogue's
        # column sums land in the saved zero rows and bn_train_dx_apply finishes the backward
        train = spec.train
        if train:
            saves = ctx.saves
            geff = [torch.ones_like(saves[i][0]) if spec.fix[i] else bnps[i][0].float().contiguous()
                    for i in range(nb)]
            bwp = [[geff[i], bnps[i][1], saves[i][0], saves[i][2]] for i in range(nb)]
            beps, bfix = [0.0] * nb, [False] * nb
        else:
            bwp, beps, bfix = bnps, spec.eps, spec.fix

        x2 = precision.x2_enabled()
        gdt = torch.float32 if x2 else torch.bfloat16  # weight-gradient dtype of the kernels

        def train_part(bn_x, nparts):
            return torch.empty(nparts * 2 * bn_x.shape[1], device=bn_x.device, dtype=torch.float32)

        def train_finish(i, o, bn_x, dres, part, nparts):
            """o = g * s from the BN-backward epilogue -> the batch-statistics BN's dx (+ dres), in
            place; gamma / beta gradients from the epilogue's column-sum partial rows (folded in a
            fixed order: deterministic)."""
            gi = nconv + 4 * i
            ng, nbb = need[gi] and not spec.fix[i], need[gi + 1]
            tg = grad_sink.target(ctx.params[gi]) if ng else None
            tb = grad_sink.target(ctx.params[gi + 1]) if nbb else None
            own_g = ng and (tg is None or tg.dtype != torch.float32 or not tg.is_contiguous())
            own_b = nbb and (tb is None or tb.dtype != torch.float32 or not tb.is_contiguous())
            C = saves[i].shape[1]
            if own_g:
                tg = torch.zeros(C, device=o.device, dtype=torch.float32)
            if own_b:
                tb = torch.zeros(C, device=o.device, dtype=torch.float32)
            dx = ext.bn_train_dx_apply(o, bn_x, saves[i], geff[i], part, nparts, dres, tg if ng else None,
                                       tb if nbb else None, x2)
            if own_g:
                grads[gi] = tg.to(bnps[i][0].dtype)
            if own_b:
                grads[gi + 1] = tb.to(bnps[i][1].dtype)
            return dx

        # weight gradients run on a side stream, concurrently with the data-gradient chain on the
        # compute stream (each wgrad only waits for the dY it reads); joined before returning, so
        # gradient-readiness hooks (DP all-reduce) and later frees see finished writes.  Looser
        # joins measured slower on ResNet-101 (scripts/gpu_ab3.sh, 129 img/s per-unit join vs 119
        # joining once per backward with record_stream, 118 joining one unit late, 122 joining after
        # the next unit's first dgrad kernel -- with the inputs kept referenced, so not the
        # allocator): any lag of the side stream behind its unit costs more than the hand-off
        main = torch.cuda.current_stream() if x.is_cuda else None
        side = _side_stream(x.device) if main is not None else None
        used_side = [False]
        # split-K reduce of the last grouped weight gradient, run by the next grouped launch's first
        # workgroups (or flushed before returning: the gradient hooks read the flat buffer)
        pending = [_XUNIT['pending']]  # a previous unit's deferred reduce, if any
        _XUNIT['pending'] = None

        def flush_pending():
            if pending[0] is not None:
                if _XUNIT['on']:  # hand it to the next unit's first grouped launch
                    _XUNIT['pending'] = pending[0]
                else:
                    ext.wgrad_reduce_run(*pending[0])
                pending[0] = None

        def wgrad(idx, dy, inp, k, stride, pad):
            if not need[idx]:
                return
            tgt = grad_sink.target(ctx.params[idx])
            if side is not None:
                side.wait_stream(main)
                used_side[0] = True
            with torch.cuda.stream(side) if side is not None else _nullctx():
                if tgt is not None and tgt.is_contiguous(memory_format=torch.channels_last) and tgt.dtype == gdt:
                    ext.conv_wgrad(dy, inp, k, k, stride, pad, 0, tgt, x2=x2)
                else:
                    grads[idx] = ext.conv_wgrad(dy, inp, k, k, stride, pad, x2=x2)
                    if side is not None:  # allocated on the side stream, consumed on the compute stream
                        grads[idx].record_stream(main)

        def bn_targets(i):
            if train:  # column sums go to partial rows (bnb_part), gamma / beta grads via train_finish
                return None, None, False
            gi = nconv + 4 * i
            ng, nbb = need[gi] and not spec.fix[i], need[gi + 1]
            if not (ng or nbb):
                return None, None, False
            tg = grad_sink.target(ctx.params[gi]) if ng else None
            tb = grad_sink.target(ctx.params[gi + 1]) if nbb else None
            if (ng and (tg is None or tg.dtype != torch.float32)) or (nbb and (tb is None or tb.dtype != torch.float32)):
                C = bnps[i][0].numel()
                tg = torch.zeros(C, device=x.device, dtype=torch.float32)
                tb = torch.zeros(C, device=x.device, dtype=torch.float32)
                return tg, tb, True
            return tg, tb, False

        folds = []

        def fold_bn(i, part, nparts, tg, tb, now=False):
            """frozen BN(i)'s gamma / beta gradients from the epilogue's partial rows (fixed order),
            batched: run by finish_folds (this unit) or flush_deferred (end of the backward); ``now``
            when the caller reads tg / tb right away (own scratch targets, finish_bn)"""
            gi = nconv + 4 * i
            ent = (part, nparts, bnps[i][0].numel(), tg if need[gi] and not spec.fix[i] else None,
                   tb if need[gi + 1] else None)
            if now:
                ext.bnb_part_fold_multi([ent])
            else:
                folds.append(ent)

        def finish_folds():
            if not folds:
                return
            if _XUNIT['on']:
                _XUNIT['folds'].extend(folds)
            else:
                ext.bnb_part_fold_multi(folds)
            folds.clear()

        def finish_bn(i, tg, tb, returned):
            if returned:
                gi = nconv + 4 * i
                if need[gi] and not spec.fix[i]:
                    grads[gi] = tg.to(bnps[i][0].dtype)
                if need[gi + 1]:
                    grads[gi + 1] = tb.to(bnps[i][1].dtype)

        def grouped_target(wg):
            """The flat-gradient target of pending weight gradient ``wg`` = (idx, dy, inp, k, stride,
            pad) when it can ride in the grouped dgrad launch, else None."""
            if wg is None or not grouped_enabled() or not need[wg[0]] or not wg[1].is_cuda:
                return None
            tgt = grad_sink.target(ctx.params[wg[0]])
            if tgt is None or not tgt.is_contiguous(memory_format=torch.channels_last) or tgt.dtype != gdt:
                return None
            return tgt

        def dgrad_bn(dy, w_idx, k, pad, bn_i, bn_x, dadd=None, dres=None, wg=None):
            """dgrad of a stride-1 conv with the BN(bn_i)-ReLU backward of its input in the epilogue;
            with ``wg`` the weight gradient of a conv (idx, dy, inp, k, stride, pad) in the SAME launch
            (csrc/hip/conv_igemm.hip conv_dgrad_wgrad), otherwise on the side stream."""
            from .conv import dgrad_args
            tg, tb, ret = bn_targets(bn_i)
            wf, wkw = dgrad_args(ctx.params[w_idx], ws[w_idx])
            tgt = grouped_target(wg)
            part, nparts = None, 0
            det = not train and tg is not None and precision.deterministic()
            if train or det:  # per-tile partial rows, folded in a fixed order
                nparts = (_rows(bn_x) + 63) // 64
                part = train_part(bn_x, nparts)
            if tgt is not None and dy.dtype == torch.bfloat16 and wf.dtype == torch.bfloat16:
                if tg is None and not train:  # statistics not needed: accumulate into scratch
                    C = bnps[bn_i][0].numel()
                    tg = torch.zeros(C, device=dy.device, dtype=torch.float32)
                    tb = torch.zeros(C, device=dy.device, dtype=torch.float32)
                idx, wdy, winp, wk, wstride, wpad = wg
                prev = pending[0]
                r = ext.conv_dgrad_wgrad(dy, wf, k - 1 - pad, None if train else dres, bwp[bn_i], beps[bn_i],
                                         bfix[bn_i], bn_x, dadd, tg, tb, wdy, winp, wk, wk, wstride, wpad, tgt, True,
                                         prev[0] if prev else None, prev[1] if prev else None, part, **wkw)
                pending[0] = (r[3], tgt) if r[3].numel() > 0 else None
            else:
                if wg is not None:
                    wgrad(*wg)
                r = ext.conv_igemm_fwd(dy, wf, None, 1, k - 1 - pad, False, 0, 0, None if train else dres, bwp[bn_i],
                                       beps[bn_i], bfix[bn_i], True, bn_x, dadd, tg, tb, bnb_part=part, **wkw)
            if det:
                fold_bn(bn_i, part, nparts, tg, tb, ret)
            finish_bn(bn_i, tg, tb, ret)
            return train_finish(bn_i, r[0], bn_x, dres, part, nparts) if train else r[0]

        def strided_dgrad_bn(dy, w_idx, k, stride, pad, bn_i, bn_x, H, W, dadd=None, dres=None):
            """strided-conv dgrad (parity classes) with the BN(bn_i)-ReLU backward in the epilogue."""
            from .conv import dgrad_weight, strided_dgrad, strided_dgrad_parts
            tg, tb, ret = bn_targets(bn_i)
            part, nparts = None, 0
            det = not train and tg is not None and precision.deterministic()
            if train or det:
                nparts = strided_dgrad_parts(bn_x.shape[0] // (x2 if x2 else 1), H, W, stride)
                part = train_part(bn_x, nparts)
            elif tg is None:  # statistics not needed: accumulate into scratch
                C = bnps[bn_i][0].numel()
                tg = torch.zeros(C, device=dy.device, dtype=torch.float32)
                tb = torch.zeros(C, device=dy.device, dtype=torch.float32)
            r = strided_dgrad(dy, dgrad_weight(ctx.params[w_idx], ws[w_idx]), H, W, k, stride, pad,
                              residual=None if train else dres, bn=bwp[bn_i], bn_eps=beps[bn_i],
                              bn_fix_gamma=bfix[bn_i], bnb_x=bn_x, dadd=dadd, dgamma=tg, dbeta=tb,
                              param=ctx.params[w_idx], bnb_part=part)
            if det:
                fold_bn(bn_i, part, nparts, tg, tb, ret)
            finish_bn(bn_i, tg, tb, ret)
            return train_finish(bn_i, r[0], bn_x, dres, part, nparts) if train else r[0]

        def bn_bwd_plain(dy_act, bn_i, bn_x, dres=None):
            if train:  # BN-ReLU backward on the batch statistics (bn_train.hip), then the shortcut
                gi = nconv + 4 * bn_i
                ng, nbb = need[gi] and not spec.fix[bn_i], need[gi + 1]
                dx, dg, db = ext.bn_train_bwd(bn_x, dy_act, bnps[bn_i][0], bnps[bn_i][1], saves[bn_i][0],
                                              saves[bn_i][1], spec.fix[bn_i], True, True, None, None, x2)
                if ng:
                    grads[gi] = dg.to(bnps[bn_i][0].dtype)
                if nbb:
                    grads[gi + 1] = db.to(bnps[bn_i][1].dtype)
                return dx + dres if dres is not None else dx
            tg, tb, ret = bn_targets(bn_i)
            p = [q.float().contiguous() for q in bnps[bn_i]]
            dx, dg, db = ext.bn_relu_bwd(bn_x, dy_act, *p, spec.eps[bn_i], spec.fix[bn_i], True, True,
                                         tg is not None, tg, tb, dres, x2)
            finish_bn(bn_i, tg, tb, ret)
            return dx

        s = spec.stride
        # each conv's weight gradient rides in the launch of a data gradient that reads the same
        # dY (grouped), or runs on the side stream (wgrad(...)); wg0 (conv1's) is issued with the
        # unit's input gradient below
        if spec.bottle:
            # conv3 (1x1) : wgrad + dgrad with bn3 backward
            d_y2 = dgrad_bn(d_out, 2, 1, 0, 2, y2, wg=(2, d_out, a3, 1, 1, 0))
            # conv2 (3x3, stride s)
            if s == 1:
                d_y1 = dgrad_bn(d_y2, 1, 3, 1, 1, y1, wg=(1, d_y2, a2, 3, s, 1))
            elif _strided_ok(ws[1], s, a2):
                wgrad(1, d_y2, a2, 3, s, 1)
                d_y1 = strided_dgrad_bn(d_y2, 1, 3, s, 1, 1, y1, a2.shape[2], a2.shape[3])
            else:
                wgrad(1, d_y2, a2, 3, s, 1)
                d_a2 = torch.ops.aten.convolution_backward(d_y2, a2, ws[1], None, [s, s], [1, 1], [1, 1], False,
                                                           [0, 0], 1, [True, False, False])[0]
                d_y1 = bn_bwd_plain(_cl(d_a2), 1, y1)
            wg0 = (0, d_y1, act1, 1, 1, 0)
            k1, p1, s1 = 1, 0, 1
        else:
            # basic: conv2 (3x3 s1) then conv1 (3x3 stride s)
            d_y1 = dgrad_bn(d_out, 1, 3, 1, 1, y1, wg=(1, d_out, a2, 3, 1, 1))
            wg0 = (0, d_y1, act1, 3, s, 1)
            k1, p1, s1 = 3, 1, s
        # bn1 (the unit's input BN) gets its gamma / beta gradients from the d_x pass below; when
        # the unit input needs no gradient (first trainable unit after frozen stages) that pass
        # still runs if bn1's own parameters are trainable (its dx is then discarded)
        bn1_trainable = need[nconv] or need[nconv + 1]
        if not ctx.needs_input_grad[1] and not bn1_trainable:
            wgrad(*wg0)
            if not spec.dim_match:
                wgrad(nconv - 1, d_out, act1, 1, s, 0)
            flush_pending()
            if used_side[0]:
                main.wait_stream(side)
            finish_folds()
            return (None, None, None) + tuple(grads)
        d_sc = None
        if not spec.dim_match:
            wgrad(nconv - 1, d_out, act1, 1, s, 0)
            from .conv import dgrad_args
            wsc, wkw = dgrad_args(ctx.params[nconv - 1], ws[nconv - 1])
            d_sub = ext.conv_igemm_fwd(d_out, wsc, None, 1, 0, False, **wkw)[0]
            if s == 1 or (s1 == 1 and ws[0].shape[0] % 64 == 0 and
                          os.environ.get('MXR_SUB_DADD', '1') != '0'):
                # stride s > 1: the stride-1 dgrad below adds d_sub at rows (i*s, j*s) itself
                # (subsampled dadd epilogue), no zero-filled full-size scatter
                d_sc = d_sub
            else:
                d_sc = torch.zeros_like(act1, memory_format=torch.channels_last)
                d_sc[:, :, ::s, ::s] = d_sub
        dres = d_out if spec.dim_match else None
        if s1 == 1 and ws[0].shape[0] % 64 == 0:
            d_x = dgrad_bn(d_y1, 0, k1, p1, 0, x, dadd=d_sc, dres=dres, wg=wg0)
        elif s1 > 1 and _strided_ok(ws[0], s1, act1):
            wgrad(*wg0)
            d_x = strided_dgrad_bn(d_y1, 0, k1, s1, p1, 0, x, act1.shape[2], act1.shape[3], dadd=d_sc, dres=dres)
        else:
            wgrad(*wg0)
            d_act1 = torch.ops.aten.convolution_backward(d_y1, act1, ws[0], None, [s1, s1], [p1, p1], [1, 1], False,
                                                         [0, 0], 1, [True, False, False])[0]
            if d_sc is not None:
                d_act1 = d_act1 + d_sc
            d_x = bn_bwd_plain(_cl(d_act1), 0, x, dres)
        flush_pending()
        if used_side[0]:
            main.wait_stream(side)
        finish_folds()
        return (None, d_x if ctx.needs_input_grad[1] else None, None) + tuple(grads)


def _strided_ok(w, s, inp):
    from .conv import strided_dgrad_ok
    return (w.shape[0] % 64 == 0 and w.shape[1] % 8 == 0 and w.shape[2] == w.shape[3] and
            strided_dgrad_ok(w.shape[2], s, (w.shape[2] - 1) // 2, inp.shape[2], inp.shape[3]))


def fused_unit(u, x, act1=None, next_bn=None, train=False):
    """Run ResidualUnit ``u`` as one fused op -> (out, next act1 or None).  Frozen BNs: act1 /
    the second output are the unit's / next unit's bn1 activation.  train=True (batch-statistics
    BNs): they are the statistics partials of the unit input / output for its / the next bn1."""
    spec = _Unit(u, next_bn, train)
    spec.infer = not torch.is_grad_enabled()  # (inside the Function's forward grad mode is always off)
    ws = [u.conv1.weight, u.conv2.weight] + ([u.conv3.weight] if u.bottle_neck else [])
    if not u.dim_match:
        ws.append(u.sc.weight)
    t = ws + _bnp(u.bn1) + _bnp(u.bn2) + (_bnp(u.bn3) if u.bottle_neck else [])
    if next_bn is not None:
        t += [p.detach() for p in _bnp(next_bn)]  # gradients of next_bn are produced by the next unit
    out, act1n = _FusedUnitFn.apply(spec, x, act1, *t)
    return out, (act1n if next_bn is not None else None)
