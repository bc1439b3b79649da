"""VGG16 trunk and Fast R-CNN head as two fused autograd functions (reference `rcnn/symbol.py:6-119`).

Per-layer autograd would run every ReLU backward as its own pass (``dy * (y > 0)``) and read a
transposed copy of each filter.  Here the backward of the whole trunk / head is one explicit
sequence in which

* a ReLU (+ inverted dropout) backward rides in the epilogue of the data gradient that produces
  its input gradient: the input of conv / FC layer L is the ReLU output of layer L-1 (or a max-pool
  of it, where ``pool_out > 0`` exactly when the winning tap is positive), so the data gradient of
  L, masked by its own forward input (ConvEpi::rmask), IS the pre-activation gradient of L-1;
* the data gradient reads the forward filter transposed in-kernel (ConvEpi::bt), no flipped copy;
* data and weight gradient of a layer share one grouped launch (both read the same dY);
* weight / bias gradients go straight into the flat gradient buffers (ops/grad_sink.py).

Only the trunk's top gradient (the sum of the RPN head's and the RoI pooling's contributions) is
masked by a separate small kernel (relu_mask_bwd).  fp32-class pairs (ops/precision.py) run
through the same sequence.
"""
import torch

from . import grad_sink
from . import precision
from ._ext import need_ext
from .head import _pair_backward, pair_eligible


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _rows(t, shape4):
    """A channels_last (O, C, H, W) filter (fc6 held as Linear(in_shape=...)) read as the 1x1
    filter ``shape4`` = (O, C*H*W, 1, 1) of its (h, w, c)-ordered rows: a free view."""
    if t.dim() == 4 and tuple(t.shape) != tuple(shape4) and shape4[2] == 1 and shape4[3] == 1:
        return t.permute(0, 2, 3, 1).reshape(shape4)
    return t.reshape(shape4)


def _wargs(w, shape4=None):
    """(filter as a channels_last (O, I, kh, kw) map, kwargs) of a launch reading weight ``w``
    (an FC's (O, I) weight as a 1x1 filter); x2: the store's pair of the fp32 parameter."""
    shape4 = tuple(w.shape) if shape4 is None else shape4
    if precision.x2_enabled():
        wh, wpl = precision.weight_pair(w)
        return _rows(wh, shape4), {'x2': precision.x2_enabled(), 'w_plane': wpl}
    return _cl(_rows(w, shape4)), {}


def _kdim(w, k=1):
    """Input channels of weight ``w`` as a k x k filter (an (O, C, H, W) fc6 filter: C*H*W)."""
    return w[0].numel() // (k * k) if (k == 1 and w.dim() == 4) else w.shape[1]


def _gdt():
    return torch.float32 if precision.x2_enabled() else torch.bfloat16


def _wtarget(param, shape4):
    """The flat-buffer gradient view of ``param`` as the channels_last (O, I, kh, kw) map the
    wgrad kernels accumulate into, or None."""
    tgt = grad_sink.target(param)
    if tgt is None or tgt.dtype != _gdt():
        return None
    if tgt.dim() == 2:
        return tgt.view(shape4) if tgt.is_contiguous() else None
    if not tgt.is_contiguous(memory_format=torch.channels_last):
        return None
    return _rows(tgt, shape4)


def _bias_grad(d, bparam, x2):
    """Per-channel sum of d into the bias's flat gradient view (None returned) or a new tensor."""
    ext = need_ext()
    tb = grad_sink.target(bparam)
    if tb is not None and tb.is_contiguous():
        ext.chan_sum(d, tb, True, x2)
        return None
    db = torch.empty(d.shape[1], dtype=torch.float32, device=d.device)
    ext.chan_sum(d, db, False, x2)
    return db.to(bparam.dtype) if bparam is not None else db


def _layer_backward(d, x, w, wparam, need_w, need_x, k, pad, rmask=None, rmask_scale=1.0):
    """Weight gradient (into the flat buffer when possible) and, with ``need_x``, the data gradient
    of a stride-1 layer given its pre-activation gradient ``d`` (channels_last maps; FCs as 1x1
    maps).  ``rmask``: the ReLU / dropout output feeding this layer (its forward input), whose
    backward the data gradient's epilogue applies.  -> (dx or None, dw or None)."""
    ext = need_ext()
    x2 = precision.x2_enabled()
    shape4 = (w.shape[0], _kdim(w, k), k, k)
    wk, kw = _wargs(w, shape4)
    kw = dict(kw, bt=True)
    dx = dw = None
    spec = grad_sink.fused_sgd(wparam) if need_w else None
    if spec is not None:
        # the parameter's SGD step rides in its weight gradient (core/params.py enable_fused_sgd):
        # data gradient first (it reads the current filter), then the update; the gradient itself
        # is never stored
        if need_x:
            dx = ext.conv_igemm_fwd(d, wk, None, 1, k - 1 - pad, False, rmask=rmask, rmask_scale=rmask_scale,
                                    **kw)[0]
        ext.conv_wgrad_sgd(d, x, k, k, 1, pad, int(x2 or 0), spec['w'], spec['mom'], spec['shadow'], spec['planes'],
                           spec['plane_stride'], spec['lr'], spec['momentum'], spec['wd'], spec['rescale'],
                           spec['clip'], spec['grad_bf16'])
        spec['applied'] = True
        return dx, None
    tgt = _wtarget(wparam, shape4) if need_w else None
    if need_x and need_w and tgt is not None:
        dx = ext.conv_dgrad_wgrad(d, wk, k - 1 - pad, None, None, 0.0, False, None, None, None, None, d, x, k, k, 1, pad,
                                  tgt, rmask=rmask, rmask_scale=rmask_scale, **kw)[0]
        return dx, None
    if need_w:
        if tgt is not None:
            ext.conv_wgrad(d, x, k, k, 1, pad, 0, tgt, x2=x2)
        else:
            dw = ext.conv_wgrad(d, x, k, k, 1, pad, x2=x2)
            if w.dim() == 4 and tuple(w.shape) != shape4:  # (h, w, c) rows -> the (O, C, H, W) filter
                dw = dw.reshape(w.shape[0], w.shape[2], w.shape[3], w.shape[1]).permute(0, 3, 1, 2)
            dw = dw.reshape(w.shape).to(w.dtype)
    if need_x:
        dx = ext.conv_igemm_fwd(d, wk, None, 1, k - 1 - pad, False, rmask=rmask, rmask_scale=rmask_scale, **kw)[0]
    return dx, dw


class _VGGTrunk(torch.autograd.Function):
    """conv1_1 .. conv5_3 (3x3, pad 1, + bias + ReLU), 2x2/2 max-pools after groups 1-4.
    Arguments: image, pool-after indices, then weight / bias of every conv."""

    @staticmethod
    def forward(ctx, x, pool_after, *wb):
        ext = need_ext()
        from .stem import stem_conv
        x2 = precision.x2_enabled()
        n = len(wb) // 2
        ws, bs = wb[0::2], wb[1::2]
        acts, args = [], {}  # acts[i - 1]: the input of conv i (a ReLU or max-pool output)
        y = stem_conv(x, ws[0], 1, 1, bias=bs[0], relu=True)  # conv1_1: 3 input channels
        for i in range(1, n):
            if (i - 1) in pool_after:
                H, W = y.shape[2], y.shape[3]
                y, arg = ext.maxpool_fwd(y, 2, 2, 0, x2)
                args[i] = (arg, H, W)
            acts.append(y)
            wk, kw = _wargs(ws[i])
            y = ext.conv_igemm_fwd(y, wk, bs[i], 1, 1, True, **kw)[0]
        ctx.n = n
        ctx.args = args
        ctx.params = tuple(p if p.is_leaf else None for p in wb)
        ctx.save_for_backward(y, *acts, *ws)
        return y

    @staticmethod
    def backward(ctx, d_out):
        ext = need_ext()
        x2 = precision.x2_enabled()
        n = ctx.n
        saved = ctx.saved_tensors
        y_top, acts, ws = saved[0], saved[1:n], saved[n:]
        ni = ctx.needs_input_grad  # (x, pool_after, w0, b0, w1, b1, ...)
        need_w = [ni[2 + 2 * i] for i in range(n)]
        need_b = [ni[3 + 2 * i] for i in range(n)]
        first = next((i for i in range(n) if need_w[i] or need_b[i]), n)
        grads = [None] * (2 * n)
        if first >= n:
            return (None, None) + tuple(grads)
        assert first >= 1, 'VGG trunk: conv1_1 is frozen (the fused stem has no backward)'
        d = ext.relu_mask_bwd(_cl(d_out), y_top, 1.0, x2)  # relu5_3
        for i in range(n - 1, first - 1, -1):
            x_in = acts[i - 1]
            wparam, bparam = ctx.params[2 * i], ctx.params[2 * i + 1]
            if need_b[i]:
                grads[2 * i + 1] = _bias_grad(d, bparam, x2)
            need_x = i > first
            dx, grads[2 * i] = _layer_backward(d, x_in, ws[i], wparam, need_w[i], need_x, 3, 1,
                                               rmask=x_in if need_x else None)
            if not need_x:
                break
            if i in ctx.args:  # a max-pool feeds conv i: its backward scatters to the winning taps
                arg, H, W = ctx.args[i]
                dx = ext.maxpool_bwd(dx, arg, H, W, 2, 2, 0, x2)
            d = dx
        return (None, None) + tuple(grads)


def vgg_trunk(x, convs, pool_after):
    """The fused trunk for VGG16Trunk's Conv modules (see module docstring)."""
    wb = []
    for c in convs:
        wb += [c.weight, c.bias]
    return _VGGTrunk.apply(x, tuple(pool_after), *wb)


class _VGGHead(torch.autograd.Function):
    """fc6 -> ReLU -> Dropout -> fc7 -> ReLU -> Dropout -> (cls_score, bbox_pred) on (R, K) rows."""

    @staticmethod
    def forward(ctx, x, p, seeds, step, w6, b6, w7, b7, wc, bc, wb, bb):
        ext = need_ext()
        x2 = precision.x2_enabled()
        R = x.shape[0] // x2 if x2 else x.shape[0]

        def fc(inp, w, b, relu, seed, out_f32=False):
            wk, kw = _wargs(w, (w.shape[0], _kdim(w), 1, 1))
            drop = p if (relu and p > 0) else 0.0
            y = ext.conv_igemm_fwd(inp.view(inp.shape[0], inp.shape[1], 1, 1), wk, b, 1, 0, relu, drop_p=drop,
                                   drop_seed=seed, drop_step=step if drop > 0 else None, out_f32=out_f32, **kw)[0]
            return y.view(y.shape[0], y.shape[1])

        x = x.contiguous()
        y6 = fc(x, w6, b6, True, seeds[0])
        y7 = fc(y6, w7, b7, True, seeds[1])
        sc = fc(y7, wc, bc, False, 0, out_f32=x2)
        bp = fc(y7, wb, bb, False, 0, out_f32=x2)
        ctx.save_for_backward(x, y6, y7, w6, w7, wc, wb)
        leaf = lambda t: t if (t is not None and t.is_leaf) else None  # noqa: E731
        ctx.params = tuple(leaf(t) for t in (w6, b6, w7, b7, wc, bc, wb, bb))
        ctx.p = p
        return sc.view(R, -1), bp.view(R, -1)

    @staticmethod
    def backward(ctx, dsc, dbp):
        x, y6, y7, w6, w7, wc, wb = ctx.saved_tensors
        ni = ctx.needs_input_grad  # (x, p, seeds, step, w6, b6, w7, b7, wc, bc, wb, bb)
        x2 = precision.x2_enabled()
        pw6, pb6, pw7, pb7, pwc, pbc, pwb, pbb = ctx.params
        R = y7.shape[0] // x2 if x2 else y7.shape[0]
        gdt = torch.float32 if x2 else y7.dtype
        if dsc is None:
            dsc = torch.zeros((R, wc.shape[0]), dtype=gdt, device=y7.device)
        if dbp is None:
            dbp = torch.zeros((R, wb.shape[0]), dtype=gdt, device=y7.device)
        scale = 1.0 / (1.0 - ctx.p) if ctx.p > 0 else 1.0
        grads = [None] * 8
        need7 = ni[6] or ni[7] or ni[4] or ni[5] or ni[0]
        # predictors: dW / db of both, and dX masked by relu7 / drop7 = fc7's pre-activation gradient
        d7, dws, dbs = _pair_backward(y7, [dsc, dbp], [wc, wb], [pwc, pwb], [pbc, pbb], [ni[8], ni[10]],
                                      [ni[9], ni[11]], need7, True, mask_scale=scale)
        grads[4], grads[5], grads[6], grads[7] = dws[0], dbs[0], dws[1], dbs[1]
        if not need7:
            return (None,) * 4 + tuple(grads)
        m = lambda t: t.view(t.shape[0], t.shape[1], 1, 1)  # noqa: E731  rows as a 1x1 map
        need6 = ni[4] or ni[5] or ni[0]
        if ni[7]:
            grads[3] = _bias_grad(m(d7), pb7, x2)
        d6, grads[2] = _layer_backward(m(d7), m(y6), w7, pw7, ni[6], need6, 1, 0, rmask=m(y6) if need6 else None,
                                       rmask_scale=scale)
        dx = None
        if need6:
            if ni[5]:
                grads[1] = _bias_grad(d6, pb6, x2)
            dx, grads[0] = _layer_backward(d6, m(x), w6, pw6, ni[4], ni[0], 1, 0)
            if dx is not None:
                dx = dx.view(x.shape)
        return (dx, None, None, None) + tuple(grads)


def vgg_head(x, head):
    """The fused head for VGGHead's Linear modules; ``x`` (R, C*7*7) rows of the pooled map in
    (h, w, c) order (its channels_last memory), the order of fc6's filter rows."""
    from .fc import layer_seed
    training = head.training
    p = float(head.dropout) if training else 0.0
    seeds = (layer_seed(head.fc6.mx_name), layer_seed(head.fc7.mx_name))
    return _VGGHead.apply(x, p, seeds, head.fc6.rng_step, head.fc6.weight, head.fc6.bias, head.fc7.weight, head.fc7.bias,
                          head.cls_score.weight, head.cls_score.bias, head.bbox_pred.weight, head.bbox_pred.bias)


def trunk_ok(x, convs):
    """True when the fused trunk can run (GPU bf16 / x2 pairs, frozen conv1_1 for the fused stem)."""
    import os
    from .conv import weight_ok
    from .stem import stem_fusable
    if os.environ.get('MXR_VGG_FUSED', '1') == '0' or not x.is_cuda:
        return False
    act = torch.zeros((), dtype=torch.bfloat16) if precision.x2_enabled() else x
    return (stem_fusable(x, convs[0].weight, convs[0].bias) and
            all(weight_ok(act, c.weight) and c.bias is not None and c.weight.shape[1] % 64 == 0 for c in convs[1:]))


def head_ok(x, head):
    """True when the fused head can run on rows ``x`` (R, K) in (h, w, c) order: fc6 must be held
    as the (O, C, H, W) filter (Linear in_shape) whose channels_last rows have that order."""
    import os
    from .conv import weight_ok
    if os.environ.get('MXR_VGG_FUSED', '1') == '0' or not x.is_cuda or x.dtype != torch.bfloat16:
        return False
    if head.fc6.weight.dim() != 4:
        return False
    fcs = (head.fc6, head.fc7)
    if head.training and head.dropout > 0 and head.fc6.rng_step is None:
        return False
    return (x.shape[1] % 64 == 0 and all(weight_ok(x, f.weight) and f.bias is not None and f.weight.shape[0] % 64 == 0
                                         for f in fcs) and
            pair_eligible(x, [head.cls_score.weight, head.bbox_pred.weight], head.fc7.weight.shape[0]) and
            head.cls_score.bias is not None and head.bbox_pred.bias is not None)
