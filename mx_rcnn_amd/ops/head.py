"""Paired prediction heads with a one-launch backward (csrc/hip/head_bwd.hip).

Both detection stages end in two small layers that read the same input:

* RPN: ``rpn_conv_3x3 -> relu -> {rpn_cls_score, rpn_bbox_pred}`` 1x1 convs with 2A / 4A outputs
  (`rcnn/symbol.py:165-172`);
* detector: ``{cls_score, bbox_pred}`` FullyConnected layers with C / 4C outputs over the pooled
  RoI feature (`rcnn/symbol.py:108-111`, `rcnn/resnet.py:167-171`).

Their output widths (24 ... 324) are below one 64-wide MFMA tile and not multiples of 8, which the
implicit-GEMM / wgrad kernels need, so their backward used to be per head a vendor GEMM for dX and
dW, a torch column sum for db, dtype casts and autograd adds -- about 14 small launches in series
on the step's critical path.  Here the pair's backward is ONE kernel (dX summed over both heads,
both dW, both db, written / accumulated straight into the flat gradient buffers), and for the RPN
the ReLU backward of ``rpn_conv_3x3`` rides in the same epilogue (dX masked by the ReLU output), so
the 3x3 conv's backward starts from the pre-activation gradient and its bias gradient is one
channel-sum kernel.  Forward is unchanged: the implicit-GEMM conv with the bias in its epilogue.
"""
import os

import torch

from . import grad_sink
from . import precision
from ._ext import need_ext
from .conv import LOWP, conv_backward, weight_ok


def head_kernel_enabled():
    return os.environ.get('MXR_HEAD_KERNEL', '1') != '0'


def _mat(t):
    """(M, K) row view of a 2-D matrix or a channels_last (N, K, H, W) map."""
    if t.dim() == 4:
        t = t.contiguous(memory_format=torch.channels_last)
        return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])
    return t.contiguous()


def _aligned(t):
    return t.data_ptr() % 16 == 0


def pair_eligible(x, ws, K):
    """x: the input tensor (device / dtype check); ws: the heads' (N, K[, 1, 1]) weights."""
    if not (head_kernel_enabled() or precision.x2_enabled()) or not (x.is_cuda and x.dtype == torch.bfloat16):
        return False
    return K % 64 == 0 and all(weight_ok(x, w) and w.is_contiguous() and _aligned(w) and
                               w.numel() == w.shape[0] * K for w in ws)


def _mat_w(w):
    """(N, K) view of a head weight for the kernels, with its lo-plane offset in the x2 mode."""
    if precision.x2_enabled():
        wh, wpl = precision.weight_pair(w)
        return wh.reshape(wh.shape[0], -1), wpl
    return w.reshape(w.shape[0], -1), 0


def _pair_backward(x2, dys, ws, wparams, bparams, need_w, need_b, need_dx, relu_mask, mask_scale=1.0):
    """-> (dx (M, K) or None, [dW_h or None], [db_h or None]); gradients with a flat-buffer target
    are accumulated there and returned as None (grad_sink)."""
    ext = need_ext()
    xp = precision.x2_enabled()  # fp32-class pairs: x2 (2M, K), dY / dW fp32
    gdt = torch.float32 if xp else torch.bfloat16
    dws, dw_acc, dw_ret, dbs, db_acc, db_ret = [], [], [], [], [], []
    empty = x2.new_empty(0)
    for h, (dy, w) in enumerate(zip(dys, ws)):
        N = dy.shape[1]
        tgt = grad_sink.target(wparams[h]) if need_w[h] else None
        if tgt is not None and tgt.is_contiguous() and tgt.dtype == gdt and _aligned(tgt):
            dws.append(tgt.view(N, -1))
            dw_acc.append(True)
            dw_ret.append(None)
        else:
            d = torch.empty((N, x2.shape[1]), dtype=gdt, device=x2.device)
            dws.append(d)  # computed even when not needed: the kernel writes every head's dW
            dw_acc.append(False)
            dw_ret.append(d.view(w.shape) if need_w[h] else None)
        if need_b[h]:
            tb = grad_sink.target(bparams[h])
            if tb is not None and tb.is_contiguous():
                dbs.append(tb)
                db_acc.append(True)
                db_ret.append(None)
            else:
                d = torch.empty(N, dtype=torch.float32, device=x2.device)
                dbs.append(d)
                db_acc.append(False)
                db_ret.append(d)
        else:
            dbs.append(empty)
            db_acc.append(False)
            db_ret.append(None)
    wm = [_mat_w(w) for w in ws]
    dx = ext.head_bwd(x2, [_mat(d).to(gdt) for d in dys], [m[0] for m in wm], dws, dw_acc, dbs, db_acc, bool(need_dx),
                      bool(relu_mask), xp, [m[1] for m in wm], float(mask_scale))
    db_ret = [d.to(bparams[h].dtype) if (d is not None and bparams[h] is not None) else d
              for h, d in enumerate(db_ret)]
    return (dx if need_dx else None), dw_ret, db_ret


class _FCPair(torch.autograd.Function):
    """(x W1^T + b1, x W2^T + b2) over 2-D x."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        ext = need_ext()
        xm = x.contiguous().view(x.shape[0], x.shape[1], 1, 1)
        xp = precision.x2_enabled()
        M = x.shape[0] // xp if xp else x.shape[0]
        ys = []
        for w, b in ((w1, b1), (w2, b2)):
            if xp:  # pairs in, fp32 predictions out
                wh, wpl = _mat_w(w)
                y = ext.conv_igemm_fwd(xm, wh.view(w.shape[0], w.shape[1], 1, 1), b, 1, 0, False, x2=precision.x2_enabled(),
                                       w_plane=wpl, out_f32=True)[0]
            else:
                y = ext.conv_igemm_fwd(xm, w.view(w.shape[0], w.shape[1], 1, 1), b, 1, 0, False)[0]
            ys.append(y.view(M, w.shape[0]))
        ctx.save_for_backward(x, w1, w2)
        ctx.params = (w1 if w1.is_leaf else None, w2 if w2.is_leaf else None)
        ctx.bparams = (b1 if (b1 is not None and b1.is_leaf) else None, b2 if (b2 is not None and b2.is_leaf) else None)
        ctx.has_b = (b1 is not None, b2 is not None)
        return ys[0], ys[1]

    @staticmethod
    def backward(ctx, dy1, dy2):
        x, w1, w2 = ctx.saved_tensors
        ni = ctx.needs_input_grad
        xp = precision.x2_enabled()
        M = x.shape[0] // xp if xp else x.shape[0]
        gdt = torch.float32 if xp else x.dtype
        if dy1 is None:
            dy1 = torch.zeros((M, w1.shape[0]), dtype=gdt, device=x.device)
        if dy2 is None:
            dy2 = torch.zeros((M, w2.shape[0]), dtype=gdt, device=x.device)
        dx, dws, dbs = _pair_backward(x.contiguous(), [dy1, dy2], [w1, w2], ctx.params, ctx.bparams,
                                      [ni[1], ni[3]], [ctx.has_b[0] and ni[2], ctx.has_b[1] and ni[4]], ni[0], False)
        return dx, dws[0], dbs[0], dws[1], dbs[1]


def fc_pair(x, fc1, fc2):
    """(fc1(x), fc2(x)) for two models.layers.Linear sharing the input; falls back to the modules."""
    x = x.reshape(x.shape[0], -1)
    w1, w2 = fc1.weight, fc2.weight
    if (x.dtype in LOWP and weight_ok(x, w1) and weight_ok(x, w2) and pair_eligible(x, [w1, w2], x.shape[1])
            and fc1.bias is not None and fc2.bias is not None):
        return _FCPair.apply(x, w1, fc1.bias, w2, fc2.bias)
    assert not precision.x2_enabled(), 'fp32 (x2) mode: prediction heads without the paired kernel'
    return fc1(x), fc2(x)


class _RpnHead(torch.autograd.Function):
    """a = relu(conv3x3(feat) + bc); (conv1x1_1(a) + b1, conv1x1_2(a) + b2)."""

    @staticmethod
    def forward(ctx, feat, wc, bc, w1, b1, w2, b2):
        ext = need_ext()
        feat = feat.contiguous(memory_format=torch.channels_last)
        if precision.x2_enabled():  # pairs through the 3x3 conv, fp32 RPN predictions
            wcc = wc
            wh, wpl = precision.weight_pair(wc)
            a = ext.conv_igemm_fwd(feat, wh, bc, 1, 1, True, x2=precision.x2_enabled(), w_plane=wpl)[0]
            ys = []
            for w, b in ((w1, b1), (w2, b2)):
                wh, wpl = precision.weight_pair(w)
                ys.append(ext.conv_igemm_fwd(a, wh, b, 1, 0, False, x2=precision.x2_enabled(), w_plane=wpl, out_f32=True)[0])
            y1, y2 = ys
        else:
            wcc = wc.contiguous(memory_format=torch.channels_last)
            a = ext.conv_igemm_fwd(feat, wcc, bc, 1, 1, True)[0]
            y1 = ext.conv_igemm_fwd(a, w1.contiguous(memory_format=torch.channels_last), b1, 1, 0, False)[0]
            y2 = ext.conv_igemm_fwd(a, w2.contiguous(memory_format=torch.channels_last), b2, 1, 0, False)[0]
        ctx.save_for_backward(feat, wcc, a, w1, w2)
        leaf = lambda p: p if (p is not None and p.is_leaf) else None  # noqa: E731
        ctx.params = (leaf(wc), leaf(bc), leaf(w1), leaf(b1), leaf(w2), leaf(b2))
        ctx.has_b = (bc is not None, b1 is not None, b2 is not None)
        return y1, y2

    @staticmethod
    def backward(ctx, dy1, dy2):
        feat, wc, a, w1, w2 = ctx.saved_tensors
        ni = ctx.needs_input_grad
        pc, pbc, p1, pb1, p2, pb2 = ctx.params
        N, C, H, W = a.shape
        xp = precision.x2_enabled()
        Nl = N // xp if xp else N  # logical images (pairs: 2N rows)
        gdt = torch.float32 if xp else a.dtype
        if dy1 is None:
            dy1 = torch.zeros((Nl, w1.shape[0], H, W), dtype=gdt, device=a.device, memory_format=torch.channels_last)
        if dy2 is None:
            dy2 = torch.zeros((Nl, w2.shape[0], H, W), dtype=gdt, device=a.device, memory_format=torch.channels_last)
        need_pre = ni[0] or ni[1] or (ctx.has_b[0] and ni[2])
        d_pre, dws, dbs = _pair_backward(_mat(a), [dy1, dy2], [w1, w2], [p1, p2], [pb1, pb2], [ni[3], ni[5]],
                                         [ctx.has_b[1] and ni[4], ctx.has_b[2] and ni[6]], need_pre, True)
        dfeat = dwc = dbc = None
        if need_pre:
            d_pre = d_pre.view(N, H, W, C).permute(0, 3, 1, 2)  # channels_last (N, C, H, W)
            if ctx.has_b[0] and ni[2]:
                tb = grad_sink.target(pbc)
                if tb is not None and tb.is_contiguous():
                    need_ext().chan_sum(d_pre, tb, True, xp)
                else:
                    dbc = torch.empty(C, dtype=torch.float32, device=a.device)
                    need_ext().chan_sum(d_pre, dbc, False, xp)
                    dbc = dbc.to(pbc.dtype if pbc is not None else torch.float32)
            if ni[0] or ni[1]:
                dfeat, dwc, _ = conv_backward(feat, wc, pc, d_pre, 1, 1, False, ni[0], ni[1], False)
        return dfeat, dwc, dbc, dws[0], dbs[0], dws[1], dbs[1]


def rpn_head(feat, conv, cls, bbox):
    """RPN 3x3 conv + ReLU + the two 1x1 predictors (models.layers.Conv modules)."""
    ws = [cls.weight, bbox.weight]
    if (feat.dtype == torch.bfloat16 and weight_ok(feat, conv.weight) and feat.shape[1] % 64 == 0 and
            conv.weight.shape[0] % 64 == 0 and int(conv.stride) == 1 and int(conv.pad) == 1 and
            conv.weight.shape[2] == 3 and all(weight_ok(feat, w) for w in ws) and
            pair_eligible(feat, ws, conv.weight.shape[0]) and all(int(c.stride) == 1 and int(c.pad) == 0 for c in (cls, bbox))):
        return _RpnHead.apply(feat, conv.weight, conv.bias, cls.weight, cls.bias, bbox.weight, bbox.bias)
    assert not precision.x2_enabled(), 'fp32 (x2) mode: RPN head without the paired kernel'
    x = conv(feat, relu=True)
    return cls(x), bbox(x)
