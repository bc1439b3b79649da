"""Fused loss ops with MXNet head semantics:

* ``rpn_softmax_ce``  = SoftmaxOutput(multi_output, use_ignore, ignore=-1, 'valid') over the
  (B, 2, A*H, W) reshape of the RPN logits (`rcnn/symbol.py:194`, `rcnn/resnet.py:96`).
* ``softmax_ce``      = SoftmaxOutput(normalization='batch' or 'null') for the R-CNN head.
* ``smooth_l1``       = MakeLoss(outside * smooth_l1(inside * (pred - target), sigma), grad_scale).

Each returns a scalar whose autograd gradient is exactly the gradient MXNet back-propagates
(the fused HIP kernels compute value and gradient in one pass and backward only rescales
the stored gradient by the incoming scalar).  Returned values are the metric quantities:
mean -log p over the normalisation count, and grad_scale * sum(elementwise loss).
"""
import torch

from ._ext import ext_available, is_unit_grad, need_ext


class _RpnCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, label, grad_scale, meta):
        B, C2, H, W = logits.shape
        A = C2 // 2
        lab = label.to(torch.int32).contiguous()
        if logits.is_cuda:
            ext = need_ext()
            if meta is not None:  # sampled fg + bg counts from anchor_sample: no count reduction
                grad, loss = ext.rpn_softmax_ce(logits, lab, None, float(grad_scale), False, meta)
            else:
                norm = (lab >= 0).sum().float().reshape(1)
                grad, loss = ext.rpn_softmax_ce(logits, lab, norm, float(grad_scale), False)
            ctx.save_for_backward(grad)
            return loss.reshape(())  # normalised in-kernel
        if ext_available():  # C++ twin (host_ops.h); the tensor version below is its oracle
            grad, loss = need_ext().rpn_softmax_ce_cpu(logits, lab, float(grad_scale))
            ctx.save_for_backward(grad.to(logits.dtype))
            return loss.reshape(())
        norm = (lab >= 0).sum().float().reshape(1)
        z = logits.float().reshape(B, 2, A * H, W)
        p = torch.softmax(z, dim=1)
        l4 = lab.reshape(B, A * H, W).long()
        valid = l4 >= 0
        onehot = torch.stack([(l4 == 0), (l4 == 1)], dim=1).float()
        g = (p - onehot) * valid[:, None].float() * (grad_scale / norm.clamp_min(1))
        grad = g.reshape(B, C2, H, W).to(logits.dtype)
        pl = torch.where(l4 == 1, p[:, 1], p[:, 0]).clamp_min(1e-14)
        loss = (-(torch.log(pl)) * valid.float()).sum().reshape(1)
        ctx.save_for_backward(grad)
        return (loss / norm.clamp_min(1)).reshape(())

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return _scale_grad(grad, g), None, None, None


def _scale_grad(grad, g):
    """The stored loss gradient times the incoming scalar (in place on the GPU: one kernel; none
    when the backward was seeded with ``unit_grad`` and the one arrives unchanged)."""
    if is_unit_grad(g):
        return grad
    if (grad.is_cuda and g.dtype == torch.float32 and
            (grad.is_contiguous() or grad.is_contiguous(memory_format=torch.channels_last))):
        return need_ext().scale_by_scalar_(grad, g.reshape(1))
    return grad * g.to(grad.dtype)


def rpn_softmax_ce(logits, label, grad_scale=1.0, sample_meta=None):
    """logits (B, 2A, H, W), label (B, A*H*W) in {-1, 0, 1}.  ``sample_meta`` (B, 4) from the GPU
    anchor sampler ([all_fg, all_bg, n_fg, n_bg]) supplies the 'valid' count directly."""
    return _RpnCE.apply(logits, label, grad_scale, sample_meta)


class _RowCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, label, norm, grad_scale):
        lab = label.to(torch.int32).contiguous()
        ctx.set_materialize_grads(False)  # prob never receives a gradient: no zero fill for it
        if logits.is_cuda:
            ext = need_ext()
            grad, prob, loss = ext.row_softmax_ce(logits.contiguous(), lab, float(norm), float(grad_scale), True)
            ctx.save_for_backward(grad)
            ctx.mark_non_differentiable(prob)
            return loss.reshape(()), prob  # divided by norm in-kernel
        if ext_available():  # C++ twin (host_ops.h)
            grad, prob, loss = need_ext().row_softmax_ce_cpu(logits, lab, float(norm), float(grad_scale))
            ctx.save_for_backward(grad.to(logits.dtype))
            ctx.mark_non_differentiable(prob)
            return loss.reshape(()), prob
        p = torch.softmax(logits.float(), dim=1)
        valid = (lab >= 0)
        onehot = torch.nn.functional.one_hot(lab.long().clamp_min(0), logits.shape[1]).float()
        grad = ((p - onehot) * valid[:, None].float() * (grad_scale / norm)).to(logits.dtype)
        prob = p
        pl = p.gather(1, lab.long().clamp_min(0)[:, None])[:, 0].clamp_min(1e-14)
        loss = (-torch.log(pl) * valid.float()).sum().reshape(1)
        ctx.save_for_backward(grad)
        ctx.mark_non_differentiable(prob)
        return (loss / norm).reshape(()), prob

    @staticmethod
    def backward(ctx, g, gprob):
        if g is None:
            return None, None, None, None
        (grad,) = ctx.saved_tensors
        return _scale_grad(grad, g), None, None, None


def softmax_ce(logits, label, normalization='batch', grad_scale=1.0):
    """logits (R, C), label (R,).  Returns (mean loss, prob (R, C) fp32)."""
    R = logits.shape[0]
    if normalization == 'batch':
        norm = float(max(R, 1))
    elif normalization == 'null':
        norm = 1.0
    else:
        raise ValueError('normalization %r not supported for the head loss' % normalization)
    return _RowCE.apply(logits, label, norm, grad_scale)


class _SmoothL1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, inside, outside, sigma, grad_scale, slot):
        t = target.float().contiguous()
        iw = inside.float().contiguous()
        ow = outside.float().contiguous()
        if pred.is_cuda:
            ext = need_ext()
            grad, loss = ext.smooth_l1(pred, t, iw, ow, float(sigma), float(grad_scale), int(slot))
        elif ext_available():  # C++ twin (host_ops.h)
            grad, loss = need_ext().smooth_l1_cpu(pred, t, iw, ow, float(sigma), float(grad_scale))
            grad = grad.to(pred.dtype)
        else:
            s2 = sigma * sigma
            x = iw * (pred.float() - t)
            ax = x.abs()
            small = ax < 1.0 / s2
            f = torch.where(small, 0.5 * s2 * x * x, ax - 0.5 / s2)
            d = torch.where(small, s2 * x, torch.sign(x))
            grad = (grad_scale * ow * d * iw).to(pred.dtype)
            loss = (ow * f).sum().reshape(1)
        ctx.save_for_backward(grad)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return _scale_grad(grad, g), None, None, None, None, None, None


def smooth_l1(pred, target, inside_weight, outside_weight, sigma=1.0, grad_scale=1.0, slot=2):
    """Returns sum(outside * f(inside * (pred - target))) (the MakeLoss output summed, i.e. the
    metric quantity); its autograd gradient is grad_scale * d/dpred of that sum.  ``slot``: the
    GPU kernel's grid-reduction ticket (2..63); calls that may run concurrently need distinct slots."""
    return _SmoothL1.apply(pred, target, inside_weight, outside_weight, float(sigma), float(grad_scale), int(slot))


class _Combine(torch.autograd.Function):
    """total = sum(terms) (carries the gradient: each term receives the incoming scalar) and
    objective = sum(w_i * term_i) (detached), plus the non-finite step counter, in one launch."""

    @staticmethod
    def forward(ctx, weights, nonfinite, *terms):
        ctx.n = len(terms)
        if terms[0].is_cuda:
            out = need_ext().loss_combine([t.reshape(1).float() for t in terms], list(weights), nonfinite)
            total, obj = out[0], out[1]
        else:
            total = sum(terms)
            obj = sum(w * t for w, t in zip(weights, terms))
            if nonfinite is not None:
                nonfinite.add_((~torch.isfinite(obj)).to(nonfinite.dtype))
        ctx.mark_non_differentiable(obj)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the objective output
        return total.reshape(()), obj.reshape(())

    @staticmethod
    def backward(ctx, g, _gobj):
        if g is None:
            return (None, None) + (None,) * ctx.n
        return (None, None) + (g,) * ctx.n


def combine_losses(terms, weights, nonfinite=None):
    """-> (total loss for backward, objective value).  ``nonfinite`` (int32 (1,) or 0-d device
    counter) is incremented when the objective is not finite (the trainer's guard)."""
    return _Combine.apply(tuple(float(w) for w in weights), nonfinite, *terms)
