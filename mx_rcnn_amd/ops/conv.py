"""Convolution dispatch for channels_last bf16 activations on MI355X.

* Cin % 64 == 0 (every ResNet/VGG conv except the 3-channel stem): hand-written MFMA
  implicit-GEMM forward (csrc/hip/conv_igemm.hip) with fused bias + ReLU epilogue and split-K
  for the latency-bound small-M shapes of 1-image detection (the LDS-DMA kernel beats
  hipBLASLt on every trunk 1x1 shape, tools/microbench/conv_tiles.py); strided 1x1 convs
  subsample first.
* Backward: stride-1 data gradient = the same kernel on dY reading the forward filter
  transposed with flipped taps (pad' = k-1-pad, ConvEpi::bt); weight gradient = the MFMA wgrad kernel (csrc/hip/conv_wgrad.hip),
  which ACCUMULATES straight into the parameter's flat-buffer gradient view when the
  parameter is managed by the FlatParamStore (ops/grad_sink.py: no AccumulateGrad add);
  strided data gradients are parity-decomposed into s*s stride-1 convs of dy written straight
  into their positions of dx (``strided_dgrad``); anything else uses MIOpen.
* Anything else: MIOpen.  ``MXR_CONV_IGEMM=0`` / ``MXR_CONV_WGRAD=0`` switch the custom
  kernels off for A/B runs.
"""
import os
import weakref

import torch
import torch.nn.functional as F

from . import grad_sink
from . import precision
from ._ext import need_ext

LOWP = (torch.bfloat16, torch.float16)  # MFMA operand dtypes (fp16: the inference path)

def igemm_enabled():
    return os.environ.get('MXR_CONV_IGEMM', '1') != '0'


def wgrad_enabled():
    return os.environ.get('MXR_CONV_WGRAD', '1') != '0'


# dgrad operand cache: id(weight Parameter) -> (weakref(param), flipped/transposed bf16 filter),
# refreshed by the FlatParamStore with ONE multi-filter kernel right after each SGD update
# (core/params.py), instead of a flip + transpose copy per conv per backward.  Entries hold the
# parameter WEAKLY and are dropped when it dies (a finalizer per parameter), so the tables neither
# pin a dead trainer's model nor hand its buffers to a later parameter that reuses the id.
_DGRAD_W = {}
# parity sub-filters of the cached flipped filters (strided dgrad): (id(param), taps) ->
# (weakref(param), source view builder, buffer); rebuilt with the cache
# (FlatParamStore.refresh_dgrad_cache)
_SUBW = {}
_FINAL = set()


def _drop_param(pid):
    _FINAL.discard(pid)
    _DGRAD_W.pop(pid, None)
    for k in [k for k in _SUBW if k[0] == pid]:
        del _SUBW[k]


def _track(param):
    pid = id(param)
    if pid not in _FINAL:
        _FINAL.add(pid)
        weakref.finalize(param, _drop_param, pid)


def register_dgrad_weight(param, buf):
    _track(param)
    _DGRAD_W[id(param)] = (weakref.ref(param), buf)


def sub_filter(param, wf, th, tw, s):
    """The (I, O, |th|, |tw|) channels_last slice of the flipped filter ``wf`` at taps th[0]::s /
    tw[0]::s; cached per parameter and refreshed with the dgrad cache, so the strided data
    gradient does not copy sub-filters on the critical path."""
    def view(w):
        return w[:, :, th[0]:th[-1] + 1:s, tw[0]:tw[-1] + 1:s]
    if param is None or cached_dgrad_weight(param) is not wf:
        return view(wf).contiguous(memory_format=torch.channels_last)
    key = (id(param), th[0], th[-1], tw[0], tw[-1], s)
    ent = _SUBW.get(key)
    if ent is None or ent[0]() is not param:
        buf = view(wf).contiguous(memory_format=torch.channels_last)
        _track(param)
        _SUBW[key] = (weakref.ref(param), view, buf)
        return buf
    return ent[2]


def sub_filter_entries():
    """[(param, view builder, buffer)] of the live parity sub-filters."""
    out = []
    for ref, view, buf in list(_SUBW.values()):
        p = ref()
        if p is not None:
            out.append((p, view, buf))
    return out


def sub_filters_of(param):
    """[(buf, row taps, col taps)] registered for ``param`` (the flip kernel's table writes them
    in the same pass as the flipped filter, core/params.py)."""
    out = []
    for (pid, r0, r1, c0, c1, s), (ref, _view, buf) in list(_SUBW.items()):
        if ref() is param:
            out.append((buf, list(range(r0, r1 + 1, s)), list(range(c0, c1 + 1, s))))
    return out


def refresh_sub_filters(skip=()):
    """Copy the sub-filters of every parameter not in ``skip`` (ids whose sub-filters the flip
    kernel already wrote)."""
    for param, view, buf in sub_filter_entries():
        if id(param) in skip:
            continue
        wf = cached_dgrad_weight(param)
        if wf is not None:
            buf.copy_(view(wf))


def cached_dgrad_weight(param):
    """The cached flipped / transposed filter of ``param`` or None."""
    ent = _DGRAD_W.get(id(param)) if param is not None else None
    return ent[1] if ent is not None and ent[0]() is param else None


def dgrad_weight(param, w):
    wf = cached_dgrad_weight(param)
    if wf is not None:
        return wf
    if precision.x2_enabled():  # the flipped fp32 filter as a pair
        return precision.split(_flip_t(w.detach().float()))
    return _flip_t(w)


def dgrad_bt_enabled():
    """Stride-1 data gradients read the forward filter transposed in-kernel (ConvEpi::bt) instead
    of a flipped / transposed copy rebuilt after every update (``MXR_DGRAD_BT=0``: the copy)."""
    return os.environ.get('MXR_DGRAD_BT', '1') != '0'


def dgrad_args(param, w):
    """(filter, conv kwargs) of a stride-1 data-gradient launch for the conv with weight ``w``
    (the tensor its forward used: the bf16 shadow, or in the x2 mode the fp32 parameter)."""
    x2 = precision.x2_enabled()
    if dgrad_bt_enabled():
        if x2:
            wh, wpl = precision.weight_pair(w)
            return wh, {'x2': x2, 'w_plane': wpl, 'bt': True}
        return w.contiguous(memory_format=torch.channels_last), {'bt': True}
    wf = dgrad_weight(param, w)
    if x2:
        wh, wpl = pair_args(wf)
        return wh, {'x2': x2, 'w_plane': wpl}
    return wf, {}


def pair_args(wpair):
    """Multi-plane modes: a filter's planes (P*O, ...) -> (plane-0 view, plane spacing) for the
    kernels' w / w_plane."""
    k = precision.nplanes() or 2
    n = wpair.shape[0] // k
    return wpair[:n], wpair.numel() // k


def _flip_t(w):
    """(O, I, kh, kw) -> (I, O, kh, kw) spatially flipped, channels_last memory."""
    if w.shape[2] == 1 and w.shape[3] == 1:
        return w.transpose(0, 1).contiguous(memory_format=torch.channels_last)
    return w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)


def _parity_taps(k, s, p, ph):
    """Filter taps of the flipped filter that reach input rows of parity ``ph`` in the data
    gradient of a (k, stride s, pad p) conv, and the dy offset of the first one."""
    q = k - 1 - p
    taps = [t for t in range(k) if (ph + t - q) % s == 0]
    off = (ph + taps[0] - q) // s if taps else 0
    return taps, off


def strided_dgrad_ok(k, s, p, H, W):
    """True when every parity class of the data gradient has taps and starts at or before its
    dy row (so it is a padded stride-1 conv over dy).  ``MXR_STRIDED_DGRAD=0`` disables the path."""
    if os.environ.get('MXR_STRIDED_DGRAD', '1') == '0':
        return False
    for ph in range(min(s, H)):
        taps, off = _parity_taps(k, s, p, ph)
        if not taps or off > 0:
            return False
    return True


def strided_dgrad_parts(N, H, W, s):
    """Partial rows the parity-class launches of strided_dgrad write with ``bnb_part`` (one per
    64-row tile of each class grid)."""
    return sum((N * ((H - ph + s - 1) // s) * ((W - pw + s - 1) // s) + 63) // 64
               for ph in range(s) for pw in range(s) if H > ph and W > pw)


def strided_dgrad(dy, wf, H, W, k, s, p, residual=None, bn=None, bn_eps=2e-5, bn_fix_gamma=False, bnb_x=None,
                  dadd=None, dgamma=None, dbeta=None, param=None, bnb_part=None):
    """Data gradient of a stride-``s`` k x k conv (pad p) on the MFMA kernel, by parity
    decomposition: input rows / columns of parity (ph, pw) receive only the filter taps of matching
    parity, so each of the s*s classes is a small stride-1 conv of dy with a sub-filter, written
    straight into its positions of dx by the epilogue's output row map (no dilated dy, no scatter
    pass).  ``wf`` is the flipped / transposed filter (I, O, k, k) of the dgrad cache.  The
    optional BN-ReLU backward epilogue (``bn`` + ``bnb_x`` [+ ``dadd``, ``residual``]) accumulates
    dgamma / dbeta over the classes, or with ``bnb_part`` writes their deterministic partial rows
    (the classes in order, strided_dgrad_parts rows in all)."""
    ext = need_ext()
    N, O, Ho, Wo = dy.shape
    x2 = precision.x2_enabled()
    I = wf.shape[0] // x2 if x2 else wf.shape[0]  # planes: wf is the flipped filter's planes
    dx = torch.empty((N, I, H, W), dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
    bwd = bnb_x is not None
    row0 = 0
    if bwd and bnb_part is not None:
        dgamma = dbeta = None
    elif bwd and dgamma is None:
        dgamma = torch.zeros(I, dtype=torch.float32, device=dy.device)
        dbeta = torch.zeros(I, dtype=torch.float32, device=dy.device)
    for ph in range(s):
        Hc = (H - ph + s - 1) // s
        if Hc <= 0:
            continue
        th, oh = _parity_taps(k, s, p, ph)
        for pw in range(s):
            Wc = (W - pw + s - 1) // s
            if Wc <= 0:
                continue
            tw, ow = _parity_taps(k, s, p, pw)
            # the taps of one parity are an arithmetic progression of step s: plain slicing (an index
            # list would be a host-to-device copy, illegal inside graph capture)
            sub = sub_filter(param, wf, th, tw, s)
            wk = {}
            if x2:
                sub, wpl = pair_args(sub)
                wk = dict(x2=x2, w_plane=wpl)
            ext.conv_igemm_fwd(dy, sub, None, 1, -oh, False, 0, 0, residual, bn, bn_eps, bn_fix_gamma, True,
                               bnb_x, dadd, dgamma, dbeta, 0.0, 0, None, -ow, dx, [Hc, Wc, H, W, s, s, ph, pw],
                               bnb_part=bnb_part, bnb_row0=row0, **wk)
            row0 += ((N // x2 if x2 else N) * Hc * Wc + 63) // 64
    if bwd:
        return dx, dgamma, dbeta
    return dx


def _grouped_target(x, w, param, dy, stride, pad):
    """The flat-gradient target when this conv's data + weight gradient can run as ONE grouped
    launch (csrc/hip/conv_igemm.hip conv_dgrad_wgrad: stride 1, same padding, bf16 / x2 pairs),
    else None."""
    if os.environ.get('MXR_GROUPED_CONV', '1') == '0' or not wgrad_enabled():
        return None
    kh = w.shape[2]
    if not (stride == 1 and 2 * pad == kh - 1 and kh == w.shape[3] and x.dtype == torch.bfloat16 and
            dy.dtype == torch.bfloat16 and w.shape[0] % 64 == 0 and w.shape[1] % 64 == 0):
        return None
    tgt = grad_sink.target(param)
    gdt = torch.float32 if precision.x2_enabled() else torch.bfloat16
    if tgt is None or tgt.dtype != gdt or not tgt.is_contiguous(memory_format=torch.channels_last):
        return None
    return tgt


def conv_backward(x, w, param, dy, stride, pad, has_bias, need_x, need_w, need_b, bparam=None):
    """(dx, dw, db) of an NHWC bf16 conv given the gradient at its (pre-activation) output.
    dw is None when it was accumulated straight into the parameter's flat gradient view."""
    kh = w.shape[2]
    dx = dw = db = None
    x2 = precision.x2_enabled()
    tgt = _grouped_target(x, w, param, dy, stride, pad) if (need_x and need_w and x.is_cuda) else None
    if tgt is not None:
        x = x.contiguous(memory_format=torch.channels_last)
        dy = dy.contiguous(memory_format=torch.channels_last)
        wf, wk = dgrad_args(param, w)
        dx = need_ext().conv_dgrad_wgrad(dy, wf, kh - 1 - pad, None, None, 0.0, False, None,
                                         None, None, None, dy, x, kh, kh, 1, pad, tgt, **wk)[0]
        if has_bias and need_b:
            db = _bias_grad(dy, w, bparam)
        return dx, None, db
    # the weight gradient runs on a side stream concurrently with the data gradient (joined before
    # returning, so readiness hooks and frees see finished writes)
    side = main = None
    if need_w and x.is_cuda and need_x:
        from .fused import _side_stream
        side = _side_stream(x.device)
        if side is not None:
            main = torch.cuda.current_stream()
            side.wait_stream(main)
    if side is not None:
        with torch.cuda.stream(side):
            dw, db = _wgrad(x, w, param, dy, stride, pad, has_bias, need_w, need_b, bparam)
    if need_x:
        if stride == 1 and w.shape[0] % 64 == 0 and 2 * pad == kh - 1:
            wf, wk = dgrad_args(param, w)
            dx = need_ext().conv_igemm_fwd(dy, wf, None, 1, kh - 1 - pad, False, **wk)[0]
        elif (stride > 1 and w.shape[0] % 64 == 0 and w.shape[1] % 8 == 0 and kh == w.shape[3] and
              strided_dgrad_ok(kh, stride, pad, x.shape[2], x.shape[3])):
            dx = strided_dgrad(dy, dgrad_weight(param, w), x.shape[2], x.shape[3], kh, stride, pad, param=param)
        else:
            assert not x2, 'fp32 (x2) mode: no MFMA data gradient for this conv shape'
            dx = torch.ops.aten.convolution_backward(
                dy, x, w, None, [stride] * 2, [pad] * 2, [1, 1], False, [0, 0], 1, [True, False, False])[0]
    if side is None:
        dw, db = _wgrad(x, w, param, dy, stride, pad, has_bias, need_w, need_b, bparam)
    else:
        main.wait_stream(side)
        for t in (dw, db):  # allocated on the side stream, consumed (and freed) on the compute stream
            if t is not None:
                t.record_stream(main)
    return dx, dw, db


def _bias_grad(dy, w, bparam):
    """Per-channel sum of dy (HIP two-pass column sum, accumulated straight into the bias's flat
    gradient view when it has one) -> db or None."""
    tb = grad_sink.target(bparam)
    x2 = precision.x2_enabled()
    if tb is not None and tb.is_contiguous():
        need_ext().chan_sum(dy, tb, True, x2)
        return None
    db = torch.empty(w.shape[0], dtype=torch.float32 if x2 else w.dtype, device=dy.device)
    need_ext().chan_sum(dy, db, False, x2)
    return db


def _wgrad(x, w, param, dy, stride, pad, has_bias, need_w, need_b, bparam=None):
    dw = db = None
    x2 = precision.x2_enabled()
    if need_w and (wgrad_enabled() or x2) and w.shape[0] % 8 == 0:
        tgt = grad_sink.target(param)
        if tgt is not None and tgt.is_contiguous(memory_format=torch.channels_last) and \
                tgt.dtype == (torch.float32 if x2 else torch.bfloat16):
            need_ext().conv_wgrad(dy, x, w.shape[2], w.shape[3], stride, pad, 0, tgt, x2=x2)
        else:
            dw = need_ext().conv_wgrad(dy, x, w.shape[2], w.shape[3], stride, pad, x2=x2)
        if has_bias and need_b:
            db = _bias_grad(dy, w, bparam)
    elif need_w or (has_bias and need_b):
        assert not x2, 'fp32 (x2) mode: no MFMA weight gradient for this conv shape'
        _, dw, db = torch.ops.aten.convolution_backward(
            dy, x, w, [w.shape[0]] if has_bias else None, [stride] * 2, [pad] * 2, [1, 1], False,
            [0, 0], 1, [False, bool(need_w), bool(has_bias and need_b)])
    return dw, db


class _ConvIgemm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, relu):
        ext = need_ext()
        x = x.contiguous(memory_format=torch.channels_last)
        if precision.x2_enabled():  # x: a pair, w: the fp32 parameter (its pair from the store)
            wc = w
            wh, wpl = precision.weight_pair(w)
            y = ext.conv_igemm_fwd(x, wh, b, stride, pad, relu, x2=precision.x2_enabled(), w_plane=wpl)[0]
        else:
            wc = w.contiguous(memory_format=torch.channels_last)
            y = ext.conv_igemm_fwd(x, wc, b, stride, pad, relu)[0]
        ctx.save_for_backward(x, wc, y if relu else None)
        ctx.param = w if w.is_leaf else None
        ctx.bparam = b if (b is not None and b.is_leaf) else None
        ctx.stride, ctx.pad, ctx.relu, ctx.has_bias = stride, pad, relu, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        if ctx.relu and precision.x2_enabled():
            # the hi plane carries the sign (hi = RNE(v)): mask every plane by it
            m = precision.hi_plane(y) > 0
            dy = dy * torch.cat([m] * precision.nplanes(), 0)
        elif ctx.relu:
            dy = dy * (y > 0)
        dx, dw, db = conv_backward(x, w, ctx.param, dy, ctx.stride, ctx.pad, ctx.has_bias, ctx.needs_input_grad[0],
                                   ctx.needs_input_grad[1], ctx.needs_input_grad[2], ctx.bparam)
        return dx, dw, db, None, None, None


def weight_ok(x, w):
    """The filter dtype the MFMA path takes with activation ``x``: the activation dtype, or in the
    fp32 (x2) mode the fp32 parameter (whose pair the store keeps)."""
    if precision.x2_enabled():
        return x.dtype == torch.bfloat16 and w.dtype == torch.float32
    return w.dtype == x.dtype


def igemm_eligible(x, w, stride=1, pad=0):
    """True when the MFMA implicit-GEMM kernel is the path conv2d would take for this conv."""
    k = w.shape[2]
    if not (x.is_cuda and x.dtype in LOWP and weight_ok(x, w) and x.shape[1] % 64 == 0 and
            x.is_contiguous(memory_format=torch.channels_last) and (igemm_enabled() or precision.x2_enabled())):
        return False
    if k == 1 and pad == 0 and stride != 1:
        return False
    return True


def conv2d(x, w, b=None, stride=1, pad=0, relu=False):
    """Conv (+bias, +optional fused ReLU) on NCHW-logical / channels_last tensors."""
    k = w.shape[2]
    if (x.is_cuda and x.dtype in LOWP and weight_ok(x, w) and x.shape[1] % 64 == 0 and
            x.is_contiguous(memory_format=torch.channels_last)):
        if k == 1 and pad == 0 and stride != 1:
            x = x[:, :, ::stride, ::stride].contiguous(memory_format=torch.channels_last)
            stride = 1
        if igemm_enabled() or precision.x2_enabled():
            return _ConvIgemm.apply(x, w, b, int(stride), int(pad), bool(relu))
    assert not precision.x2_enabled(), 'fp32 (x2) mode: conv shape without an MFMA path'
    y = F.conv2d(x, w, b, stride=stride, padding=pad)
    return F.relu(y, inplace=True) if relu else y
