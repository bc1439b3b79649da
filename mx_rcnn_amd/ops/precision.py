"""fp32-class training on the bf16 MFMA ("x2" pairs).

The reference trains in fp32 end to end (MXNet's default dtype; SGD in `train_end2end.py:98-105`).
MI355X's matrix cores run fp32 at 1/16 of the bf16 rate, so the fp32 mode keeps every MFMA
operand as a PAIR of bf16 values, v = hi + lo with hi = RNE(v) and lo = RNE(v - hi): 16
significant bits (relative error <= 2^-17, finer than the TF32 inputs cuDNN uses for "fp32"
convolutions), and every product is computed as hi*hi + hi*lo + lo*hi on the bf16 MFMA with fp32
accumulation (the dropped lo*lo term is below 2^-16 relative).  Accumulators, BN statistics,
losses, gradients of parameters, SGD state and master weights are fp32.

Representation (csrc/hip/common.h): an activation / gradient pair is ONE bf16 tensor of shape
(2N, C, H, W) (or (2M, K)), the hi plane first, the lo plane N*C*H*W elements further.  A weight
keeps its fp32 master as the module Parameter; its pair lives in the flat parameter store's
shadow buffer (hi plane, lo plane one group further, rewritten by the SGD kernel) or in a cache
built here for parameters outside a store.  The mode is a process-wide switch (`x2_mode`) that
the trainer holds around forward + backward; inside it, every bf16 tensor reaching an op is a
pair.
"""
import contextlib

import torch

_STATE = {'on': False}


def x2_enabled():
    return _STATE['on']


@contextlib.contextmanager
def x2_mode(on=True):
    prev = _STATE['on']
    _STATE['on'] = bool(on)
    try:
        yield
    finally:
        _STATE['on'] = prev


def is_pair(t):
    """True for a pair tensor of the x2 mode (bf16 inside the mode)."""
    return _STATE['on'] and torch.is_tensor(t) and t.dtype == torch.bfloat16


def split(t):
    """fp32 tensor (N, ...) -> pair (2N, ...) bf16 in t's memory format (hi plane first)."""
    t = t.float()
    hi = t.to(torch.bfloat16)
    lo = (t - hi.float()).to(torch.bfloat16)
    fmt = torch.channels_last if (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)
                                  and not t.is_contiguous()) else torch.contiguous_format
    return torch.cat([hi, lo], 0).contiguous(memory_format=fmt)


def join(p):
    """pair (2N, ...) -> fp32 (N, ...) (hi + lo)."""
    n = p.shape[0] // 2
    return p[:n].float() + p[n:].float()


def plane(p):
    """Elements between a pair's hi and lo planes."""
    return p.numel() // 2


# weight pairs: id(param) -> (param, hi view, plane)
_WEIGHTS = {}
_CACHE = {}


def register_weight(param, hi_view, w_plane):
    """The store's shadow pair of ``param``: ``hi_view`` shaped like the filter the kernels read
    (channels_last conv filter / (out, in) matrix), its lo plane ``w_plane`` elements further."""
    _WEIGHTS[id(param)] = (param, hi_view, int(w_plane))


def clear_weights():
    _WEIGHTS.clear()
    _CACHE.clear()


def weight_pair(w):
    """-> (hi view, plane) of weight ``w`` (an fp32 Parameter / tensor).  Store-managed weights
    use the SGD-maintained shadow; anything else gets a cached pair rebuilt when the tensor's
    version counter moves."""
    ent = _WEIGHTS.get(id(w))
    if ent is not None and ent[0] is w:
        return ent[1], ent[2]
    key = id(w)
    ver = (w.data_ptr(), w._version, tuple(w.shape))
    hit = _CACHE.get(key)
    if hit is None or hit[0] != ver or hit[1] is not w:
        fmt = torch.channels_last if w.dim() == 4 else torch.contiguous_format
        wf = w.detach().float().contiguous(memory_format=fmt)
        pr = split(wf) if w.dim() == 4 else split(wf)
        n = w.shape[0]
        hit = (ver, w, pr[:n], pr.numel() // 2, pr)
        _CACHE[key] = hit
    return hit[2], hit[3]
