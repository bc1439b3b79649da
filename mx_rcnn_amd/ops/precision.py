"""fp32 training on the bf16 matrix cores: multi-plane operands.

The reference trains in IEEE fp32 end to end (MXNet's default dtype; SGD in
`train_end2end.py:98-105`).  MI355X's matrix cores run fp32 at 1/16 of the bf16 rate, so the
fp32 modes keep every MFMA operand as bf16 PLANES and compute products on the bf16 MFMA with fp32
accumulation:

* ``fp32`` (x3, three planes): v = hi + mid + lo with hi = RNE(v), mid = RNE(v - hi),
  lo = RNE(v - hi - mid).  The split is EXACT (hi + mid + lo == v: 24 significant bits, the
  IEEE fp32 value itself is what is stored between kernels) and a product is the six terms
  hh + hm + mh + hl + lh + mm; the dropped ml + lm + ll are below 2^-23 relative, the size of
  one fp32 rounding.  Memory order of the planes: (mid, hi, lo) -- csrc/hip/common.h explains
  why (the MFMA kernels run x3 as their pair loop twice with a uniform one-plane shift).
* ``bf16x3`` (x2, two planes): v ~ hi + lo with hi = RNE(v), lo = RNE(v - hi): 16 significant
  bits (relative error <= 2^-17), products hi*hi + hi*lo + lo*hi -- three bf16 MFMAs.  Faster,
  below fp32 precision.

Accumulators, BN statistics, losses, parameter gradients, SGD state and master weights are fp32
in both.

Representation (csrc/hip/common.h): an activation / gradient is ONE bf16 tensor of shape
(P*N, C, H, W) (or (P*M, K)), P = 2 or 3 planes, each plane N*C*H*W elements after the previous.
A weight keeps its fp32 master as the module Parameter; its planes live in the flat parameter
store's shadow buffer (one plane spacing per group, rewritten by the SGD kernel) or in a cache
built here for parameters outside a store.  The mode is a process-wide switch (`x2_mode`, the
plane count) that the trainer holds around forward + backward; inside it, every bf16 tensor
reaching an op is a multi-plane tensor.
"""
import contextlib
import weakref

import torch

_STATE = {'planes': 0}

# precision names of the training entry points -> plane count of the mode (0: plain bf16 operands)
PLANES = {'fp32': 3, 'bf16x3': 2, 'bf16': 0}


_DEFAULT = {'name': 'fp32'}


def set_default(name):
    """Training precision the entry points use when none is named (the CLIs' --dtype)."""
    if name not in PLANES:
        raise ValueError('precision must be one of %s, not %r' % (sorted(PLANES), name))
    _DEFAULT['name'] = name


def default_name():
    return _DEFAULT['name']


_DET = {'on': __import__('os').environ.get('MXR_NONDETERMINISTIC', '0') == '0'}


def set_deterministic(on=True):
    """Bitwise-reproducible gradients (default on; MXR_NONDETERMINISTIC=1 turns it off): the
    frozen-BN gamma / beta column sums of the conv epilogues go to per-tile partial rows folded in
    a fixed order (ConvEpi::bnb_part + bnb_part_fold) instead of fp32 atomics.  The RoI-pool and
    BN-ReLU backward reductions are order-fixed unconditionally."""
    _DET['on'] = bool(on)


def deterministic():
    return _DET['on']


def x2_enabled():
    """Plane count of the active multi-plane mode (2: bf16x3, 3: fp32), 0 when off."""
    return _STATE['planes']


nplanes = x2_enabled


def x3_enabled():
    return _STATE['planes'] == 3


@contextlib.contextmanager
def x2_mode(on=True):
    """Run a block in a multi-plane mode: ``on`` is the plane count (2 or 3; True means 2), or
    False / 0 for off."""
    prev = _STATE['planes']
    _STATE['planes'] = 0 if not on else (3 if on == 3 else 2)
    try:
        yield
    finally:
        _STATE['planes'] = prev


def is_pair(t):
    """The plane count when ``t`` is a multi-plane tensor of the active mode (bf16 inside it), else 0."""
    p = _STATE['planes']
    return p if (p and torch.is_tensor(t) and t.dtype == torch.bfloat16) else 0


def split(t, planes=None):
    """fp32 tensor (N, ...) -> (P*N, ...) bf16 planes in t's memory format: (hi, lo) for P = 2,
    (mid, hi, lo) for P = 3."""
    p = planes or _STATE['planes'] or 2
    t = t.float()
    hi = t.to(torch.bfloat16)
    r = t - hi.float()
    if p == 3:
        mid = r.to(torch.bfloat16)
        lo = (r - mid.float()).to(torch.bfloat16)
        parts = [mid, hi, lo]
    else:
        parts = [hi, r.to(torch.bfloat16)]
    fmt = torch.channels_last if (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)
                                  and not t.is_contiguous()) else torch.contiguous_format
    return torch.cat(parts, 0).contiguous(memory_format=fmt)


def join(p, planes=None):
    """(P*N, ...) planes -> fp32 (N, ...) (their exact sum)."""
    k = planes or _STATE['planes'] or 2
    n = p.shape[0] // k
    out = p[:n].float() + p[n:2 * n].float()
    if k == 3:
        out = out + p[2 * n:].float()
    return out


def plane(p, planes=None):
    """Elements between consecutive planes of ``p``."""
    return p.numel() // (planes or _STATE['planes'] or 2)


def logical(n, planes=None):
    """Logical leading size of a (P*n, ...) multi-plane tensor (n itself when the mode is off)."""
    k = _STATE['planes'] if planes is None else planes
    return n // k if k else n


def hi_plane(p, planes=None):
    """View of the hi plane (the one carrying the sign): plane 0 of a pair, plane 1 of a triple."""
    k = planes or _STATE['planes'] or 2
    n = p.shape[0] // k
    return p[n:2 * n] if k == 3 else p[:n]


# weight planes: id(param) -> (weakref(param), plane-0 view, plane spacing, plane count); the
# entries (and the cached planes below) go away with their parameter, so a later trainer's store
# never sees an earlier one's shadows
_WEIGHTS = {}
_CACHE = {}


def _drop(key):
    _WEIGHTS.pop(key, None)
    _CACHE.pop(key, None)


def register_weight(param, base_view, w_plane, planes=2):
    """The store's shadow planes of ``param``: ``base_view`` (plane 0) shaped like the filter the
    kernels read (channels_last conv filter / (out, in) matrix), the next planes ``w_plane``
    elements further each."""
    key = id(param)
    if key not in _WEIGHTS and key not in _CACHE:
        weakref.finalize(param, _drop, key)
    _WEIGHTS[key] = (weakref.ref(param), base_view, int(w_plane), int(planes))


def clear_weights():
    _WEIGHTS.clear()
    _CACHE.clear()


def forget_weight(param):
    """Drop every cache derived from ``param``'s values (its data was rewritten through ``.data``,
    which does not move the version counter): the planes cached here, and -- through the reload
    epoch -- the per-tensor packings of other ops (ops/stem.py)."""
    _CACHE.pop(id(param), None)
    param.__dict__['_mxr_epoch'] = weight_epoch(param) + 1


def weight_epoch(param):
    """Reload counter of ``param`` (bumped by forget_weight); part of every derived cache's key."""
    return param.__dict__.get('_mxr_epoch', 0)


# Training generation: the SGD kernels rewrite trainable parameters in place (inside a replayed
# hipGraph, or through the flat store), which moves neither their version counters nor their
# reload epochs.  Every step bumps this counter (core/trainer.py), and the inference-time caches
# derived from TRAINABLE parameters (the stem's packed filter, the GEMM route's BN-folded filter)
# key on it, so evaluating between training steps never reads a stale fold.
_GEN = [0]


def bump_generation():
    _GEN[0] += 1


def train_generation(*params):
    """The training generation if any of ``params`` is trainable, else 0 (frozen values change
    only through loads, which bump their reload epochs)."""
    return _GEN[0] if any(p is not None and p.requires_grad for p in params) else 0


def weight_pair(w):
    """-> (plane-0 view, plane spacing) of weight ``w`` (an fp32 Parameter / tensor) in the active
    mode.  Store-managed weights use the SGD-maintained shadow; anything else gets cached planes
    rebuilt when the tensor's version counter moves."""
    p = _STATE['planes'] or 2
    ent = _WEIGHTS.get(id(w))
    if ent is not None and ent[0]() is w and ent[3] == p:
        return ent[1], ent[2]
    key = id(w)
    ver = (w.data_ptr(), w._version, tuple(w.shape), p, weight_epoch(w))
    hit = _CACHE.get(key)
    if hit is None or hit[0] != ver or hit[1]() is not w:
        fmt = torch.channels_last if w.dim() == 4 else torch.contiguous_format
        wf = w.detach().float().contiguous(memory_format=fmt)
        pr = split(wf, p)
        n = w.shape[0]
        if key not in _WEIGHTS and key not in _CACHE:
            weakref.finalize(w, _drop, key)
        hit = (ver, weakref.ref(w), pr[:n], pr.numel() // p, pr)
        _CACHE[key] = hit
    return hit[2], hit[3]
