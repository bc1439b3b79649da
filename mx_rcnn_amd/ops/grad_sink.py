"""Direct gradient delivery into the flat gradient buffers (core/params.py).

Parameters managed by the FlatParamStore carry a pre-set ``.grad`` that is a view of a flat
buffer.  Kernels that produce a parameter gradient (MFMA conv wgrad, fused BN backward) can
ACCUMULATE straight into that view and return ``None`` to autograd, which removes one
AccumulateGrad ``add`` kernel per parameter per step (~300 launches on ResNet-101).  The
engine still visits the parameter's AccumulateGrad node with an undefined gradient and runs
its post-accumulate hooks (verified on torch 2.10, tests/test_kernels.py
test_direct_grad_delivery), so the readiness hooks -- the bucketed all-reduce -- fire exactly
once per step either way; producers must NOT call ``delivered`` themselves.

The registrations live ON the parameter (``_mxr_direct`` / ``_mxr_hooks`` attributes), not in
module-level ``id()``-keyed tables: a dead trainer's parameters, stores and reducers are freed with
their model instead of being pinned by a registry, and a later parameter that happens to reuse an
``id`` inherits nothing.
"""


def enable_direct(param):
    if param.__dict__.get('_mxr_direct'):
        return
    param.__dict__['_mxr_direct'] = True
    param.register_post_accumulate_grad_hook(delivered)


def target(param):
    """The buffer to accumulate ``param``'s gradient into, or None (use autograd)."""
    if param is None or not param.__dict__.get('_mxr_direct'):
        return None
    return param.grad


def add_hook(param, fn):
    param.__dict__.setdefault('_mxr_hooks', []).append(fn)


def clear_hooks(params):
    """Drop the readiness hooks of ``params`` (a reducer replacing an earlier one on the same
    parameters calls this first, so a dead reducer is never driven again)."""
    for p in params:
        p.__dict__.pop('_mxr_hooks', None)


def delivered(param):
    for fn in param.__dict__.get('_mxr_hooks', ()):
        fn(param)
