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


# ---- fused SGD (core/params.py FlatParamStore.enable_fused_sgd) --------------------------------
# A parameter may carry a spec for an update fused into its weight-gradient kernel (the VGG16 FC
# weights: ops/vgg_fused.py).  Producers use it only inside an active scope (Trainer step bodies);
# they mark it applied, and the store's SGD then skips that parameter's range for the step.
_SCOPE = [False]


class fused_sgd_scope:
    def __init__(self, on):
        self.on = bool(on)

    def __enter__(self):
        self.prev = _SCOPE[0]
        _SCOPE[0] = self.on
        return self

    def __exit__(self, *exc):
        _SCOPE[0] = self.prev
        return False


def set_fused_sgd(param, spec):
    if spec is None:
        param.__dict__.pop('_mxr_fsgd', None)
    else:
        param.__dict__['_mxr_fsgd'] = spec


def fused_sgd(param):
    """The fused-update spec of ``param`` when the current step may apply it, else None."""
    if param is None or not _SCOPE[0]:
        return None
    return param.__dict__.get('_mxr_fsgd')

