"""Direct gradient delivery into the flat gradient buffers (core/params.py).

Parameters managed by the FlatParamStore carry a pre-set ``.grad`` that is a view of a flat
buffer.  Kernels that produce a parameter gradient (MFMA conv wgrad, fused BN backward) can
ACCUMULATE straight into that view and return ``None`` to autograd, which removes one
AccumulateGrad ``add`` kernel per parameter per step (~300 launches on ResNet-101).  The
engine still visits the parameter's AccumulateGrad node with an undefined gradient and runs
its post-accumulate hooks (verified on torch 2.10, tests/test_kernels.py
test_direct_grad_delivery), so the readiness hooks -- the bucketed all-reduce -- fire exactly
once per step either way; producers must NOT call ``delivered`` themselves.
"""
_ENABLED = set()
_HOOKS = {}


def enable_direct(param):
    _ENABLED.add(id(param))
    param.register_post_accumulate_grad_hook(lambda p: delivered(p))


def target(param):
    """The buffer to accumulate ``param``'s gradient into, or None (use autograd)."""
    if param is None or id(param) not in _ENABLED:
        return None
    g = param.grad
    return g if g is not None else None


def add_hook(param, fn):
    _HOOKS.setdefault(id(param), []).append(fn)


def clear_hooks():
    _HOOKS.clear()


def delivered(param):
    for fn in _HOOKS.get(id(param), ()):
        fn(param)
