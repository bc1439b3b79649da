"""Loader for the in-tree gfx950 extension (``mx_rcnn_amd/_C*.so``).

Dispatch rule used by every op in this package: a GPU tensor MUST run the HIP kernel
(``need_ext`` raises loudly if the extension is missing -- no silent eager fallback on a
GPU box); a CPU tensor runs the PyTorch reference implementation, which is also the
numerics oracle in tests.
"""
import importlib
import importlib.util
import os

_EXT = None
_ERR = None


def _load():
    global _EXT, _ERR
    if _EXT is not None or _ERR is not None:
        return _EXT
    try:
        import torch  # noqa: F401  (loads libc10_hip / libamdhip64 first)
        path = os.environ.get('MXR_EXT_PATH')  # A/B of two builds on one box (scripts/gpu_ab_prof.sh)
        if path:
            spec = importlib.util.spec_from_file_location('mx_rcnn_amd._C', path)
            _EXT = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_EXT)
        else:
            _EXT = importlib.import_module('mx_rcnn_amd._C')
    except ImportError as e:  # pragma: no cover - depends on build state
        _ERR = e
    if _EXT is not None:
        from . import tune_plan  # the shipped / user conv plans, before the first conv
        tune_plan.ensure_loaded(_EXT)
    return _EXT


def ext_available():
    return _load() is not None


class _SyncProxy(object):
    """RCNN_SYNC=1 (the reference's NaiveEngine debug mode): every kernel launcher
    is followed by a device synchronisation, so an asynchronous fault is reported at the op
    that caused it (with its name) instead of at some later API call."""

    def __init__(self, ext):
        self._ext = ext

    def __getattr__(self, name):
        fn = getattr(self._ext, name)
        if not callable(fn):
            return fn

        def wrapped(*a, **k):
            import torch
            out = fn(*a, **k)
            if torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
                try:
                    torch.cuda.synchronize()
                except Exception as e:  # pragma: no cover - only on a faulting kernel
                    raise RuntimeError('RCNN_SYNC: kernel %s failed: %s' % (name, e)) from e
            return out
        return wrapped


def need_ext():
    ext = _load()
    if ext is None:
        raise RuntimeError(
            'mx_rcnn_amd HIP extension is not built (%s). Run `python -m mx_rcnn_amd.csrc.build` '
            '(hipcc --offload-arch=gfx950) before using GPU tensors.' % _ERR)
    if sync_debug():
        return _SyncProxy(ext)
    return ext


def on_gpu(t):
    return t.is_cuda


def sync_debug():
    """RCNN_SYNC=1: synchronise + check after every custom kernel."""
    return os.environ.get('RCNN_SYNC', '0') == '1'


def check_sync(name):
    if sync_debug():
        import torch
        torch.cuda.synchronize()
        err = torch.cuda.current_stream()  # touching the stream surfaces async errors
        del err


_CONSTS = {}


_UNIT = {}


def unit_grad(device):
    """The cached 0-d fp32 one that seeds a backward pass (``loss.backward(unit_grad(dev))``).  The
    loss ops recognise it by identity and hand back their stored gradients unscaled -- no ones
    fill for the seed and no scale-by-1 kernel per loss term.  Never written in place."""
    import torch
    key = str(device)
    t = _UNIT.get(key)
    if t is None:
        t = torch.ones((), dtype=torch.float32, device=device)
        _UNIT[key] = t
    return t


def is_unit_grad(g):
    if os.environ.get('MXR_UNIT_SEED', '1') == '0':
        return False
    t = _UNIT.get(str(g.device))
    return t is not None and g is t


def const_tensor(values, device, dtype=None):
    """Cached small constant tensor on ``device`` (built once, outside any hipGraph capture:
    creating it from host data inside a capture would be a forbidden synchronous copy)."""
    import torch
    dtype = dtype or torch.float32
    key = (tuple(float(v) for v in values), str(device), dtype)
    t = _CONSTS.get(key)
    if t is None:
        t = torch.tensor([float(v) for v in values], dtype=dtype, device=device)
        _CONSTS[key] = t
    return t
