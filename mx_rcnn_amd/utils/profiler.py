"""Per-stage step profiler (SURVEY §5.1 plan): named ranges around the stages of a training
step (trunk, rpn, anchor_target, proposal, proposal_target, roi_pool, head, losses, backward,
allreduce, sgd).  Each range is (a) a roctx range, so ``rocprofv3 --marker-trace`` timelines
show the stages, and (b) a pair of HIP events whose elapsed times are averaged per stage and
reported by the Speedometer.  Enabled with ``MXR_PROFILE=1`` or ``enable()``; disabled ranges
cost one attribute check.  Events cannot live inside a captured hipGraph, so a profiled run
executes eagerly (``MutableModule`` / ``bench.py --mode eager``).
"""
import contextlib
import os
from collections import OrderedDict

import torch

_STATE = {'enabled': os.environ.get('MXR_PROFILE', '0') == '1', 'pending': [], 'acc': OrderedDict()}


def enable(flag=True):
    _STATE['enabled'] = bool(flag)


def enabled():
    return _STATE['enabled']


def _roctx_push(name):
    try:
        torch.cuda.nvtx.range_push(name)  # roctx on ROCm builds
        return True
    except Exception:
        return False


@contextlib.contextmanager
def range(name):  # noqa: A001 - mirrors the profiler vocabulary
    if not _STATE['enabled'] or not torch.cuda.is_available() or torch.cuda.is_current_stream_capturing():
        yield
        return
    pushed = _roctx_push(name)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    try:
        yield
    finally:
        e.record()
        _STATE['pending'].append((name, s, e))
        if pushed:
            torch.cuda.nvtx.range_pop()


def collect():
    """Synchronise once and fold pending event pairs into the per-stage totals."""
    if not _STATE['pending']:
        return
    torch.cuda.synchronize()
    for name, s, e in _STATE['pending']:
        tot, n = _STATE['acc'].get(name, (0.0, 0))
        _STATE['acc'][name] = (tot + s.elapsed_time(e), n + 1)
    _STATE['pending'] = []


def report(reset=True):
    """-> OrderedDict stage -> mean ms per occurrence."""
    collect()
    out = OrderedDict((k, tot / max(n, 1)) for k, (tot, n) in _STATE['acc'].items())
    if reset:
        _STATE['acc'] = OrderedDict()
    return out


def format_report(rep):
    return ' '.join('%s=%.2fms' % (k, v) for k, v in rep.items())
