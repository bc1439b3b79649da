"""MI355X-native Faster R-CNN (mx-rcnn capabilities on PyTorch-ROCm + gfx950 HIP kernels).

Importing the package sets the HIP runtime defaults the training step is tuned for; they are
read when the HIP runtime initialises (the first GPU call), so the package must be imported
before anything touches the GPU -- every entry point here does.  A value already in the
environment wins.

* ``DEBUG_HIP_FORCE_GRAPH_QUEUES=2`` (a HIP runtime debug variable; ``MXR_GRAPH_QUEUES`` picks the
  value, 0 leaves the runtime default, and a warning says when the import came too late for it
  to act): a replayed hipGraph's independent branches are spread over
  two hardware queues instead of the runtime's default four.  The step's concurrency is two-way
  (the compute stream plus one side stream at a time: anchor targets / RPN losses / proposal
  chain / dgrad filter cache), and every extra queue adds cross-queue dependency waits.
  Measured on the ResNet-101 e2e step (bench.py, same box, interleaved): 1 queue 157.2,
  2 queues 159.7, 3 queues 150.8, default 151.5 img/s (docs/DESIGN.md §2); round 4
  (profiles/r4_ab_defaults.txt): fp32 77.4 with 2 vs 75.9 / 75.9 / 75.7 with the default / 1 / 3,
  bf16 160.3 vs 151.4 / 159.4.
"""
import os
import sys
import warnings

# MXR_GRAPH_QUEUES=n picks the queue count (0: leave the runtime's default and its variable alone)
_GQ = os.environ.get('MXR_GRAPH_QUEUES', '2')
RUNTIME_DEFAULTS = {'DEBUG_HIP_FORCE_GRAPH_QUEUES': _GQ} if _GQ not in ('', '0') else {}


def runtime_settings():
    """The HIP runtime variables in effect (recorded with benchmark results)."""
    return {k: os.environ.get(k) for k in ('DEBUG_HIP_FORCE_GRAPH_QUEUES', 'GPU_MAX_HW_QUEUES')}


for _k, _v in RUNTIME_DEFAULTS.items():
    if _k not in os.environ:
        os.environ[_k] = _v
        # the runtime reads it once, when it initialises: imported after the first GPU call, the
        # setting silently does nothing -- say so
        _tc = sys.modules.get('torch')
        if _tc is not None and getattr(getattr(_tc, 'cuda', None), 'is_initialized', lambda: False)():
            warnings.warn('mx_rcnn_amd imported after the HIP runtime initialised: %s=%s has no effect in '
                          'this process (import the package first)' % (_k, _v), RuntimeWarning)
