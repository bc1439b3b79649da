"""MI355X-native Faster R-CNN (mx-rcnn capabilities on PyTorch-ROCm + gfx950 HIP kernels).

Importing the package sets the HIP runtime defaults the training step is tuned for; they are
read when the HIP runtime initialises (the first GPU call), so the package must be imported
before anything touches the GPU -- every entry point here does.  A value already in the
environment wins.

* ``DEBUG_HIP_FORCE_GRAPH_QUEUES=2``: a replayed hipGraph's independent branches are spread over
  two hardware queues instead of the runtime's default four.  The step's concurrency is two-way
  (the compute stream plus one side stream at a time: anchor targets / RPN losses / proposal
  chain / dgrad filter cache), and every extra queue adds cross-queue dependency waits.
  Measured on the ResNet-101 e2e step (bench.py, same box, interleaved): 1 queue 157.2,
  2 queues 159.7, 3 queues 150.8, default 151.5 img/s (docs/DESIGN.md §2).
"""
import os

RUNTIME_DEFAULTS = {
    'DEBUG_HIP_FORCE_GRAPH_QUEUES': '2',
}

for _k, _v in RUNTIME_DEFAULTS.items():
    os.environ.setdefault(_k, _v)
