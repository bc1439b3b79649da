"""Uniform draws for the sampling ops (csrc/hip/rng.hip).

The anchor / RoI subset keys and the proposal layer's random pad (`rcnn/rpn/proposal.py`,
`rcnn/rpn/proposal_target.py`, `rcnn/minibatch.py` use numpy.random) are drawn on the device
from the default generator's graph-safe Philox state -- the same state torch.rand advances, so a
replayed hipGraph draws fresh numbers every step -- by our Philox kernel instead of a torch
distribution kernel.  An explicit ``generator`` (tests) or a CPU device takes torch.rand.
"""
import torch

from ._ext import need_ext


def uniform(shape, device, generator=None):
    """U[0, 1) float32 of ``shape`` on ``device``."""
    dev = torch.device(device)
    if generator is None and dev.type == 'cuda':
        return need_ext().philox_uniform_(torch.empty(shape, dtype=torch.float32, device=dev))
    return torch.rand(shape, device=dev, generator=generator)
