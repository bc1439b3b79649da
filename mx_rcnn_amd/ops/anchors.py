"""Anchor tables on device (SURVEY §2.12 golden anchors; reference
`helper/processing/generate_anchor.py`).  Base anchors are computed once per
(stride, scales, ratios, device) with the reference's float64 arithmetic and cached."""
import numpy as np
import torch

from ..processing.generate_anchor import generate_anchors

_CACHE = {}


def base_anchors(feat_stride=16, scales=(8, 16, 32), ratios=(0.5, 1, 2), device='cpu'):
    key = (float(feat_stride), tuple(float(s) for s in scales), tuple(float(r) for r in ratios), str(device))
    t = _CACHE.get(key)
    if t is None:
        a = generate_anchors(base_size=feat_stride, ratios=list(ratios), scales=np.array(scales, dtype=np.float64))
        t = torch.tensor(a, dtype=torch.float32, device=device)
        _CACHE[key] = t
    return t


def all_anchors(H, W, feat_stride=16, scales=(8, 16, 32), ratios=(0.5, 1, 2), device='cpu'):
    """(H*W*A, 4) anchors, index (h*W + w)*A + a."""
    base = base_anchors(feat_stride, scales, ratios, device)
    sx = torch.arange(W, device=device, dtype=torch.float32) * feat_stride
    sy = torch.arange(H, device=device, dtype=torch.float32) * feat_stride
    yy, xx = torch.meshgrid(sy, sx, indexing='ij')
    shifts = torch.stack([xx, yy, xx, yy], dim=-1).reshape(-1, 1, 4)
    return (shifts + base[None]).reshape(-1, 4)
