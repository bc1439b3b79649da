"""Base anchor enumeration (reference: `helper/processing/generate_anchor.py:8-72`).

Ratio-major / scale-minor order, ``+1`` pixel convention.  The golden tables
for A=9 (VGG) and A=12 (ResNet) are pinned in tests/test_geometry.py.
"""
import numpy as np


def _whctrs(anchor):
    w = anchor[2] - anchor[0] + 1
    h = anchor[3] - anchor[1] + 1
    return w, h, anchor[0] + 0.5 * (w - 1), anchor[1] + 0.5 * (h - 1)


def _mkanchors(ws, hs, x_ctr, y_ctr):
    ws = np.asarray(ws, dtype=np.float64)[:, None]
    hs = np.asarray(hs, dtype=np.float64)[:, None]
    return np.hstack((x_ctr - 0.5 * (ws - 1), y_ctr - 0.5 * (hs - 1),
                      x_ctr + 0.5 * (ws - 1), y_ctr + 0.5 * (hs - 1)))


def _ratio_enum(anchor, ratios):
    w, h, x_ctr, y_ctr = _whctrs(anchor)
    size_ratios = (w * h) / np.asarray(ratios, dtype=np.float64)
    ws = np.round(np.sqrt(size_ratios))
    hs = np.round(ws * np.asarray(ratios, dtype=np.float64))
    return _mkanchors(ws, hs, x_ctr, y_ctr)


def _scale_enum(anchor, scales):
    w, h, x_ctr, y_ctr = _whctrs(anchor)
    scales = np.asarray(scales, dtype=np.float64)
    return _mkanchors(w * scales, h * scales, x_ctr, y_ctr)


def generate_anchors(base_size=16, ratios=(0.5, 1, 2), scales=2 ** np.arange(3, 6)):
    """(A, 4) float64 anchors around the (0, 0, base-1, base-1) window."""
    base_anchor = np.array([1, 1, base_size, base_size], dtype=np.float64) - 1
    ratio_anchors = _ratio_enum(base_anchor, ratios)
    return np.vstack([_scale_enum(ratio_anchors[i, :], scales)
                      for i in range(ratio_anchors.shape[0])])


def shifted_anchors(feat_h, feat_w, feat_stride=16, scales=(8, 16, 32), ratios=(0.5, 1, 2)):
    """All anchors of a feature map, index ``(h*W + w)*A + a`` (proposal.py:77-91)."""
    base = generate_anchors(base_size=feat_stride, ratios=list(ratios), scales=np.array(scales))
    shift_x = np.arange(0, feat_w) * feat_stride
    shift_y = np.arange(0, feat_h) * feat_stride
    sx, sy = np.meshgrid(shift_x, shift_y)
    shifts = np.vstack((sx.ravel(), sy.ravel(), sx.ravel(), sy.ravel())).transpose()
    A, K = base.shape[0], shifts.shape[0]
    return (base.reshape((1, A, 4)) + shifts.reshape((1, K, 4)).transpose((1, 0, 2))).reshape((K * A, 4))
