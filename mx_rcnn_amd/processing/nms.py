"""Greedy NMS and nest filter, host reference (`helper/processing/nms.py:4-70`).

Suppression rule: drop j when IoU(i, j) > thresh (keep ``ovr <= thresh``).
Order is descending score with a deterministic tie rule (lower index first);
the reference's ``argsort()[::-1]`` leaves tie order unspecified.
"""
import numpy as np


def _order(scores):
    # stable descending: highest score first, ties by ascending index
    return np.lexsort((np.arange(scores.shape[0]), -scores))


def nms(dets, thresh):
    dets = np.asarray(dets)
    if dets.shape[0] == 0:
        return []
    x1, y1, x2, y2, scores = dets[:, 0], dets[:, 1], dets[:, 2], dets[:, 3], dets[:, 4]
    areas = (x2 - x1 + 1) * (y2 - y1 + 1)
    order = _order(scores)
    keep = []
    while order.size > 0:
        i = order[0]
        keep.append(int(i))
        xx1 = np.maximum(x1[i], x1[order[1:]])
        yy1 = np.maximum(y1[i], y1[order[1:]])
        xx2 = np.minimum(x2[i], x2[order[1:]])
        yy2 = np.minimum(y2[i], y2[order[1:]])
        w = np.maximum(0.0, xx2 - xx1 + 1)
        h = np.maximum(0.0, yy2 - yy1 + 1)
        inter = w * h
        ovr = inter / (areas[i] + areas[order[1:]] - inter)
        order = order[np.where(ovr <= thresh)[0] + 1]
    return keep


def nest(dets, thresh=0.90):
    """Drop box i if inter(i, j) / area_i > thresh for any other box j (vectorised O(N^2));
    a GPU tensor runs the HIP kernel (csrc/hip/det_post.hip)."""
    try:
        import torch
        if torch.is_tensor(dets) and dets.is_cuda:
            from ..ops._ext import need_ext
            keep = need_ext().nest_keep(dets.float().contiguous(), float(thresh))
            return [int(i) for i in torch.nonzero(keep).flatten().tolist()]
    except ImportError:  # pragma: no cover
        pass
    dets = np.asarray(dets)
    n = dets.shape[0]
    if n == 0:
        return []
    x1, y1, x2, y2 = dets[:, 0], dets[:, 1], dets[:, 2], dets[:, 3]
    areas = (x2 - x1 + 1) * (y2 - y1 + 1)
    w = np.maximum(0, np.minimum(x2[:, None], x2[None]) - np.maximum(x1[:, None], x1[None]) + 1)
    h = np.maximum(0, np.minimum(y2[:, None], y2[None]) - np.maximum(y1[:, None], y1[None]) + 1)
    ratio = (w * h) / areas[:, None]
    np.fill_diagonal(ratio, 0)
    return [int(i) for i in np.where(~(ratio > thresh).any(axis=1))[0]]
