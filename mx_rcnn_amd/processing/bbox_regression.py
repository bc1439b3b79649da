"""IoU + offline regression targets (reference: `helper/processing/bbox_regression.py:11-85`).

``bbox_overlaps`` is a chunked, vectorised replacement for the reference's
pure-Python double loop (its worst CPU hot spot); the values are identical.
"""
import numpy as np

from ..config import config
from .bbox_transform import bbox_transform


def bbox_overlaps(boxes, query_boxes, chunk=1 << 22):
    """(n, k) IoU with ``+1`` areas; 0 where the boxes do not intersect."""
    boxes = np.asarray(boxes, dtype=np.float64)
    query_boxes = np.asarray(query_boxes, dtype=np.float64)
    n, k = boxes.shape[0], query_boxes.shape[0]
    out = np.zeros((n, k), dtype=np.float64)
    if n == 0 or k == 0:
        return out
    q_area = (query_boxes[:, 2] - query_boxes[:, 0] + 1) * (query_boxes[:, 3] - query_boxes[:, 1] + 1)
    step = max(1, chunk // max(k, 1))
    for s in range(0, n, step):
        b = boxes[s:s + step]
        iw = np.minimum(b[:, None, 2], query_boxes[None, :, 2]) - np.maximum(b[:, None, 0], query_boxes[None, :, 0]) + 1
        ih = np.minimum(b[:, None, 3], query_boxes[None, :, 3]) - np.maximum(b[:, None, 1], query_boxes[None, :, 1]) + 1
        valid = (iw > 0) & (ih > 0)
        inter = np.where(valid, iw * ih, 0.0)
        b_area = (b[:, 2] - b[:, 0] + 1) * (b[:, 3] - b[:, 1] + 1)
        union = b_area[:, None] + q_area[None, :] - inter
        with np.errstate(divide='ignore', invalid='ignore'):
            out[s:s + step] = np.where(valid, inter / union, 0.0)
    return out


def compute_bbox_regression_targets(rois, overlaps, labels):
    """Per roidb entry: ``[cls, dx, dy, dw, dh]`` for rois with overlap >= BBOX_REGRESSION_THRESH."""
    rois = rois.astype(np.float64, copy=False)
    gt_inds = np.where(overlaps == 1)[0]
    ex_inds = np.where(overlaps >= config.TRAIN.BBOX_REGRESSION_THRESH)[0]
    targets = np.zeros((rois.shape[0], 5), dtype=np.float32)
    if len(gt_inds) == 0 or len(ex_inds) == 0:
        return targets
    ex_gt = bbox_overlaps(rois[ex_inds, :], rois[gt_inds, :])
    gt_assignment = ex_gt.argmax(axis=1)
    targets[ex_inds, 0] = labels[ex_inds]
    targets[ex_inds, 1:] = bbox_transform(rois[ex_inds, :], rois[gt_inds[gt_assignment], :])
    return targets


def expand_bbox_regression_targets(bbox_targets_data, num_classes):
    """(k, 5) -> (k, 4C) targets + inside weights, non-zero only in the assigned class slot."""
    classes = bbox_targets_data[:, 0].astype(np.int64)
    k = classes.size
    bbox_targets = np.zeros((k, 4 * num_classes), dtype=np.float32)
    inside = np.zeros_like(bbox_targets)
    idx = np.where(classes > 0)[0]
    if idx.size:
        cols = 4 * classes[idx][:, None] + np.arange(4)[None, :]
        bbox_targets[idx[:, None], cols] = bbox_targets_data[idx, 1:]
        inside[idx[:, None], cols] = np.asarray(config.TRAIN.BBOX_INSIDE_WEIGHTS, dtype=np.float32)
    return bbox_targets, inside
