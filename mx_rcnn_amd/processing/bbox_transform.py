"""Box encode / decode / clip (reference: `helper/processing/bbox_transform.py:8-111`)."""
import numpy as np


def bbox_transform(ex_rois, gt_rois):
    """Regression targets (dx, dy, dw, dh) from ``ex_rois`` to ``gt_rois`` (N,4)."""
    ex_w = ex_rois[:, 2] - ex_rois[:, 0] + 1.0
    ex_h = ex_rois[:, 3] - ex_rois[:, 1] + 1.0
    ex_cx = ex_rois[:, 0] + 0.5 * (ex_w - 1.0)
    ex_cy = ex_rois[:, 1] + 0.5 * (ex_h - 1.0)
    gt_w = gt_rois[:, 2] - gt_rois[:, 0] + 1.0
    gt_h = gt_rois[:, 3] - gt_rois[:, 1] + 1.0
    gt_cx = gt_rois[:, 0] + 0.5 * (gt_w - 1.0)
    gt_cy = gt_rois[:, 1] + 0.5 * (gt_h - 1.0)
    dx = (gt_cx - ex_cx) / (ex_w + 1e-14)
    dy = (gt_cy - ex_cy) / (ex_h + 1e-14)
    dw = np.log(gt_w / ex_w)
    dh = np.log(gt_h / ex_h)
    return np.vstack((dx, dy, dw, dh)).transpose()


def bbox_pred(boxes, box_deltas, is_train=False):
    """Apply (N, 4C) deltas to (N, 4) boxes; ``is_train`` clamps like the reference (unused there)."""
    if boxes.shape[0] == 0:
        return np.zeros((0, box_deltas.shape[1]))
    boxes = boxes.astype(np.float64, copy=False)
    widths = boxes[:, 2] - boxes[:, 0] + 1.0
    heights = boxes[:, 3] - boxes[:, 1] + 1.0
    ctr_x = boxes[:, 0] + 0.5 * (widths - 1.0)
    ctr_y = boxes[:, 1] + 0.5 * (heights - 1.0)
    dx = box_deltas[:, 0::4]
    dy = box_deltas[:, 1::4]
    dw = box_deltas[:, 2::4]
    dh = box_deltas[:, 3::4]
    if is_train:
        dx = np.clip(dx, -10, 10)
        dy = np.clip(dy, -10, 10)
        dw = np.clip(dw, -8, 8)
        dh = np.clip(dh, -8, 8)
    pcx = dx * widths[:, None] + ctr_x[:, None]
    pcy = dy * heights[:, None] + ctr_y[:, None]
    pw = np.exp(dw) * widths[:, None]
    ph = np.exp(dh) * heights[:, None]
    out = np.zeros(box_deltas.shape)
    out[:, 0::4] = pcx - 0.5 * (pw - 1.0)
    out[:, 1::4] = pcy - 0.5 * (ph - 1.0)
    out[:, 2::4] = pcx + 0.5 * (pw - 1.0)
    out[:, 3::4] = pcy + 0.5 * (ph - 1.0)
    return out


def clip_boxes(boxes, im_shape):
    """Clamp x to [0, W-1] and y to [0, H-1] for every class slot (in place)."""
    boxes[:, 0::4] = np.maximum(np.minimum(boxes[:, 0::4], im_shape[1] - 1), 0)
    boxes[:, 1::4] = np.maximum(np.minimum(boxes[:, 1::4], im_shape[0] - 1), 0)
    boxes[:, 2::4] = np.maximum(np.minimum(boxes[:, 2::4], im_shape[1] - 1), 0)
    boxes[:, 3::4] = np.maximum(np.minimum(boxes[:, 3::4], im_shape[0] - 1), 0)
    return boxes


def clip_pad(boxes, pad_shape):
    """Crop an (n, c, H, W) map to (h, w)."""
    H, W = boxes.shape[2:]
    h, w = pad_shape
    if h < H:
        boxes = boxes[:, :, :h, :].copy()
    if w < W:
        boxes = boxes[:, :, :, :w].copy()
    return boxes
