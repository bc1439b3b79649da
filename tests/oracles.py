"""Independent numpy re-statements of the reference's detection ops, used as
test oracles.  Deterministic tie rule (score desc, index asc) replaces numpy's unstable sort."""
import numpy as np

from mx_rcnn_amd.processing.generate_anchor import generate_anchors
from mx_rcnn_amd.processing.bbox_transform import bbox_pred, clip_boxes, bbox_transform
from mx_rcnn_amd.processing.bbox_regression import bbox_overlaps
from mx_rcnn_amd.processing.nms import nms


def softmax2(bg, fg):
    m = np.maximum(bg, fg)
    eb, ef = np.exp(bg - m), np.exp(fg - m)
    return ef / (eb + ef)


def proposal_np(cls, dlt, im_info, stride, scales, ratios, pre, post, thresh, min_size, train):
    """Single image, cls logits (2A, H, W), dlt (4A, H, W) -> kept (n, 4) boxes, scores (in keep order)."""
    A = cls.shape[0] // 2
    H, W = cls.shape[1:]
    if train:
        H, W = min(H, int(im_info[0] / stride)), min(W, int(im_info[1] / stride))
    scores = softmax2(cls[:A, :H, :W], cls[A:, :H, :W]).transpose(1, 2, 0).reshape(-1)
    base = generate_anchors(stride, list(ratios), np.array(scales))
    sx, sy = np.meshgrid(np.arange(W) * stride, np.arange(H) * stride)
    shifts = np.vstack((sx.ravel(), sy.ravel(), sx.ravel(), sy.ravel())).T
    anchors = (base[None] + shifts[:, None]).reshape(-1, 4)
    d = dlt[:, :H, :W].transpose(1, 2, 0).reshape(-1, 4)
    p = clip_boxes(bbox_pred(anchors, d.astype(np.float64)), im_info[:2])
    ws = p[:, 2] - p[:, 0] + 1
    hs = p[:, 3] - p[:, 1] + 1
    keep = np.where((ws >= min_size * im_info[2]) & (hs >= min_size * im_info[2]))[0]
    p, scores = p[keep], scores[keep]
    order = np.lexsort((np.arange(scores.size), -scores))
    if pre > 0:
        order = order[:pre]
    p, scores = p[order], scores[order]
    k = nms(np.hstack([p, scores[:, None]]), thresh)
    if post > 0:
        k = k[:post]
    return p[k], scores[k]


def assign_anchor_labels_np(H, W, gt, im_info, stride=16, scales=(8, 16, 32), ratios=(0.5, 1, 2), border=0,
                            neg=0.3, pos=0.7):
    """Pre-sampling labels (H*W*A,) in (h, w, a) order and targets (H*W*A, 4) (rcnn/minibatch.py:258-316)."""
    base = generate_anchors(16, list(ratios), np.array(scales))
    A = base.shape[0]
    sx, sy = np.meshgrid(np.arange(W) * stride, np.arange(H) * stride)
    shifts = np.vstack((sx.ravel(), sy.ravel(), sx.ravel(), sy.ravel())).T
    all_a = (base[None] + shifts[:, None]).reshape(-1, 4)
    inside = np.where((all_a[:, 0] >= -border) & (all_a[:, 1] >= -border) &
                      (all_a[:, 2] < im_info[1] + border) & (all_a[:, 3] < im_info[0] + border))[0]
    anchors = all_a[inside]
    labels = np.full(len(inside), -1.0)
    targets = np.zeros((len(inside), 4))
    if gt.size > 0:
        ov = bbox_overlaps(anchors, gt[:, :4])
        am = ov.argmax(axis=1)
        mo = ov[np.arange(len(inside)), am]
        gam = ov.argmax(axis=0)
        gmax = ov[gam, np.arange(ov.shape[1])]
        gam = np.where(ov == gmax)[0]
        labels[mo < neg] = 0
        labels[gam] = 1
        labels[mo >= pos] = 1
        targets = bbox_transform(anchors, gt[am, :4])
    else:
        labels[:] = 0
    full = np.full(H * W * A, -1.0)
    full[inside] = labels
    ft = np.zeros((H * W * A, 4))
    ft[inside] = targets
    return full, ft, inside
