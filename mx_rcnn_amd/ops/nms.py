"""Greedy NMS (reference `helper/processing/nms.py:4-38`) on tensors.

* ``nms(boxes, scores, thresh)``: general single-set NMS returning kept indices in
  descending-score order (ties: lower index first).  Used by test-time per-class NMS.
* ``batched_nms``: per-class NMS for all classes at once via the coordinate-offset trick
  (boxes of different classes never overlap), one bitmask pass instead of C launches.
* The proposal layer calls the fused bitmask kernel directly (ops/proposal.py).

GPU tensors run the two-stage bitmask kernel (csrc/hip/nms.hip); CPU tensors a
vectorised greedy loop with the same visiting order and suppression rule (IoU > thresh).
"""
import os

import torch

from ._ext import need_ext

MAX_GPU_BOXES = 65536  # one bitmask pass: at most 1024 64-box blocks (keep list in LDS or, if larger, global)


def _greedy_ref(boxes, n_valid, thresh, max_keep=None, fp32=False):
    """boxes already score-sorted (P, 4); returns list of kept positions among the first n_valid.
    Runs the extension's C++ twin when it is built (CPU configuration), else the tensor loop
    below (the oracle the twin is tested against).  fp32=True: IoU in float32, bit-identical to
    the GPU bitmask kernel (the default float64 can differ from it on exact-threshold ties)."""
    n = int(n_valid)
    if n == 0:
        return []
    from ._ext import ext_available
    if ext_available() and not boxes.is_cuda:
        return need_ext().nms_cpu(boxes[:n], n, float(thresh), -1 if max_keep is None else int(max_keep),
                                  bool(fp32)).tolist()
    return _greedy_loop(boxes, n, thresh, max_keep, fp32)


def _greedy_loop(boxes, n, thresh, max_keep=None, fp32=False):
    b = boxes[:n].float() if fp32 else boxes[:n].double()
    x1, y1, x2, y2 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    areas = (x2 - x1 + 1) * (y2 - y1 + 1)
    removed = torch.zeros(n, dtype=torch.bool)
    keep = []
    for i in range(n):
        if removed[i]:
            continue
        keep.append(i)
        if max_keep is not None and len(keep) >= max_keep:
            break
        if i + 1 < n:
            xx1 = torch.maximum(x1[i], x1[i + 1:])
            yy1 = torch.maximum(y1[i], y1[i + 1:])
            xx2 = torch.minimum(x2[i], x2[i + 1:])
            yy2 = torch.minimum(y2[i], y2[i + 1:])
            w = (xx2 - xx1 + 1).clamp_min(0)
            h = (yy2 - yy1 + 1).clamp_min(0)
            inter = w * h
            ovr = inter / (areas[i] + areas[i + 1:] - inter)
            removed[i + 1:] |= ovr > thresh
    return keep


def nms_debug_check(sboxes, n_valid, thresh, post, keep, n_keep):
    """``MXR_NMS_CHECK=1``: recompute the greedy keep list on the device with a plain flag loop
    (csrc/hip/nms.hip ``nms_check_kernel``) and raise on the first position where the bitmask
    reducer differs.  Synchronises, so it is skipped while a graph is being captured."""
    if os.environ.get('MXR_NMS_CHECK', '0') != '1' or torch.cuda.is_current_stream_capturing():
        return
    res = need_ext().nms_check(sboxes, n_valid, float(thresh), int(post), keep, n_keep).cpu()
    for b in range(res.shape[0]):
        bad, cnt = int(res[b, 0]), int(res[b, 1])
        if bad >= 0:
            got = keep[b, max(bad - 2, 0):bad + 3].tolist()
            raise RuntimeError('MXR_NMS_CHECK: image %d: NMS reducer differs from the device greedy oracle at keep '
                               'position %d (oracle kept %d, reducer %d; reducer keep[%d:%d] = %s)'
                               % (b, bad, cnt, int(n_keep[b]), max(bad - 2, 0), bad + 3, got))


def sort_desc(scores):
    """Descending stable order (ties -> lower index first)."""
    return torch.sort(scores, dim=-1, descending=True, stable=True)


def nms(boxes, scores, thresh, max_keep=None):
    """Indices (int64, original numbering) of boxes kept by greedy NMS."""
    if boxes.numel() == 0:
        return torch.zeros(0, dtype=torch.long, device=boxes.device)
    s, order = sort_desc(scores.float())
    b = boxes.float()[order].contiguous()
    n = b.shape[0]
    if boxes.is_cuda:
        C = need_ext()
        post = n if max_keep is None else min(max_keep, n)
        nv = torch.full((1,), n, dtype=torch.int32, device=boxes.device)
        u = torch.zeros(1, post, device=boxes.device)
        _, _, keep, n_keep = C.nms_proposals(b[None], s[None].contiguous(), nv, float(thresh), post, u)
        nms_debug_check(b[None], nv, thresh, post, keep, n_keep)
        k = int(n_keep.item())  # host read: test-time API returns a variable-length list
        return order[keep[0, :k]]
    keep = _greedy_ref(b, n, thresh, max_keep)
    return order[torch.tensor(keep, dtype=torch.long)]


def batched_nms(boxes, scores, classes, thresh, max_keep=None):
    """Per-class NMS in one pass: offset each class's boxes by class_id * (max_coord + 1)."""
    if boxes.numel() == 0:
        return torch.zeros(0, dtype=torch.long, device=boxes.device)
    if boxes.is_cuda and boxes.shape[0] > MAX_GPU_BOXES:
        # one bitmask pass holds at most MAX_GPU_BOXES boxes: run the classes separately
        # (classes never interact), then restore the global descending-score order
        keeps = []
        for c in torch.unique(classes).tolist():
            idx = torch.nonzero(classes == c).flatten()
            keeps.append(idx[nms(boxes[idx], scores[idx], thresh, max_keep)])
        keep = torch.cat(keeps)
        order = torch.sort(scores[keep].float(), descending=True, stable=True).indices
        keep = keep[order]
        return keep if max_keep is None else keep[:max_keep]
    max_coord = boxes.max()
    offs = classes.to(boxes.dtype) * (max_coord + 1)
    return nms(boxes + offs[:, None], scores, thresh, max_keep)
