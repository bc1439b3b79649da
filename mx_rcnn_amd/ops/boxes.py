"""Box encode/decode/clip/IoU on tensors (reference `helper/processing/bbox_transform.py`,
`bbox_regression.py:11-31`).  ``iou_max`` dispatches to the HIP row-reduction kernel."""
import torch

from ._ext import ext_available, need_ext


def bbox_transform(ex, gt):
    ew = ex[..., 2] - ex[..., 0] + 1.0
    eh = ex[..., 3] - ex[..., 1] + 1.0
    ecx = ex[..., 0] + 0.5 * (ew - 1.0)
    ecy = ex[..., 1] + 0.5 * (eh - 1.0)
    gw = gt[..., 2] - gt[..., 0] + 1.0
    gh = gt[..., 3] - gt[..., 1] + 1.0
    gcx = gt[..., 0] + 0.5 * (gw - 1.0)
    gcy = gt[..., 1] + 0.5 * (gh - 1.0)
    return torch.stack([(gcx - ecx) / (ew + 1e-14), (gcy - ecy) / (eh + 1e-14),
                        torch.log(gw / ew), torch.log(gh / eh)], dim=-1)


def bbox_pred(boxes, deltas):
    """boxes (..., 4), deltas (..., 4C) -> (..., 4C)."""
    w = boxes[..., 2] - boxes[..., 0] + 1.0
    h = boxes[..., 3] - boxes[..., 1] + 1.0
    cx = boxes[..., 0] + 0.5 * (w - 1.0)
    cy = boxes[..., 1] + 0.5 * (h - 1.0)
    dx, dy, dw, dh = deltas[..., 0::4], deltas[..., 1::4], deltas[..., 2::4], deltas[..., 3::4]
    pcx = dx * w[..., None] + cx[..., None]
    pcy = dy * h[..., None] + cy[..., None]
    pw = torch.exp(dw) * w[..., None]
    ph = torch.exp(dh) * h[..., None]
    out = torch.stack([pcx - 0.5 * (pw - 1.0), pcy - 0.5 * (ph - 1.0),
                       pcx + 0.5 * (pw - 1.0), pcy + 0.5 * (ph - 1.0)], dim=-1)
    return out.reshape(deltas.shape)


def clip_boxes(boxes, im_h, im_w):
    """Clamp (..., 4C) boxes; im_h / im_w may be python numbers or broadcastable tensors."""
    out = boxes.clone()
    if not torch.is_tensor(im_w):
        im_w = torch.tensor(float(im_w), device=boxes.device)
        im_h = torch.tensor(float(im_h), device=boxes.device)
    wmax = (im_w - 1).to(boxes.dtype)
    hmax = (im_h - 1).to(boxes.dtype)
    zero = torch.zeros((), device=boxes.device, dtype=boxes.dtype)
    out[..., 0::4] = torch.maximum(torch.minimum(boxes[..., 0::4], wmax), zero)
    out[..., 1::4] = torch.maximum(torch.minimum(boxes[..., 1::4], hmax), zero)
    out[..., 2::4] = torch.maximum(torch.minimum(boxes[..., 2::4], wmax), zero)
    out[..., 3::4] = torch.maximum(torch.minimum(boxes[..., 3::4], hmax), zero)
    return out


def box_iou(a, b):
    """(..., n, 4) x (..., k, 4) -> (..., n, k) IoU with +1 areas (dense, reference op)."""
    iw = torch.minimum(a[..., :, None, 2], b[..., None, :, 2]) - torch.maximum(a[..., :, None, 0], b[..., None, :, 0]) + 1
    ih = torch.minimum(a[..., :, None, 3], b[..., None, :, 3]) - torch.maximum(a[..., :, None, 1], b[..., None, :, 1]) + 1
    valid = (iw > 0) & (ih > 0)
    inter = torch.where(valid, iw * ih, torch.zeros_like(iw))
    aa = (a[..., 2] - a[..., 0] + 1) * (a[..., 3] - a[..., 1] + 1)
    ba = (b[..., 2] - b[..., 0] + 1) * (b[..., 3] - b[..., 1] + 1)
    union = aa[..., :, None] + ba[..., None, :] - inter
    return torch.where(valid, inter / union, torch.zeros_like(inter))


def _gt_valid(gt, n_gt):
    G = gt.shape[1]
    return torch.arange(G, device=gt.device)[None, :] < n_gt[:, None].long()


def iou_max(boxes, gt, n_gt, off=0, want_gt_max=False):
    """Row max/argmax of IoU(boxes[b, :, off:off+4], gt[b, :n_gt[b], :4]) per image.

    boxes (B, N, bs) fp32, gt (B, G, 5), n_gt (B,) int32.  Returns (max_ov, argmax[, gt_max]).
    Rows of an image without gt get max 0 / argmax 0 (numpy argmax of an all-zero row).
    """
    if boxes.is_cuda:
        C = need_ext()
        return tuple(C.iou_max(boxes.contiguous().float(), int(off), gt.contiguous().float(),
                               n_gt.to(torch.int32).contiguous(), bool(want_gt_max)))
    if ext_available():  # C++ twin (host_ops.h iou_max_rows); the tensor version below is its oracle
        return tuple(need_ext().iou_max_cpu(boxes, int(off), gt, n_gt, bool(want_gt_max)))
    return iou_max_ref(boxes, gt, n_gt, off, want_gt_max)


def iou_max_ref(boxes, gt, n_gt, off=0, want_gt_max=False):
    """Dense tensor version of :func:`iou_max` (CPU oracle)."""
    b4 = boxes[..., off:off + 4].float()
    ov = box_iou(b4, gt[..., :4].float())  # (B, N, G)
    valid = _gt_valid(gt, n_gt)[:, None, :]
    ov = torch.where(valid, ov, torch.full_like(ov, -1.0))
    if ov.shape[-1] == 0:
        mx = torch.zeros(ov.shape[:2], device=boxes.device)
        am = torch.zeros(ov.shape[:2], dtype=torch.int32, device=boxes.device)
    else:
        am = ov.argmax(dim=-1)  # first max, like numpy
        mx = ov.gather(-1, am[..., None])[..., 0]
        has = (n_gt > 0)[:, None]
        mx = torch.where(has, mx, torch.zeros_like(mx))
        am = torch.where(has, am, torch.zeros_like(am)).to(torch.int32)
    if want_gt_max:
        gm = ov.clamp_min(0).amax(dim=1) if ov.shape[1] else torch.zeros(gt.shape[:2], device=boxes.device)
        return mx, am, gm
    return mx, am
