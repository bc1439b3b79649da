"""RPN anchor-target assignment on device (reference
`rcnn/minibatch.py:204-395` `assign_anchor`, which the reference runs on the CPU inside
the data loader every step).

Labels/targets come from the fused HIP kernel (IoU row max/argmax, per-gt column max over
inside anchors, label rules, encode); fg/bg subsampling is a device random-rank select.
Output layout matches the reference: label (B, A*H*W) in (a, h, w) order; bbox_target /
inside / outside weights (B, 4A, H, W).
"""
import os

import numpy as np
import torch

from ..config import config as _global_cfg
from ._ext import ext_available, need_ext, const_tensor
from .anchors import base_anchors
from .boxes import bbox_transform, box_iou
from .sampling import keep_random
from .rng import uniform


def _assign_ref(H, W, base, feat_stride, im_info, border, gt, n_gt, neg, pos, clobber):
    B, G = gt.shape[0], gt.shape[1]
    sx = torch.arange(W, dtype=torch.float32) * feat_stride
    sy = torch.arange(H, dtype=torch.float32) * feat_stride
    yy, xx = torch.meshgrid(sy, sx, indexing='ij')
    shifts = torch.stack([xx, yy, xx, yy], -1).reshape(-1, 1, 4)
    anchors = (shifts + base.cpu()[None]).reshape(-1, 4)
    N = anchors.shape[0]
    labels = torch.full((B, N), -1, dtype=torch.int32)
    targets = torch.zeros(B, N, 4)
    for b in range(B):
        im_h, im_w = float(im_info[b, 0]), float(im_info[b, 1])
        inside = ((anchors[:, 0] >= -border) & (anchors[:, 1] >= -border) &
                  (anchors[:, 2] < im_w + border) & (anchors[:, 3] < im_h + border))
        ng = int(n_gt[b])
        idx = torch.nonzero(inside)[:, 0]
        if ng == 0 or idx.numel() == 0:
            labels[b, idx] = 0
            continue
        g = gt[b, :ng, :4].float()
        ov = box_iou(anchors[idx], g)
        am = ov.argmax(dim=1)
        mo = ov.gather(1, am[:, None])[:, 0]
        gmax = ov.max(dim=0).values
        is_best = (ov == gmax[None, :]).any(dim=1)
        lab = torch.full((idx.numel(),), -1, dtype=torch.int32)
        if not clobber:
            lab[mo < neg] = 0
        lab[is_best] = 1
        lab[mo >= pos] = 1
        if clobber:
            lab[mo < neg] = 0
        labels[b, idx] = lab
        targets[b, idx] = bbox_transform(anchors[idx], g[am]).float()
    return labels, targets


def anchor_target(feat_shape, gt_boxes, n_gt, im_info, feat_stride=16, scales=(8, 16, 32), ratios=(0.5, 1, 2),
                  allowed_border=0, cfg=None, generator=None):
    """Returns dict(label, bbox_target, bbox_inside_weight, bbox_outside_weight) in reference layout.

    feat_shape: (H, W) of the RPN score map; gt_boxes (B, G, 5) padded rows beyond n_gt[b]
    (scaled to the network input); im_info (B, 3).
    """
    cfg = cfg or _global_cfg
    H, W = int(feat_shape[0]), int(feat_shape[1])
    dev = gt_boxes.device
    base = base_anchors(feat_stride, scales, ratios, dev)
    A = base.shape[0]
    B = gt_boxes.shape[0]
    n_gt = n_gt.to(torch.int32).contiguous()
    with torch.no_grad():
        num_fg = int(cfg.TRAIN.RPN_FG_FRACTION * cfg.TRAIN.RPN_BATCH_SIZE)
        if gt_boxes.is_cuda and os.environ.get('MXR_ANCHOR_FUSED', '1') != '0':
            # assignment + subsampling + layout in four grid-wide launches (csrc/hip/sample.hip
            # anchor_mark: histogram thresholds instead of a one-workgroup selection pass)
            C = need_ext()
            keys = uniform((B, H * W * A), dev, generator)
            iw = [float(v) for v in np.asarray(cfg.TRAIN.RPN_BBOX_INSIDE_WEIGHTS, dtype=np.float64).ravel()[:4]]
            lab, bt, inside, outside, meta = C.anchor_target_fused(
                base, H, W, float(feat_stride), im_info.float().contiguous(), int(allowed_border),
                gt_boxes.float().contiguous(), n_gt, float(cfg.TRAIN.RPN_NEGATIVE_OVERLAP),
                float(cfg.TRAIN.RPN_POSITIVE_OVERLAP), bool(cfg.TRAIN.RPN_CLOBBER_POSITIVES), keys, num_fg,
                int(cfg.TRAIN.RPN_BATCH_SIZE), iw, float(cfg.TRAIN.RPN_POSITIVE_WEIGHT))
            return {'label': lab, 'bbox_target': bt, 'bbox_inside_weight': inside, 'bbox_outside_weight': outside,
                    'sample_meta': meta}
        if gt_boxes.is_cuda:
            C = need_ext()
            label, targets, _, _ = C.anchor_target_assign(
                base, H, W, float(feat_stride), im_info.float().contiguous(), int(allowed_border),
                gt_boxes.float().contiguous(), n_gt, float(cfg.TRAIN.RPN_NEGATIVE_OVERLAP),
                float(cfg.TRAIN.RPN_POSITIVE_OVERLAP), bool(cfg.TRAIN.RPN_CLOBBER_POSITIVES))
            # fused subsampling + weights + reference layout (csrc/hip/sample.hip): 3 launches
            keys = uniform(label.shape, dev, generator)
            iw = [float(v) for v in np.asarray(cfg.TRAIN.RPN_BBOX_INSIDE_WEIGHTS, dtype=np.float64).ravel()[:4]]
            lab, bt, inside, outside, meta = C.anchor_sample(label, targets.contiguous(), keys, A, H, W, num_fg,
                                                             int(cfg.TRAIN.RPN_BATCH_SIZE), iw,
                                                             float(cfg.TRAIN.RPN_POSITIVE_WEIGHT))
            # meta (B, 4) = [all_fg, all_bg, n_fg, n_bg]: the RPN loss's 'valid' count without a reduction
            return {'label': lab, 'bbox_target': bt, 'bbox_inside_weight': inside, 'bbox_outside_weight': outside,
                    'sample_meta': meta}
        elif ext_available():  # C++ twin (host_ops.h); _assign_ref is its test oracle
            label, targets = need_ext().anchor_assign_cpu(
                base, H, W, float(feat_stride), im_info.float(), int(allowed_border), gt_boxes.float(), n_gt,
                float(cfg.TRAIN.RPN_NEGATIVE_OVERLAP), float(cfg.TRAIN.RPN_POSITIVE_OVERLAP),
                bool(cfg.TRAIN.RPN_CLOBBER_POSITIVES))
        else:
            label, targets = _assign_ref(H, W, base, feat_stride, im_info, allowed_border, gt_boxes, n_gt,
                                         cfg.TRAIN.RPN_NEGATIVE_OVERLAP, cfg.TRAIN.RPN_POSITIVE_OVERLAP,
                                         cfg.TRAIN.RPN_CLOBBER_POSITIVES)
        # subsample: fg to FG_FRACTION*BATCH, bg to BATCH - #fg (rcnn/minibatch.py:319-334)
        fg = label == 1
        fg_keep = keep_random(fg, num_fg, generator)
        label = torch.where(fg & ~fg_keep, torch.full_like(label, -1), label)
        num_bg = cfg.TRAIN.RPN_BATCH_SIZE - fg_keep.sum(dim=1)
        bg = label == 0
        bg_keep = keep_random(bg, num_bg, generator)
        label = torch.where(bg & ~bg_keep, torch.full_like(label, -1), label)
        # weights (RPN_POSITIVE_WEIGHT < 0: uniform 1/num_examples)
        inside_w = const_tensor(cfg.TRAIN.RPN_BBOX_INSIDE_WEIGHTS, dev)
        inside = (label == 1).float()[..., None] * inside_w
        if cfg.TRAIN.RPN_POSITIVE_WEIGHT < 0:
            num_ex = (label >= 0).sum(dim=1).clamp_min(1).float()
            pw = nw = (1.0 / num_ex)[:, None]
        else:
            p = float(cfg.TRAIN.RPN_POSITIVE_WEIGHT)
            pw = (p / (label == 1).sum(dim=1).clamp_min(1).float())[:, None]
            nw = ((1.0 - p) / (label == 0).sum(dim=1).clamp_min(1).float())[:, None]
        outside = ((label == 1).float() * pw + (label == 0).float() * nw)[..., None].expand(-1, -1, 4)
        # layout: (B, H, W, A) -> label (B, A*H*W); (B, H, W, A, 4) -> (B, 4A, H, W)
        lab = label.reshape(B, H, W, A).permute(0, 3, 1, 2).reshape(B, A * H * W).contiguous()

        def chw(t):
            return t.reshape(B, H, W, A * 4).permute(0, 3, 1, 2).contiguous()
        return {'label': lab, 'bbox_target': chw(targets), 'bbox_inside_weight': chw(inside),
                'bbox_outside_weight': chw(outside.contiguous())}
