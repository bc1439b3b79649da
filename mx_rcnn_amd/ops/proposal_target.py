"""Proposal-target sampling on device (reference
`rcnn/rpn/proposal_target.py:34-76,135-195`), batched over images, static shapes.

Per image: append gt boxes to the proposals, IoU row max/argmax against gt (HIP
`iou_max`), fg = max >= FG_THRESH (exactly FG slots, with-replacement pad prepended),
bg in [BG_LO, BG_HI) (TRAIN fallback [0, BG_HI+0.2) when empty), labels zeroed from slot
fg_this onwards, class-specific targets (optionally normalised by BBOX_MEANS/STDS) with
inside weights on the assigned class slot and outside = (inside > 0).
"""
import numpy as np
import torch

from ..config import config as _global_cfg
from .boxes import bbox_transform, iou_max
from .sampling import sample_slots
from ._ext import const_tensor
from .rng import uniform


def proposal_target(rois, gt_boxes, n_gt, num_classes, cfg=None, is_train=True, generator=None):
    """rois (B, P, 5), gt_boxes (B, G, 5), n_gt (B,) -> dict of
    rois (B*R, 5), label (B*R,) int32, bbox_target / bbox_inside_weight / bbox_outside_weight (B*R, 4C)."""
    cfg = cfg or _global_cfg
    with torch.no_grad():
        B, P, _ = rois.shape
        G = gt_boxes.shape[1]
        dev = rois.device
        R = int(cfg.TRAIN.BATCH_SIZE)  # rois per image (symbol built before the *= ngpu)
        F = int(round(cfg.TRAIN.FG_FRACTION * R))
        gtf = gt_boxes.float()
        n_gt = n_gt.to(torch.int32)
        if rois.is_cuda:
            # fused sampling + targets (csrc/hip/sample.hip): iou_max + one draw + one kernel
            from ._ext import need_ext
            rf = rois.float().contiguous()
            max_ov, argmax = iou_max(rf, gtf, n_gt, off=1)
            F = int(round(cfg.TRAIN.FG_FRACTION * R))
            rnd = uniform((B, 2 * (P + G) + R), dev, generator)
            out = need_ext().proposal_sample(
                rf, gtf.contiguous(), n_gt.contiguous(), max_ov.contiguous(), argmax.contiguous(), rnd, R, F,
                int(num_classes), float(cfg.TRAIN.FG_THRESH), float(cfg.TRAIN.BG_THRESH_HI),
                float(cfg.TRAIN.BG_THRESH_LO), bool(is_train), bool(cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED),
                [float(v) for v in np.asarray(cfg.TRAIN.BBOX_MEANS, dtype=np.float64).ravel()[:4]],
                [float(v) for v in np.asarray(cfg.TRAIN.BBOX_STDS, dtype=np.float64).ravel()[:4]],
                [float(v) for v in np.asarray(cfg.TRAIN.BBOX_INSIDE_WEIGHTS, dtype=np.float64).ravel()[:4]])
            return {'rois': out[0], 'label': out[1], 'bbox_target': out[2], 'bbox_inside_weight': out[3],
                    'bbox_outside_weight': out[4]}
        bidx = torch.arange(B, device=dev, dtype=torch.float32)[:, None, None].expand(B, G, 1)
        all_rois = torch.cat([rois.float(), torch.cat([bidx, gtf[..., :4]], dim=-1)], dim=1).contiguous()
        M = P + G
        row = torch.arange(M, device=dev)[None, :]
        valid = (row < P) | ((row - P) < n_gt[:, None].long())
        max_ov, argmax = iou_max(all_rois, gtf, n_gt, off=1)
        argmax = argmax.long()
        labels_all = torch.gather(gtf[..., 4], 1, argmax.clamp(max=max(G - 1, 0))) if G > 0 else \
            torch.zeros(B, M, device=dev)
        fg = valid & (max_ov >= cfg.TRAIN.FG_THRESH)
        bg = valid & (max_ov < cfg.TRAIN.BG_THRESH_HI) & (max_ov >= cfg.TRAIN.BG_THRESH_LO)
        if is_train:
            bg_fb = valid & (max_ov < cfg.TRAIN.BG_THRESH_HI + 0.2) & (max_ov >= 0)
            bg = torch.where((bg.sum(dim=1) == 0)[:, None], bg_fb, bg)
        # fall back to "any valid row" when a pool is empty (the reference would raise)
        fg_pool = torch.where((fg.sum(dim=1) == 0)[:, None], valid, fg)
        bg_pool = torch.where((bg.sum(dim=1) == 0)[:, None], valid, bg)
        fg_idx, _ = sample_slots(fg_pool, F, generator)
        fg_this = torch.clamp(fg.sum(dim=1), max=F)
        bg_idx, _ = sample_slots(bg_pool, R - F, generator)
        keep = torch.cat([fg_idx, bg_idx], dim=1)  # (B, R)
        slot = torch.arange(R, device=dev)[None, :]
        labels = torch.gather(labels_all, 1, keep)
        labels = torch.where(slot < fg_this[:, None], labels, torch.zeros_like(labels))
        out_rois = torch.gather(all_rois, 1, keep[..., None].expand(-1, -1, 5))
        assigned = torch.gather(argmax, 1, keep)
        gt_sel = torch.gather(gtf[..., :4], 1, assigned.clamp(max=max(G - 1, 0))[..., None].expand(-1, -1, 4)) \
            if G > 0 else torch.zeros(B, R, 4, device=dev)
        t = bbox_transform(out_rois[..., 1:5], gt_sel)
        if cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED:
            means = const_tensor(cfg.TRAIN.BBOX_MEANS, dev)
            stds = const_tensor(cfg.TRAIN.BBOX_STDS, dev)
            t = (t - means) / stds
        pos = labels > 0
        t = torch.where(pos[..., None], t, torch.zeros_like(t))
        cls = labels.long().clamp(0, num_classes - 1)
        onehot = torch.nn.functional.one_hot(cls, num_classes).to(torch.float32) * pos[..., None].float()
        targets = (onehot[..., None] * t[..., None, :]).reshape(B, R, 4 * num_classes)
        inside_w = const_tensor(np.asarray(cfg.TRAIN.BBOX_INSIDE_WEIGHTS).ravel(), dev)
        inside = (onehot[..., None] * inside_w).reshape(B, R, 4 * num_classes)
        outside = (inside > 0).float()
        return {'rois': out_rois.reshape(B * R, 5).contiguous(),
                'label': labels.reshape(B * R).to(torch.int32).contiguous(),
                'bbox_target': targets.reshape(B * R, -1).contiguous(),
                'bbox_inside_weight': inside.reshape(B * R, -1).contiguous(),
                'bbox_outside_weight': outside.reshape(B * R, -1).contiguous()}
