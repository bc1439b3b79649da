"""Proposal layer (reference `rcnn/rpn/proposal.py:39-149`), batched
over images with static output shapes so the whole training step can be captured in a
hipGraph (no host synchronisation):

  1. fused softmax(fg) + anchors + decode + clip + min-size   -> HIP `proposal_decode`
  2. stable descending sort, truncate to PRE_NMS_TOP_N        -> HIP `proposal_topk` (grid radix
                                                                 select + rank; MXR_TOPK=0: device
                                                                 sort + gather)
  3. bitmask NMS (IoU > thresh suppresses), keep POST_NMS_TOP_N,
     random pad (choice with replacement from keep), assemble (post, 5) RoIs
                                                              -> HIP `nms_proposals`

Deviation (documented): in TRAIN the scores are cropped to the same
(int(im_h/16), int(im_w/16)) grid as the deltas.  Tie order among equal scores is
"lower anchor index first" (numpy's unstable argsort leaves it unspecified).
"""
import os

import torch

from ._ext import ext_available, need_ext
from .anchors import base_anchors
from .boxes import bbox_pred, clip_boxes
from .nms import _greedy_ref, nms_debug_check
from .rng import uniform


def _decode_ref(cls, dlt, im_info, base, feat_stride, min_size, crop, is_prob):
    B, C2, H, W = cls.shape
    A = C2 // 2
    N = H * W * A
    boxes_all = torch.zeros(B, N, 4)
    keys_all = torch.full((B, N), float('-inf'))
    for b in range(B):
        im_h, im_w, im_scale = [float(v) for v in im_info[b]]
        Hc, Wc = H, W
        if crop:
            Hc, Wc = min(H, int(im_h / feat_stride)), min(W, int(im_w / feat_stride))
        c = cls[b, :, :Hc, :Wc].float()
        if is_prob:
            fg = c[A:]
        else:
            fg = torch.softmax(torch.stack([c[:A], c[A:]], 0), dim=0)[1]
        scores = fg.permute(1, 2, 0).reshape(-1)  # (h, w, a)
        d = dlt[b, :, :Hc, :Wc].float().permute(1, 2, 0).reshape(-1, 4)
        sx = torch.arange(Wc, dtype=torch.float32) * feat_stride
        sy = torch.arange(Hc, dtype=torch.float32) * feat_stride
        yy, xx = torch.meshgrid(sy, sx, indexing='ij')
        shifts = torch.stack([xx, yy, xx, yy], -1).reshape(-1, 1, 4)
        anchors = (shifts + base.cpu()[None]).reshape(-1, 4)
        p = clip_boxes(bbox_pred(anchors, d), im_h, im_w)
        ws = p[:, 2] - p[:, 0] + 1
        hs = p[:, 3] - p[:, 1] + 1
        ms = min_size * im_scale
        keep = (ws >= ms) & (hs >= ms) & ~torch.isnan(scores)
        n = p.shape[0]
        boxes_all[b, :n] = p
        keys_all[b, :n] = torch.where(keep, scores, torch.full_like(scores, float('-inf')))
    return boxes_all, keys_all


def proposal(cls, bbox_deltas, im_info, feat_stride=16, scales=(8, 16, 32), ratios=(0.5, 1, 2),
             pre_nms_top_n=12000, post_nms_top_n=6000, nms_thresh=0.7, min_size=16, is_train=False,
             is_prob=False, generator=None, after_mask=None, gave_up=None):
    """RPN outputs -> (rois (B, post, 5) fp32 [b, x1, y1, x2, y2], scores (B, post)).

    cls: (B, 2A, H, W) logits (or probabilities with is_prob=True), bbox_deltas (B, 4A, H, W),
    im_info (B, 3) = [height, width, scale] on the same device.  No gradient flows back
    (the reference's backward writes zeros).  after_mask: called (GPU) between the NMS bitmask
    and the serial NMS reduce, e.g. to record an event other streams start from.
    """
    with torch.no_grad():
        dev = cls.device
        base = base_anchors(feat_stride, scales, ratios, dev)
        im_info = im_info.float().contiguous()
        B = cls.shape[0]
        if cls.is_cuda:
            C = need_ext()
            boxes, keys = C.proposal_decode(cls, bbox_deltas, im_info, base, float(feat_stride), float(min_size),
                                            bool(is_train), bool(is_prob))
        elif ext_available():  # C++ twin (host_ops.h); the tensor version below is its test oracle
            boxes, keys = need_ext().proposal_decode_cpu(cls, bbox_deltas, im_info, base, float(feat_stride),
                                                         float(min_size), bool(is_train), bool(is_prob))
        else:
            boxes, keys = _decode_ref(cls, bbox_deltas, im_info, base, feat_stride, min_size, is_train, is_prob)
        N = keys.shape[1]
        P = N if pre_nms_top_n <= 0 else min(int(pre_nms_top_n), N)
        if cls.is_cuda and os.environ.get('MXR_TOPK', '1') == '1':
            # grid radix select + rank-by-counting top-P in stable descending order
            # (csrc/hip/topk.hip; MXR_TOPK=0: the device sort + gather below)
            skeys, sboxes, n_valid = C.proposal_topk(keys.contiguous(), boxes.contiguous(), P)
        else:
            skeys, order = torch.sort(keys, dim=1, descending=True, stable=True)
            if cls.is_cuda and os.environ.get('MXR_PROPOSAL_GATHER', '1') != '0':  # one launch: keys, boxes, count
                skeys, sboxes, n_valid = C.proposal_gather(skeys, order, boxes.contiguous(), P)
            else:
                skeys = skeys[:, :P].contiguous()
                order = order[:, :P]
                sboxes = torch.gather(boxes, 1, order[..., None].expand(-1, -1, 4)).contiguous()
                n_valid = (skeys > float('-inf')).sum(dim=1).to(torch.int32)
        post = int(post_nms_top_n) if post_nms_top_n > 0 else P
        rand_u = uniform((B, post), dev, generator)
        if cls.is_cuda:
            mask = None
            if after_mask is not None:
                mask = C.nms_mask_build(sboxes, n_valid, float(nms_thresh))
                after_mask()
            # gave_up: an int32 device counter, +1 per image whose multi-workgroup NMS chain gave up
            # a poll and was finished by the serial fallback (same output; observability only)
            rois, scores, keep, n_keep = C.nms_proposals(sboxes, skeys, n_valid, float(nms_thresh), post, rand_u,
                                                         mask, gave_up)
            nms_debug_check(sboxes, n_valid, nms_thresh, post, keep, n_keep)
            return rois, scores
        rois = torch.zeros(B, post, 5)
        scores = torch.zeros(B, post)
        for b in range(B):
            keep = _greedy_ref(sboxes[b], int(n_valid[b]), nms_thresh, post)
            nk = len(keep)
            if nk == 0:
                idx = [0] * post
            else:
                pad = [keep[min(int(float(u) * nk), nk - 1)] for u in rand_u[b, nk:post]]
                idx = keep + pad
            idx = torch.tensor(idx, dtype=torch.long)
            rois[b, :, 0] = float(b)
            rois[b, :, 1:] = sboxes[b, idx]
            scores[b] = skeys[b, idx]
        return rois, scores
