"""Minibatch construction (reference `rcnn/minibatch.py:36-395`).

``get_minibatch`` / ``get_image_array`` / ``sample_rois`` keep the reference's semantics on
the host (image decode, flip, resize, offline-proposal RoI sampling).  ``assign_anchor`` is
provided for API parity, but the training loop computes anchor targets ON THE DEVICE
inside the model step (ops/anchor_target.py) instead of in the loader thread.
"""
import numpy as np
import numpy.random as npr

from ..config import config
from ..processing import image_processing
from ..processing.bbox_regression import expand_bbox_regression_targets


def load_image(entry):
    if entry.get('synthetic_seed') is not None:
        from .synthetic import synthetic_image
        im = synthetic_image(entry)
    else:
        im = image_processing.imread(entry['image'])
    if entry.get('flipped'):
        im = im[:, ::-1, :]
    return im


def get_image_array(roidb, scales, scale_indexes, need_mean=True, raw=False):
    """-> (batch array, scales).  ``raw``: the resized uint8 BGR images as a zero-padded
    (B, H, W, 3) array, converted on the device (ops/image.py) instead of here."""
    processed, im_scales = [], []
    for i, entry in enumerate(roidb):
        im = load_image(entry)
        im, im_scale = image_processing.resize(im, scales[scale_indexes[i]], config.MAX_SIZE)
        if raw:
            processed.append(np.ascontiguousarray(im, dtype=np.uint8))
        else:
            processed.append(image_processing.transform(im, config.PIXEL_MEANS, need_mean=need_mean).astype(np.float32))
        im_scales.append(im_scale)
    if raw:
        h = max(p.shape[0] for p in processed)
        w = max(p.shape[1] for p in processed)
        out = np.zeros((len(processed), h, w, 3), np.uint8)
        for k, p in enumerate(processed):
            out[k, :p.shape[0], :p.shape[1]] = p
        return out, im_scales
    return image_processing.tensor_vstack(processed), im_scales


def sample_rois(roidb, fg_rois_per_image, rois_per_image, num_classes):
    """Offline-proposal sampler: fg >= FG_THRESH, bg in [LO, HI), random fill to a fixed count."""
    labels = roidb['max_classes']
    overlaps = roidb['max_overlaps']
    rois = roidb['boxes']
    fg = np.where(overlaps >= config.TRAIN.FG_THRESH)[0]
    fg_this = int(np.minimum(fg_rois_per_image, fg.size))
    if fg.size > 0:
        fg = npr.choice(fg, size=fg_this, replace=False)
    bg = np.where((overlaps < config.TRAIN.BG_THRESH_HI) & (overlaps >= config.TRAIN.BG_THRESH_LO))[0]
    bg_this = int(np.minimum(rois_per_image - fg_this, bg.size))
    if bg.size > 0:
        bg = npr.choice(bg, size=bg_this, replace=False)
    keep = np.append(fg, bg).astype(np.int64)
    if keep.shape[0] < rois_per_image:
        gap = rois_per_image - keep.shape[0]
        keep = np.append(keep, npr.choice(np.arange(len(rois)), size=gap, replace=gap > len(rois)))
    labels = labels[keep].copy()
    labels[fg_this:] = 0
    overlaps = overlaps[keep]
    rois = rois[keep]
    bbox_targets, bbox_inside = expand_bbox_regression_targets(roidb['bbox_targets'][keep, :], num_classes)
    return rois, labels, bbox_targets, bbox_inside, overlaps


def get_minibatch(roidb, num_classes, mode='test', need_mean=True, has_rpn=None, scale_indexes=None, raw=False):
    """``has_rpn`` overrides config[TRAIN|TEST].HAS_RPN (thread-safe use from loader workers);
    ``scale_indexes`` fixes the per-image SCALES choice (the loaders plan it per global batch);
    ``raw``: data is the uint8 (B, H, W, 3) image batch (get_image_array)."""
    num_images = len(roidb)
    scale_idx = npr.randint(0, high=len(config.SCALES), size=num_images) if scale_indexes is None \
        else np.asarray(scale_indexes)
    im_array, im_scales = get_image_array(roidb, config.SCALES, scale_idx, need_mean=need_mean, raw=raw)
    cfg_key = 'TRAIN' if mode == 'train' else 'TEST'
    if (config[cfg_key].HAS_RPN if has_rpn is None else has_rpn):
        # per-image im_info (the reference asserts a single image here)
        im_info = np.array([[r_h, r_w, s] for (r_h, r_w), s in
                            zip([_resized_hw(r, s) for r, s in zip(roidb, im_scales)], im_scales)], dtype=np.float32)
        data = {'data': im_array, 'im_info': im_info}
        label = {}
        if mode == 'train':
            gts = []
            for r, s in zip(roidb, im_scales):
                gi = np.where(r['gt_classes'] != 0)[0]
                g = np.empty((gi.size, 5), dtype=np.float32)
                g[:, :4] = r['boxes'][gi, :] * s
                g[:, 4] = r['gt_classes'][gi]
                gts.append(g)
            label = {'gt_boxes': gts}
        return data, label
    if mode == 'train':
        assert config.TRAIN.BATCH_SIZE % config.TRAIN.BATCH_IMAGES == 0
        rois_per_image = config.TRAIN.BATCH_SIZE // config.TRAIN.BATCH_IMAGES
        fg_per_image = int(np.round(config.TRAIN.FG_FRACTION * rois_per_image))
        rois_a, labels_a, tgt_a, inw_a = [], [], [], []
        for i in range(num_images):
            rois, labels, tgt, inw, _ = sample_rois(roidb[i], fg_per_image, rois_per_image, num_classes)
            rois_a.append(np.hstack((i * np.ones((rois.shape[0], 1)), rois * im_scales[i])))
            labels_a.append(labels)
            tgt_a.append(tgt)
            inw_a.append(inw)
        inw = np.array(inw_a)
        data = {'data': im_array, 'rois': np.array(rois_a, dtype=np.float32)}
        label = {'label': np.array(labels_a), 'bbox_target': np.array(tgt_a), 'bbox_inside_weight': inw,
                 'bbox_outside_weight': (inw > 0).astype(np.float32)}
        return data, label
    rois_a = [np.hstack((i * np.ones((r['boxes'].shape[0], 1)), r['boxes'] * im_scales[i]))
              for i, r in enumerate(roidb)]
    im_info = np.array([[*_resized_hw(r, s), s] for r, s in zip(roidb, im_scales)], dtype=np.float32)
    return {'data': im_array, 'rois': np.vstack(rois_a).astype(np.float32), 'im_info': im_info}, {}


def _resized_hw(entry, scale):
    h = entry.get('height')
    w = entry.get('width')
    if h is None or w is None:
        h, w = load_image(entry).shape[:2]
    return int(round(h * scale)), int(round(w * scale))


def assign_anchor(feat_shape, gt_boxes, im_info, feat_stride=16, scales=(8, 16, 32), ratios=(0.5, 1, 2),
                  allowed_border=0):
    """Reference-layout RPN targets for ONE image on the host (API parity; the trainer computes
    these on the device).  feat_shape: (..., H, W); im_info: [[h, w, scale]]."""
    import torch
    from ..ops.anchor_target import anchor_target
    H, W = int(feat_shape[-2]), int(feat_shape[-1])
    g = np.asarray(gt_boxes, dtype=np.float32).reshape(-1, 5)
    gt = torch.from_numpy(g)[None] if g.size else torch.zeros(1, 0, 5)
    out = anchor_target((H, W), gt, torch.tensor([g.shape[0]], dtype=torch.int32),
                        torch.as_tensor(np.asarray(im_info, dtype=np.float32).reshape(1, 3)), feat_stride, scales,
                        ratios, allowed_border)
    return {k: v.numpy().astype(np.float32) for k, v in out.items()}
