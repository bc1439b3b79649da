"""roidb preparation (reference `helper/processing/roidb.py:14-90`)."""
import logging

import numpy as np

from ..config import config
from ..processing.bbox_regression import compute_bbox_regression_targets


def prepare_roidb(imdb, roidb):
    """Add image path, height/width (header-only read), max_overlaps and max_classes."""
    logging.info('prepare roidb')
    for i in range(len(roidb)):
        roidb[i]['image'] = imdb.image_path_from_index(imdb.image_set_index[i])
        if config.TRAIN.ASPECT_GROUPING and ('height' not in roidb[i] or 'width' not in roidb[i]):
            h, w = imdb.image_size_from_index(imdb.image_set_index[i])
            roidb[i]['height'], roidb[i]['width'] = h, w
        gt_overlaps = roidb[i]['gt_overlaps'].toarray()
        max_overlaps = gt_overlaps.max(axis=1) if gt_overlaps.size else np.zeros(0, np.float32)
        max_classes = gt_overlaps.argmax(axis=1) if gt_overlaps.size else np.zeros(0, np.int64)
        roidb[i]['max_overlaps'] = max_overlaps
        roidb[i]['max_classes'] = max_classes
        assert all(max_classes[np.where(max_overlaps == 0)[0]] == 0)
        assert all(max_classes[np.where(max_overlaps > 0)[0]] != 0)


def add_bbox_regression_targets(roidb):
    """Add normalised 'bbox_targets'; returns flattened (means, stds) of shape (C*4,)."""
    logging.info('add bounding box regression targets')
    assert len(roidb) > 0 and 'max_classes' in roidb[0]
    num_classes = roidb[0]['gt_overlaps'].shape[1]
    for r in roidb:
        r['bbox_targets'] = compute_bbox_regression_targets(r['boxes'], r['max_overlaps'], r['max_classes'])
    if config.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED:
        means = np.tile(np.array(config.TRAIN.BBOX_MEANS), (num_classes, 1))
        stds = np.tile(np.array(config.TRAIN.BBOX_STDS), (num_classes, 1))
    else:
        counts = np.zeros((num_classes, 1)) + config.EPS
        sums = np.zeros((num_classes, 4))
        sq = np.zeros((num_classes, 4))
        for r in roidb:
            t = r['bbox_targets']
            for cls in range(1, num_classes):
                idx = np.where(t[:, 0] == cls)[0]
                if idx.size:
                    counts[cls] += idx.size
                    sums[cls] += t[idx, 1:].sum(axis=0)
                    sq[cls] += (t[idx, 1:] ** 2).sum(axis=0)
        means = sums / counts
        stds = np.sqrt(np.maximum(sq / counts - means ** 2, 0))
        stds[stds == 0] = 1.0
    for r in roidb:
        t = r['bbox_targets']
        for cls in range(1, num_classes):
            idx = np.where(t[:, 0] == cls)[0]
            t[idx, 1:] -= means[cls, :]
            t[idx, 1:] /= stds[cls, :]
    return means.ravel(), stds.ravel()
