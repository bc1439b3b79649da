"""Image database base class (reference `helper/dataset/imdb.py:13-191`)."""
import logging

import numpy as np
import scipy.sparse

from ..processing.bbox_regression import bbox_overlaps
from ..processing.image_processing import image_size


class IMDB(object):
    def __init__(self, name):
        self.name = name
        self.classes = []
        self.num_classes = 0
        self.image_set_index = []
        self.num_images = 0
        self.config = {}

    def image_path_from_index(self, index):
        raise NotImplementedError

    def image_size_from_index(self, index):
        """(height, width) from the file header (the reference decodes the whole image)."""
        return image_size(self.image_path_from_index(index))

    def gt_roidb(self):
        raise NotImplementedError

    def roidb(self, gt_roidb):
        raise NotImplementedError

    def create_roidb_from_box_list(self, box_list, gt_roidb):
        """Proposals -> roidb entries with sparse max-IoU-per-class overlaps vs gt."""
        assert len(box_list) == self.num_images, 'number of boxes matrix must match number of images'
        roidb = []
        for i in range(self.num_images):
            boxes = np.asarray(box_list[i])[:, :4]
            n = boxes.shape[0]
            overlaps = np.zeros((n, self.num_classes), dtype=np.float32)
            if gt_roidb is not None and gt_roidb[i]['boxes'].size > 0 and n > 0:
                gt_boxes = gt_roidb[i]['boxes']
                gt_classes = gt_roidb[i]['gt_classes']
                gt_ov = bbox_overlaps(boxes.astype(np.float64), gt_boxes.astype(np.float64))
                argmaxes = gt_ov.argmax(axis=1)
                maxes = gt_ov.max(axis=1)
                idx = np.where(maxes > 0)[0]
                overlaps[idx, gt_classes[argmaxes[idx]]] = maxes[idx]
            roidb.append({'boxes': boxes, 'gt_classes': np.zeros((n,), dtype=np.int32),
                          'gt_overlaps': scipy.sparse.csr_matrix(overlaps), 'flipped': False})
        return roidb

    @staticmethod
    def merge_roidbs(a, b):
        assert len(a) == len(b)
        for i in range(len(a)):
            a[i]['boxes'] = np.vstack((a[i]['boxes'], b[i]['boxes']))
            a[i]['gt_classes'] = np.hstack((a[i]['gt_classes'], b[i]['gt_classes']))
            a[i]['gt_overlaps'] = scipy.sparse.vstack([a[i]['gt_overlaps'], b[i]['gt_overlaps']])
        return a

    def append_flipped_images(self, roidb):
        """Mirror boxes x1' = W - x2 - 1; images are flipped when loaded."""
        logging.info('append flipped images to roidb')
        assert self.num_images == len(roidb)
        widths = []
        for i in range(self.num_images):
            w = roidb[i].get('width')
            widths.append(w if w is not None else self.image_size_from_index(self.image_set_index[i])[1])
        for i in range(self.num_images):
            boxes = roidb[i]['boxes'].copy()
            oldx1 = boxes[:, 0].copy()
            oldx2 = boxes[:, 2].copy()
            boxes[:, 0] = widths[i] - oldx2 - 1
            boxes[:, 2] = widths[i] - oldx1 - 1
            assert (boxes[:, 2] >= boxes[:, 0]).all()
            entry = {'boxes': boxes, 'gt_classes': roidb[i]['gt_classes'], 'gt_overlaps': roidb[i]['gt_overlaps'],
                     'flipped': True}
            for k in ('height', 'width', 'synthetic_seed'):
                if k in roidb[i]:
                    entry[k] = roidb[i][k]
            roidb.append(entry)
        self.image_set_index = list(self.image_set_index) * 2
        self.num_images = len(self.image_set_index)
        return roidb

    def evaluate_recall(self, roidb, candidate_boxes=None, thresholds=None, area='all', limit=None):
        """Greedy gt<->proposal matching recall over IoU thresholds; returns (ar, recalls, thresholds)."""
        areas = {'all': 0, 'small': 1, 'medium': 2, 'large': 3, '96-128': 4, '128-256': 5, '256-512': 6,
                 '512-inf': 7}
        area_ranges = [[0 ** 2, 1e5 ** 2], [0 ** 2, 32 ** 2], [32 ** 2, 96 ** 2], [96 ** 2, 1e5 ** 2],
                       [96 ** 2, 128 ** 2], [128 ** 2, 256 ** 2], [256 ** 2, 512 ** 2], [512 ** 2, 1e5 ** 2]]
        assert area in areas, 'unknown area range: {}'.format(area)
        area_range = area_ranges[areas[area]]
        gt_overlaps = np.zeros(0)
        num_pos = 0
        for i in range(len(roidb)):
            max_gt = roidb[i]['gt_overlaps'].toarray().max(axis=1)
            gt_inds = np.where((roidb[i]['gt_classes'] > 0) & (max_gt == 1))[0]
            gt_boxes = roidb[i]['boxes'][gt_inds, :]
            gt_areas = (gt_boxes[:, 2] - gt_boxes[:, 0] + 1) * (gt_boxes[:, 3] - gt_boxes[:, 1] + 1)
            valid = np.where((gt_areas >= area_range[0]) & (gt_areas <= area_range[1]))[0]
            gt_boxes = gt_boxes[valid, :]
            num_pos += len(valid)
            if candidate_boxes is None:
                boxes = roidb[i]['boxes'][np.where(roidb[i]['gt_classes'] == 0)[0], :]
            else:
                boxes = np.asarray(candidate_boxes[i])[:, :4]
            if boxes.shape[0] == 0:
                continue
            if limit is not None and boxes.shape[0] > limit:
                boxes = boxes[:limit, :]
            overlaps = bbox_overlaps(boxes.astype(np.float64), gt_boxes.astype(np.float64))
            _gt = np.zeros((gt_boxes.shape[0]))
            for j in range(gt_boxes.shape[0]):
                argmax_ov = overlaps.argmax(axis=0)
                max_ov = overlaps.max(axis=0)
                gt_ind = max_ov.argmax()
                gt_ovr = max_ov.max()
                assert gt_ovr >= 0
                box_ind = argmax_ov[gt_ind]
                _gt[j] = overlaps[box_ind, gt_ind]
                overlaps[box_ind, :] = -1
                overlaps[:, gt_ind] = -1
            gt_overlaps = np.hstack((gt_overlaps, _gt))
        gt_overlaps = np.sort(gt_overlaps)
        if thresholds is None:
            thresholds = np.arange(0.5, 0.95 + 1e-5, 0.05)
        recalls = np.zeros_like(thresholds, dtype=np.float64)
        for i, t in enumerate(thresholds):
            recalls[i] = (gt_overlaps >= t).sum() / float(max(num_pos, 1))
        ar = recalls.mean()
        logging.info('average recall: %.3f', ar)
        for t, r in zip(thresholds, recalls):
            logging.info('recall @%.2f: %.3f', t, r)
        return ar, recalls, thresholds

    def evaluate_detections(self, detections):
        raise NotImplementedError
