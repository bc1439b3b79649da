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

    # gt-area buckets of the recall report (pixel areas, inclusive), keyed like the reference
    RECALL_AREAS = {'all': (0.0, 1e10), 'small': (0.0, 32.0 ** 2), 'medium': (32.0 ** 2, 96.0 ** 2),
                    'large': (96.0 ** 2, 1e10), '96-128': (96.0 ** 2, 128.0 ** 2),
                    '128-256': (128.0 ** 2, 256.0 ** 2), '256-512': (256.0 ** 2, 512.0 ** 2),
                    '512-inf': (512.0 ** 2, 1e10)}

    @staticmethod
    def greedy_gt_coverage(overlaps):
        """One-to-one proposal<->gt matching, best pair first: all (proposal, gt) pairs are visited
        in decreasing IoU and a pair is taken when neither side is used yet.  Returns, per gt
        column, the IoU of its matched proposal (0 when it gets none).  Same assignment as the
        reference's repeated global-argmax loop (`helper/dataset/imdb.py:160-171`), in
        O(P*G log(P*G)) instead of G full passes, and without its failure when there are fewer
        proposals than gt boxes."""
        n_box, n_gt = overlaps.shape
        cover = np.zeros(n_gt)
        if n_box == 0 or n_gt == 0:
            return cover
        order = np.argsort(-overlaps, axis=None, kind='stable')
        box_used = np.zeros(n_box, bool)
        gt_used = np.zeros(n_gt, bool)
        left = min(n_box, n_gt)
        for flat in order:
            b, g = divmod(int(flat), n_gt)
            if box_used[b] or gt_used[g]:
                continue
            box_used[b] = gt_used[g] = True
            cover[g] = overlaps[b, g]
            left -= 1
            if left == 0:
                break
        return cover

    def evaluate_recall(self, roidb, candidate_boxes=None, thresholds=None, area='all', limit=None):
        """Proposal recall of the gt boxes in an area bucket, over IoU thresholds (default
        0.5:0.05:0.95); returns (average recall, recalls, thresholds).  Proposals are the roidb's
        non-gt rows unless ``candidate_boxes`` is given; ``limit`` keeps the first N per image."""
        if area not in self.RECALL_AREAS:
            raise ValueError('unknown area range: %s' % area)
        lo, hi = self.RECALL_AREAS[area]
        covers, num_pos = [], 0
        for i, entry in enumerate(roidb):
            boxes_all = np.asarray(entry['boxes'], dtype=np.float64)
            is_gt = (entry['gt_classes'] > 0) & (entry['gt_overlaps'].toarray().max(axis=1) == 1)
            gt = boxes_all[is_gt]
            a = (gt[:, 2] - gt[:, 0] + 1) * (gt[:, 3] - gt[:, 1] + 1)
            gt = gt[(a >= lo) & (a <= hi)]
            num_pos += gt.shape[0]
            if candidate_boxes is None:
                props = boxes_all[entry['gt_classes'] == 0]
            else:
                props = np.asarray(candidate_boxes[i], dtype=np.float64)[:, :4]
            if limit is not None:
                props = props[:limit]
            if props.shape[0] == 0 or gt.shape[0] == 0:
                continue
            covers.append(self.greedy_gt_coverage(bbox_overlaps(props, gt)))
        cover = np.sort(np.concatenate(covers)) if covers else np.zeros(0)
        thresholds = np.arange(0.5, 0.95 + 1e-5, 0.05) if thresholds is None else np.asarray(thresholds)
        # matched gts with IoU >= t, for every t at once
        hits = cover.size - np.searchsorted(cover, thresholds, side='left')
        recalls = hits / float(max(num_pos, 1))
        ar = float(recalls.mean())
        logging.info('average recall: %.3f', ar)
        for t, r in zip(thresholds, recalls):
            logging.info('recall @%.2f: %.3f', t, r)
        return ar, recalls, thresholds

    def evaluate_detections(self, detections):
        raise NotImplementedError
