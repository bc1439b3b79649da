"""Generic ``.lst`` detection-list database (reference `helper/dataset/detection_list.py:20-127`),
used for WIDER FACE (`data/trainval.lst`).

Format: ``num_class:N`` / ``classes:name1 name2 ...`` / then per image
``relpath nbox x y w h [cls] ...``.  Boxes are xywh -> ``x2 = x + w - 1``; degenerate boxes are
widened to 2 px.  Extension over the reference (whose multi-class branch is a no-op): with
N > 1 each box carries a 5th field, the 1-based class id (``x y w h cls``).
"""
import logging
import os

import numpy as np
import scipy.sparse

from . import cache as cache_io
from .imdb import IMDB


class DetectionList(IMDB):
    def __init__(self, dataset_name, list_file, dataset_root, outdata_path):
        super(DetectionList, self).__init__(dataset_name)
        self.dataset_name = dataset_name
        self.list_file = list_file
        self.dataset_root = dataset_root
        self.outdata_path = outdata_path
        with open(list_file) as f:
            line = f.readline().strip('\n').split(':')
            assert line[0] == 'num_class', 'first line should be: num_class:XX'
            self.num_classes = int(line[1]) + 1
            line = f.readline().strip('\n').split(':')
            assert line[0] == 'classes', 'second line should be: classes:XX1 XX2 XX3...'
            names = line[1].split() if len(line) > 1 else []
            self.classes = ['__background__'] + names[:self.num_classes - 1]
            self.annos = [x.strip('\n').split() for x in f.readlines() if x.strip()]
        self.num_images = len(self.annos)
        self.image_set_index = list(range(self.num_images))

    @property
    def cache_path(self):
        path = os.path.join(self.outdata_path, 'cache')
        os.makedirs(path, exist_ok=True)
        return path

    def image_path_from_index(self, index):
        f = os.path.join(self.dataset_root, self.annos[index][0])
        assert os.path.exists(f), 'Path does not exist: {}'.format(f)
        return f

    def evaluate_detections(self, detections):
        """mAP against the list's own boxes (the reference's list dataset had no evaluator)."""
        from .voc_eval import eval_in_memory
        return eval_in_memory(self.gt_roidb(), detections, self.classes)

    def gt_roidb(self):
        cache_file = os.path.join(self.cache_path, self.name + '_gt_roidb.npz')
        if os.path.exists(cache_file):
            roidb = cache_io.load_roidb(cache_file)
            logging.info('%s gt roidb loaded from %s', self.name, cache_file)
            return roidb
        roidb = [self.load_annotation(i) for i in self.image_set_index]
        cache_io.save_roidb(cache_file, roidb)
        return roidb

    def load_annotation(self, index):
        rec = self.annos[index]
        num_objs = int(rec[1])
        assert num_objs > 0
        per = 4 if self.num_classes == 2 else 5
        boxes = np.zeros((num_objs, 4), dtype=np.int16)
        gt_classes = np.zeros((num_objs,), dtype=np.int32)
        overlaps = np.zeros((num_objs, self.num_classes), dtype=np.float32)
        for ix in range(num_objs):
            f = rec[2 + per * ix: 2 + per * ix + per]
            x1, y1 = float(f[0]), float(f[1])
            x2 = x1 + float(f[2]) - 1.0
            y2 = y1 + float(f[3]) - 1.0
            if x2 - x1 <= 0:
                x2 = x1 + 2
            if y2 - y1 <= 0:
                y2 = y1 + 2
            cls = 1 if per == 4 else int(f[4])
            boxes[ix, :] = [x1, y1, x2, y2]
            gt_classes[ix] = cls
            overlaps[ix, cls] = 1.0
        return {'boxes': boxes, 'gt_classes': gt_classes, 'gt_overlaps': scipy.sparse.csr_matrix(overlaps),
                'flipped': False}
