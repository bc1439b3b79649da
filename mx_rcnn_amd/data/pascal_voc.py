"""PASCAL VOC image database (reference `helper/dataset/pascal_voc.py:19-291`).

Annotations are 0-based (`xmin - 1`), difficult objects excluded; selective-search
proposals from `<root>/selective_search_data/<name>.mat`; RPN proposals from the
`<root>/rpn_data/<name>_rpn.npz` dump written by ``rcnn.rpn.generate``; detections written
as `comp4_det_<set>_<cls>.txt` and scored with the Python VOC AP (07 11-point if year < 2010).
Caches are pickle-free .npz (data/cache.py).
"""
import logging
import os
import xml.etree.ElementTree as ET

import numpy as np
import scipy.sparse

from ..processing.bbox_process import unique_boxes, filter_small_boxes
from . import cache as cache_io
from .imdb import IMDB
from .voc_eval import voc_eval

VOC_CLASSES = ['__background__', 'aeroplane', 'bicycle', 'bird', 'boat', 'bottle', 'bus', 'car', 'cat', 'chair',
               'cow', 'diningtable', 'dog', 'horse', 'motorbike', 'person', 'pottedplant', 'sheep', 'sofa', 'train',
               'tvmonitor']


class PascalVOC(IMDB):
    def __init__(self, image_set, year, root_path, devkit_path):
        super(PascalVOC, self).__init__('voc_' + year + '_' + image_set)
        self.image_set = image_set
        self.year = year
        self.root_path = root_path
        self.devkit_path = devkit_path
        self.data_path = os.path.join(devkit_path, 'VOC' + year)
        self.classes = list(VOC_CLASSES)
        self.num_classes = 21
        self.image_set_index = self.load_image_set_index()
        self.num_images = len(self.image_set_index)
        self.config = {'comp_id': 'comp4', 'use_diff': False, 'min_size': 2}

    @property
    def cache_path(self):
        path = os.path.join(self.root_path, 'cache')
        os.makedirs(path, exist_ok=True)
        return path

    def load_image_set_index(self):
        f = os.path.join(self.data_path, 'ImageSets', 'Main', self.image_set + '.txt')
        assert os.path.exists(f), 'Path does not exist: {}'.format(f)
        with open(f) as fh:
            return [x.strip() for x in fh.readlines() if x.strip()]

    def image_path_from_index(self, index):
        f = os.path.join(self.data_path, 'JPEGImages', index + '.jpg')
        assert os.path.exists(f), 'Path does not exist: {}'.format(f)
        return f

    def gt_roidb(self):
        cache_file = os.path.join(self.cache_path, self.name + '_gt_roidb.npz')
        if os.path.exists(cache_file):
            roidb = cache_io.load_roidb(cache_file)
            logging.info('%s gt roidb loaded from %s', self.name, cache_file)
            return roidb
        roidb = [self.load_pascal_annotation(i) for i in self.image_set_index]
        cache_io.save_roidb(cache_file, roidb)
        logging.info('wrote gt roidb to %s', cache_file)
        return roidb

    def load_pascal_annotation(self, index):
        filename = os.path.join(self.data_path, 'Annotations', index + '.xml')
        objs = ET.parse(filename).findall('object')
        if not self.config['use_diff']:
            objs = [o for o in objs if o.find('difficult') is None or int(o.find('difficult').text) == 0]
        n = len(objs)
        boxes = np.zeros((n, 4), dtype=np.uint16)
        gt_classes = np.zeros((n,), dtype=np.int32)
        overlaps = np.zeros((n, self.num_classes), dtype=np.float32)
        class_to_index = dict(zip(self.classes, range(self.num_classes)))
        for ix, obj in enumerate(objs):
            bb = obj.find('bndbox')
            x1, y1, x2, y2 = [float(bb.find(t).text) - 1 for t in ('xmin', 'ymin', 'xmax', 'ymax')]
            cls = class_to_index[obj.find('name').text.lower().strip()]
            boxes[ix, :] = [x1, y1, x2, y2]
            gt_classes[ix] = cls
            overlaps[ix, cls] = 1.0
        return {'boxes': boxes, 'gt_classes': gt_classes, 'gt_overlaps': scipy.sparse.csr_matrix(overlaps),
                'flipped': False}

    def roidb(self, gt_roidb):
        return self.selective_search_roidb(gt_roidb)

    def load_selective_search_roidb(self, gt_roidb):
        import scipy.io
        matfile = os.path.join(self.root_path, 'selective_search_data', self.name + '.mat')
        assert os.path.exists(matfile), 'selective search data does not exist: {}'.format(matfile)
        raw = scipy.io.loadmat(matfile)['boxes'].ravel()
        box_list = []
        for i in range(raw.shape[0]):
            boxes = raw[i][:, (1, 0, 3, 2)] - 1
            boxes = boxes[unique_boxes(boxes), :]
            boxes = boxes[filter_small_boxes(boxes, self.config['min_size']), :]
            box_list.append(boxes)
        return self.create_roidb_from_box_list(box_list, gt_roidb)

    def selective_search_roidb(self, gt_roidb):
        cache_file = os.path.join(self.cache_path, self.name + '_ss_roidb.npz')
        if os.path.exists(cache_file):
            return cache_io.load_roidb(cache_file)
        if self.image_set != 'test':
            roidb = IMDB.merge_roidbs(gt_roidb, self.load_selective_search_roidb(gt_roidb))
        else:
            roidb = self.load_selective_search_roidb(None)
        cache_io.save_roidb(cache_file, roidb)
        return roidb

    def rpn_file(self):
        return os.path.join(self.root_path, 'rpn_data', self.name + '_rpn.npz')

    def load_rpn_roidb(self, gt_roidb):
        f = self.rpn_file()
        logging.info('loading %s', f)
        assert os.path.exists(f), 'rpn data not found at {}'.format(f)
        return self.create_roidb_from_box_list(cache_io.load_box_list(f), gt_roidb)

    def rpn_roidb(self, gt_roidb):
        if self.image_set != 'test':
            return IMDB.merge_roidbs(gt_roidb, self.load_rpn_roidb(gt_roidb))
        return self.load_rpn_roidb(gt_roidb)

    # ------------------------------------------------------------------ evaluation
    def evaluate_detections(self, detections):
        os.makedirs(os.path.join(self.devkit_path, 'results', 'VOC' + self.year, 'Main'), exist_ok=True)
        self.write_pascal_results(detections)
        return self.do_python_eval()

    def get_result_file_template(self):
        folder = os.path.join(self.devkit_path, 'results', 'VOC' + self.year, 'Main')
        return os.path.join(folder, self.config['comp_id'] + '_det_' + self.image_set + '_{:s}.txt')

    def write_pascal_results(self, all_boxes):
        for cls_ind, cls in enumerate(self.classes):
            if cls == '__background__':
                continue
            with open(self.get_result_file_template().format(cls), 'wt') as f:
                for im_ind, index in enumerate(self.image_set_index):
                    dets = all_boxes[cls_ind][im_ind]
                    if len(dets) == 0:
                        continue
                    for k in range(dets.shape[0]):
                        f.write('{:s} {:.3f} {:.1f} {:.1f} {:.1f} {:.1f}\n'.format(
                            index, dets[k, -1], dets[k, 0] + 1, dets[k, 1] + 1, dets[k, 2] + 1, dets[k, 3] + 1))

    def do_python_eval(self):
        annopath = os.path.join(self.data_path, 'Annotations', '{0!s}.xml')
        imageset_file = os.path.join(self.data_path, 'ImageSets', 'Main', self.image_set + '.txt')
        cache_dir = os.path.join(self.cache_path, self.name)
        aps = []
        use_07 = int(self.year) < 2010
        logging.info('VOC07 metric? %s', 'Y' if use_07 else 'No')
        for cls in self.classes:
            if cls == '__background__':
                continue
            _, _, ap = voc_eval(self.get_result_file_template().format(cls), annopath, imageset_file, cls,
                                cache_dir, ovthresh=0.5, use_07_metric=use_07)
            aps.append(ap)
            logging.info('AP for %s = %.4f', cls, ap)
        logging.info('Mean AP = %.4f', float(np.mean(aps)))
        return float(np.mean(aps))
