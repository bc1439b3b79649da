#!/usr/bin/env python
"""Single-image VOC demo (reference `demo.py`): VGG16 Faster R-CNN test graph, per-class score
> 0.8, NMS 0.3, boxes drawn into result.jpg.  Unlike the reference (which calls transform()
without need_mean), the input IS mean-subtracted as the VGG model expects."""
import argparse

import numpy as np

from mx_rcnn_amd.config import config
from mx_rcnn_amd.core import launch
from mx_rcnn_amd.core.detector import Detector
from mx_rcnn_amd.core.tester import save_all_detection
from mx_rcnn_amd.data.pascal_voc import VOC_CLASSES
from mx_rcnn_amd.processing.image_processing import imread, resize, transform
from mx_rcnn_amd.processing.nms import nms
from mx_rcnn_amd.utils.load_model import load_param

CLASSES = VOC_CLASSES


def get_net(prefix, epoch, ctx, network='vgg16', dtype='fp32'):
    arg, aux, num_classes = load_param(prefix, epoch, convert=False)
    config.TEST.HAS_RPN = True
    config.TEST.RPN_PRE_NMS_TOP_N = 6000
    config.TEST.RPN_POST_NMS_TOP_N = 300
    model, _, _ = launch.build_model(network, num_classes, train_mode='test')
    return Detector(model, ctx, arg, aux, compute_dtype=dtype)


def demo_net(detector, image_name, out='result.jpg', conf_thresh=0.8, nms_thresh=0.3, classes=CLASSES):
    im = imread(image_name)
    im_r, scale = resize(im, config.SCALES[0], config.MAX_SIZE)
    im_tensor = transform(im_r, config.PIXEL_MEANS, need_mean=True).astype(np.float32)
    im_info = np.array([[im_tensor.shape[2], im_tensor.shape[3], scale]], dtype=np.float32)
    scores, boxes = detector.im_detect(im_tensor, im_info)
    all_boxes = [[] for _ in classes]
    for j in range(1, len(classes)):
        cls_boxes = boxes[:, 4 * j:4 * (j + 1)]
        cls_dets = np.hstack((cls_boxes, scores[:, j, None]))
        keep = nms(cls_dets, nms_thresh)
        cls_dets = cls_dets[keep, :]
        all_boxes[j] = cls_dets[cls_dets[:, -1] > conf_thresh]
    save_all_detection(im_tensor, all_boxes, classes, conf_thresh, path=out)
    return all_boxes


def parse_args(argv=None):
    p = argparse.ArgumentParser(description='Demonstrate a Faster R-CNN network')
    p.add_argument('--image', required=True)
    p.add_argument('--prefix', default='model/final')
    p.add_argument('--epoch', type=int, default=0)
    p.add_argument('--gpu', type=int, default=0)
    p.add_argument('--out', default='result.jpg')
    launch.add_common_args(p, eval_cli=True)
    return p.parse_args(argv)


if __name__ == '__main__':
    a = parse_args()
    rank, world, dev = launch.init_runtime(a)
    demo_net(get_net(a.prefix, a.epoch, dev, a.network, a.dtype), a.image, a.out)
