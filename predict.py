#!/usr/bin/env python
"""WIDER FACE single-image inference (reference `predict.py`): resize (640, 1024), class-1
scores >= thresh, NMS, then the ``nest`` filter (drop boxes nested inside others), boxes
drawn on the ORIGINAL image into result.jpg."""
import argparse

import numpy as np

from mx_rcnn_amd.config import config
from mx_rcnn_amd.core import launch
from mx_rcnn_amd.core.detector import Detector
from mx_rcnn_amd.core.tester import draw_boxes
from mx_rcnn_amd.processing.image_processing import imread, imwrite, resize, transform
from mx_rcnn_amd.processing.nms import nms, nest
from mx_rcnn_amd.utils.load_model import load_param


def predict(args, ctx):
    color = imread(args.img)
    img, scale = resize(color.copy(), args.scale, args.max_scale)
    im_info = np.array([[img.shape[0], img.shape[1], scale]], dtype=np.float32)
    data = transform(img, config.PIXEL_MEANS, need_mean=False).astype(np.float32)
    arg, aux, num_classes = load_param(args.prefix, args.epoch, convert=False)
    network = args.network if args.network != 'vgg16' or 'resnet' not in args.prefix else 'resnet50'
    config.TEST.HAS_RPN = True
    model, _, _ = launch.build_model(network, 2 if num_classes == 1000 else num_classes, train_mode='test')
    det = Detector(model, ctx, arg, aux, compute_dtype=getattr(args, 'dtype', 'fp32'))
    scores, boxes = det.im_detect(data, im_info)
    cls_boxes, cls_scores = boxes[:, 4:8], scores[:, 1]
    keep = np.where(cls_scores >= args.thresh)[0]
    dets = np.hstack((cls_boxes[keep], cls_scores[keep, None])).astype(np.float32)
    dets = dets[nms(dets, args.nms_thresh), :]
    if getattr(ctx, 'type', str(ctx)) == 'cuda' and len(dets):
        import torch
        dets = dets[nest(torch.as_tensor(dets, device=ctx), thresh=args.nest_thresh), :]  # HIP nest kernel
    else:
        dets = dets[nest(dets, thresh=args.nest_thresh), :]
    dets = dets[(dets[:, 2] - dets[:, 0] + 1 >= args.min_size * scale) |
                (dets[:, 3] - dets[:, 1] + 1 >= args.min_size * scale)] if dets.size else dets
    out = draw_boxes(color, dets[:, :4] / scale, color=(0, 255, 0))
    imwrite(args.out, out)
    return dets


def parse_args(argv=None):
    p = argparse.ArgumentParser(description='WIDER FACE prediction')
    p.add_argument('--img', default='test.jpg')
    p.add_argument('--gpu', type=int, default=0)
    p.add_argument('--prefix', default='resnet-50')
    p.add_argument('--epoch', type=int, default=0)
    p.add_argument('--thresh', type=float, default=0.5)
    p.add_argument('--nms-thresh', dest='nms_thresh', type=float, default=0.3)
    p.add_argument('--nest-thresh', dest='nest_thresh', type=float, default=0.8)
    p.add_argument('--min-size', dest='min_size', type=int, default=24)
    p.add_argument('--scale', type=int, default=640)
    p.add_argument('--max-scale', dest='max_scale', type=int, default=1024)
    p.add_argument('--out', default='result.jpg')
    launch.add_common_args(p, eval_cli=True)
    return p.parse_args(argv)


if __name__ == '__main__':
    a = parse_args()
    rank, world, dev = launch.init_runtime(a)
    predict(a, dev)
