#!/usr/bin/env python
"""Dump RPN proposals for an image set and report recall (reference `tools/test_rpn.py`)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mx_rcnn_amd.config import config  # noqa: E402
from mx_rcnn_amd.core import launch  # noqa: E402
from mx_rcnn_amd.core.generate import Detector, generate_detections  # noqa: E402
from mx_rcnn_amd.data.load_data import load_gt_roidb  # noqa: E402
from mx_rcnn_amd.data.loader import ROIIter  # noqa: E402
from mx_rcnn_amd.parallel import dist as pdist  # noqa: E402
from mx_rcnn_amd.utils.load_model import load_param  # noqa: E402


def test_rpn(image_set, year, root_path, devkit_path, prefix, epoch, ctx, vis=False, network='vgg16',
             imdb_roidb=None, dtype='fp32'):
    """``dtype``: the RPN test graph's precision on the GPU ('fp32' as the reference, 'bf16', 'fp16')."""
    config.TEST.HAS_RPN = True
    config.TEST.RPN_PRE_NMS_TOP_N = -1
    config.TEST.RPN_POST_NMS_TOP_N = 2000
    if imdb_roidb is None:
        imdb, roidb = load_gt_roidb(image_set, year, root_path, devkit_path)
    else:
        imdb, roidb = imdb_roidb
    # data parallel: each rank runs images rank::world, the dump is gathered (core/generate.py)
    rank, world = pdist.get_rank(), pdist.get_world_size()
    test_data = _rpn_test_iter(roidb[rank::world])
    arg, aux, num_classes = load_param(prefix, epoch, convert=False)
    model, _, _ = launch.build_model(network, num_classes if num_classes != 1000 else imdb.num_classes,
                                     train_mode='rpn_test')
    det = Detector(model, ctx, arg, aux, compute_dtype=dtype)
    boxes = generate_detections(det, test_data, imdb, vis=vis, shard=(rank, world))
    imdb.evaluate_recall(roidb, candidate_boxes=boxes)
    return boxes


def _rpn_test_iter(roidb):
    """Single-image non-shuffled iterator yielding data + im_info (RPN test graph inputs)."""
    from mx_rcnn_amd.data.loader import AnchorLoader
    return AnchorLoader(None, roidb, batch_size=1, shuffle=False, mode='test')


def parse_args(argv=None):
    p = argparse.ArgumentParser(description='Test a Region Proposal Network')
    p.add_argument('--image_set', default='trainval')
    p.add_argument('--year', default='2007')
    p.add_argument('--root_path', default='data')
    p.add_argument('--devkit_path', default='data/VOCdevkit')
    p.add_argument('--prefix', default='model/rpn')
    p.add_argument('--epoch', type=int, default=8)
    p.add_argument('--gpu', type=int, default=0)
    p.add_argument('--vis', action='store_true')
    launch.add_common_args(p, eval_cli=True)
    return p.parse_args(argv)


if __name__ == '__main__':
    a = parse_args()
    rank, world, dev = launch.init_runtime(a)
    test_rpn(a.image_set, a.year, a.root_path, a.devkit_path, a.prefix, a.epoch, dev, a.vis, a.network, dtype=a.dtype)
