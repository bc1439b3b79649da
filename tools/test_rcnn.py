#!/usr/bin/env python
"""Evaluate a detector on a VOC image set (reference `tools/test_rcnn.py`).  ``--has_rpn`` uses
the Faster R-CNN test graph (RPN proposals, TEST 6000 -> 300); otherwise precomputed proposals
(``--proposal rpn|ss``).  ``--end2end`` is accepted (the reference's test.sh passes it but its
parser did not define it)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mx_rcnn_amd.config import config  # noqa: E402
from mx_rcnn_amd.core import launch  # noqa: E402
from mx_rcnn_amd.core.detector import Detector  # noqa: E402
from mx_rcnn_amd.core.tester import pred_eval  # noqa: E402
from mx_rcnn_amd.data import load_data  # noqa: E402
from mx_rcnn_amd.data.loader import AnchorLoader, ROIIter  # noqa: E402
from mx_rcnn_amd.utils.load_model import load_param  # noqa: E402


def test_rcnn(image_set, year, root_path, devkit_path, prefix, epoch, ctx, vis=False, has_rpn=True,
              proposal='rpn', network='vgg16', end2end=False, imdb_roidb=None, shard=(0, 1), dtype='fp32'):
    """``shard=(rank, world)``: each rank runs images ``rank::world`` and ``pred_eval`` gathers
    them (one process per GPU under torchrun; the reference tests on a single device).
    ``dtype``: the test graph's precision on the GPU ('fp32' as the reference, 'bf16', 'fp16')."""
    rank, world = shard
    if imdb_roidb is not None:  # e.g. synthetic set (in-memory evaluation)
        config.TEST.HAS_RPN = True
        imdb, roidb = imdb_roidb
        test_data = AnchorLoader(None, roidb[rank::world], batch_size=1, shuffle=False, mode='test')
    elif has_rpn:
        config.TEST.HAS_RPN = True
        config.TEST.RPN_PRE_NMS_TOP_N = 6000
        config.TEST.RPN_POST_NMS_TOP_N = 300
        imdb, roidb = load_data.load_gt_roidb(image_set, year, root_path, devkit_path)
        test_data = AnchorLoader(None, roidb[rank::world], batch_size=1, shuffle=False, mode='test')
    else:
        imdb, roidb = getattr(load_data, 'load_test_%s_roidb' % proposal)(image_set, year, root_path, devkit_path)
        test_data = ROIIter(roidb[rank::world], batch_size=1, shuffle=False, mode='test')
    arg, aux, num_classes = load_param(prefix, epoch, convert=False)
    model, _, _ = launch.build_model(network, num_classes, train_mode='test')
    det = Detector(model, ctx, arg, aux, compute_dtype=dtype)
    return pred_eval(det, test_data, imdb, vis=vis, shard=shard)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description='Test a Fast R-CNN network')
    p.add_argument('--image_set', default='test')
    p.add_argument('--year', default='2007')
    p.add_argument('--root_path', default='data')
    p.add_argument('--devkit_path', default='data/VOCdevkit')
    p.add_argument('--prefix', default='model/final')
    p.add_argument('--epoch', type=int, default=8)
    p.add_argument('--gpu', type=int, default=0)
    p.add_argument('--vis', action='store_true')
    p.add_argument('--has_rpn', action='store_true')
    p.add_argument('--end2end', action='store_true')
    p.add_argument('--proposal', default='rpn')
    p.add_argument('--num-classes', dest='num_classes', type=int, default=21, help='for --synthetic sets')
    launch.add_common_args(p, eval_cli=True)
    return p.parse_args(argv)


if __name__ == '__main__':
    a = parse_args()
    rank, world, dev = launch.init_runtime(a)
    syn = launch.synthetic_roidb(a, a.num_classes) if a.synthetic else None
    test_rcnn(a.image_set, a.year, a.root_path, a.devkit_path, a.prefix, a.epoch, dev, a.vis,
              a.has_rpn or a.end2end, a.proposal, a.network, a.end2end, imdb_roidb=syn, shard=(rank, world),
              dtype=a.dtype)
