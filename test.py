#!/usr/bin/env python
"""Evaluate a trained detector (reference `test.py` -> tools/test_rcnn.py)."""
from tools.test_rcnn import parse_args, test_rcnn
from mx_rcnn_amd.core import launch

if __name__ == '__main__':
    a = parse_args()
    rank, world, dev = launch.init_runtime(a)
    syn = launch.synthetic_roidb(a, a.num_classes) if a.synthetic else None
    test_rcnn(a.image_set, a.year, a.root_path, a.devkit_path, a.prefix, a.epoch, dev, a.vis,
              a.has_rpn or a.end2end, a.proposal, a.network, a.end2end, imdb_roidb=syn, shard=(rank, world),
              dtype=a.dtype)
