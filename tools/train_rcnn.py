#!/usr/bin/env python
"""Train a Fast R-CNN head on precomputed proposals (reference `tools/train_rcnn.py`; stages 2/4
of alternate training).  After training, every saved epoch gets the empirical target
normalisation folded into bbox_pred (`tools/train_rcnn.py:87-93`)."""
import argparse
import logging
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mx_rcnn_amd.config import config  # noqa: E402
from mx_rcnn_amd.core import launch  # noqa: E402
from mx_rcnn_amd.core.callback import Speedometer  # noqa: E402
from mx_rcnn_amd.core.lr_scheduler import FactorScheduler  # noqa: E402
from mx_rcnn_amd.core.metric import rcnn_metrics  # noqa: E402
from mx_rcnn_amd.core.module import MutableModule  # noqa: E402
from mx_rcnn_amd.data import load_data  # noqa: E402
from mx_rcnn_amd.data.loader import ROIIter  # noqa: E402
from mx_rcnn_amd.utils.load_model import (do_checkpoint, load_checkpoint, load_param, save_checkpoint,  # noqa: E402
                                          fold_bbox_pred)


def train_rcnn(image_set, year, root_path, devkit_path, pretrained, epoch, prefix, ctx, begin_epoch, end_epoch,
               frequent, kv_store, work_load_list=None, resume=False, proposal='rpn', network='vgg16',
               roidb_override=None, max_steps=None, use_graph=False, seed=0, rank=0, world=1):
    config.TRAIN.HAS_RPN = False
    if roidb_override is not None:
        imdb, roidb, means, stds = roidb_override
    else:
        imdb, roidb, means, stds = getattr(load_data, 'load_%s_roidb' % proposal)(image_set, year, root_path,
                                                                                  devkit_path, flip=True)
    model, arg, aux = launch.build_model(network, imdb.num_classes, None, 0, resume, train_mode='rcnn')
    if pretrained:
        try:
            arg, aux, _ = load_param(pretrained, epoch, convert=False)
            for k in ('fc8_weight', 'fc8_bias', 'fc1_weight', 'fc1_bias'):
                arg.pop(k, None)
            if not resume:
                for k in ('cls_score_weight', 'cls_score_bias', 'bbox_pred_weight', 'bbox_pred_bias'):
                    arg.pop(k, None)
        except FileNotFoundError:
            logging.warning('pretrained %s-%04d.params not found: random init', pretrained, epoch)
    train_data = ROIIter(roidb, batch_size=config.TRAIN.BATCH_IMAGES, shuffle=True, mode='train', rank=rank,
                         world_size=world, seed=seed, work_load_list=work_load_list)
    fam = launch.family(network)
    fixed = (['conv1', 'conv2', 'conv3', 'conv4', 'conv5'] if config.TRAIN.FINETUNE else ['conv1', 'conv2']) \
        if fam == 'vgg' else launch.FIXED_PREFIX['resnet']
    launch.calibrate_if_random(model, train_data, arg)
    mod = MutableModule(model, ['data', 'rois'], ['label', 'bbox_target', 'bbox_inside_weight',
                                                  'bbox_outside_weight'], context=ctx, fixed_param_prefix=fixed,
                        mode='rcnn', use_graph=use_graph)
    mod.fit(train_data, eval_metric=rcnn_metrics(), epoch_end_callback=do_checkpoint(prefix),
            batch_end_callback=Speedometer(config.TRAIN.BATCH_IMAGES * world, frequent=frequent),
            kvstore=kv_store, optimizer='sgd',
            optimizer_params={'momentum': 0.9, 'wd': 0.0005, 'learning_rate': 0.001,
                              'lr_scheduler': FactorScheduler(30000, 0.1),
                              'rescale_grad': 1.0 / config.TRAIN.BATCH_SIZE},
            arg_params=arg, aux_params=aux, begin_epoch=begin_epoch, num_epoch=end_epoch, max_steps=max_steps)
    if rank == 0:
        for e in range(begin_epoch + 1, end_epoch + 1):
            try:
                a, x = load_checkpoint(prefix, e)
            except FileNotFoundError:
                continue
            save_checkpoint(prefix, e, fold_bbox_pred(a, means, stds), x)
    return mod


def parse_args(argv=None):
    p = argparse.ArgumentParser(description='Train a Fast R-CNN Network')
    p.add_argument('--image_set', default='trainval')
    p.add_argument('--year', default='2007')
    p.add_argument('--root_path', default='data')
    p.add_argument('--devkit_path', default='data/VOCdevkit')
    p.add_argument('--pretrained', default='model/vgg16')
    p.add_argument('--epoch', type=int, default=1)
    p.add_argument('--prefix', default='model/rcnn')
    p.add_argument('--gpus', default='0')
    p.add_argument('--begin_epoch', type=int, default=0)
    p.add_argument('--end_epoch', type=int, default=8)
    p.add_argument('--frequent', type=int, default=20)
    p.add_argument('--kv_store', default='device')
    p.add_argument('--work_load_list', default=None)
    p.add_argument('--finetune', action='store_true')
    p.add_argument('--resume', action='store_true')
    p.add_argument('--proposal', default='rpn', help='rpn | ss')
    launch.add_common_args(p)
    return p.parse_args(argv)


if __name__ == '__main__':
    a = parse_args()
    rank, world, dev = launch.init_runtime(a)
    config.TRAIN.FINETUNE = a.finetune
    train_rcnn(a.image_set, a.year, a.root_path, a.devkit_path, a.pretrained, a.epoch, a.prefix, dev,
               a.begin_epoch, a.end_epoch, a.frequent, a.kv_store, resume=a.resume, proposal=a.proposal,
               network=a.network, max_steps=a.max_steps, use_graph=not a.eager, rank=rank, world=world)
