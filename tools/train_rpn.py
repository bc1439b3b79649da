#!/usr/bin/env python
"""Train an RPN (reference `tools/train_rpn.py`; stage 1/3 of alternate training)."""
import argparse
import logging
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mx_rcnn_amd.config import config  # noqa: E402
from mx_rcnn_amd.core import launch  # noqa: E402
from mx_rcnn_amd.core.callback import Speedometer  # noqa: E402
from mx_rcnn_amd.core.lr_scheduler import FactorScheduler  # noqa: E402
from mx_rcnn_amd.core.metric import rpn_metrics  # noqa: E402
from mx_rcnn_amd.core.module import MutableModule  # noqa: E402
from mx_rcnn_amd.data.load_data import load_gt_roidb  # noqa: E402
from mx_rcnn_amd.data.loader import AnchorLoader  # noqa: E402
from mx_rcnn_amd.utils.load_model import do_checkpoint, load_param  # noqa: E402


def train_rpn(image_set, year, root_path, devkit_path, pretrained, epoch, prefix, ctx, begin_epoch, end_epoch,
              frequent, kv_store, work_load_list=None, resume=False, network='vgg16', synthetic=None,
              max_steps=None, use_graph=True, seed=0, rank=0, world=1):
    config.TRAIN.HAS_RPN = True
    config.TRAIN.BATCH_SIZE = 1
    model, arg, aux = launch.build_model(network, 21 if synthetic is None else synthetic[1].num_classes, None,
                                         0, resume, train_mode='rpn')
    if pretrained:
        try:
            arg, aux, _ = load_param(pretrained, epoch, convert=False)
            for k in ('fc8_weight', 'fc8_bias', 'fc1_weight', 'fc1_bias'):
                arg.pop(k, None)
            if not resume:
                for k in [k for k in arg if k.startswith('rpn_')]:
                    arg.pop(k)
        except FileNotFoundError:
            logging.warning('pretrained %s-%04d.params not found: random init', pretrained, epoch)
    if synthetic is not None:
        roidb = synthetic[0]
    else:
        _, roidb = load_gt_roidb(image_set, year, root_path, devkit_path, flip=True)
    train_data = AnchorLoader(model, roidb, batch_size=1, shuffle=True, anchor_scales=model.anchor_scales,
                              rank=rank, world_size=world, seed=seed, work_load_list=work_load_list,
                              raw_images=launch.raw_images(ctx))
    fam = launch.family(network)
    fixed = (['conv1', 'conv2', 'conv3', 'conv4', 'conv5'] if config.TRAIN.FINETUNE else ['conv1', 'conv2']) \
        if fam == 'vgg' else launch.FIXED_PREFIX['resnet']
    launch.calibrate_if_random(model, train_data, arg)
    mod = MutableModule(model, ['data', 'im_info'], ['gt_boxes'], context=ctx, fixed_param_prefix=fixed,
                        mode='rpn', use_graph=use_graph)
    mod.fit(train_data, eval_metric=rpn_metrics(), epoch_end_callback=do_checkpoint(prefix),
            batch_end_callback=Speedometer(world, frequent=frequent), kvstore=kv_store, optimizer='sgd',
            optimizer_params={'momentum': 0.9, 'wd': 0.0005, 'learning_rate': 0.001,
                              'lr_scheduler': FactorScheduler(60000, 0.1),
                              'rescale_grad': 1.0 / config.TRAIN.BATCH_SIZE},
            arg_params=arg, aux_params=aux, begin_epoch=begin_epoch, num_epoch=end_epoch, max_steps=max_steps)
    return mod


def parse_args(argv=None):
    p = argparse.ArgumentParser(description='Train a Region Proposal Network')
    p.add_argument('--image_set', default='trainval')
    p.add_argument('--year', default='2007')
    p.add_argument('--root_path', default='data')
    p.add_argument('--devkit_path', default='data/VOCdevkit')
    p.add_argument('--pretrained', default='model/vgg16')
    p.add_argument('--epoch', type=int, default=1)
    p.add_argument('--prefix', default='model/rpn')
    p.add_argument('--gpus', default='0')
    p.add_argument('--begin_epoch', type=int, default=0)
    p.add_argument('--end_epoch', type=int, default=8)
    p.add_argument('--frequent', type=int, default=20)
    p.add_argument('--kv_store', default='device')
    p.add_argument('--work_load_list', default=None)
    p.add_argument('--finetune', action='store_true')
    p.add_argument('--resume', action='store_true')
    launch.add_common_args(p)
    return p.parse_args(argv)


if __name__ == '__main__':
    a = parse_args()
    rank, world, dev = launch.init_runtime(a)
    config.TRAIN.FINETUNE = a.finetune
    syn = None
    if a.synthetic:
        imdb, roidb = launch.synthetic_roidb(a, 21, flip=True)
        syn = (roidb, imdb)
    train_rpn(a.image_set, a.year, a.root_path, a.devkit_path, a.pretrained, a.epoch, a.prefix, dev, a.begin_epoch,
              a.end_epoch, a.frequent, a.kv_store, resume=a.resume, network=a.network, synthetic=syn,
              max_steps=a.max_steps, use_graph=not a.eager, rank=rank, world=world)
