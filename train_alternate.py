#!/usr/bin/env python
"""4-step alternate training (reference `train_alternate.py:15-63`):
RPN1 -> dump proposals -> RCNN1 -> RPN2 (finetune, conv frozen) -> dump -> combine(RPN2, RCNN1)
-> RCNN2 -> combine(RPN2, RCNN2) = final.  The hand-off between stages is the filesystem
(``.params`` checkpoints and ``rpn_data/<imdb>_rpn.npz``).  Unlike the reference fork (whose
tools unpack 2 values from the 3-valued ``load_param`` and crash), this path runs end to end,
and ``TRAIN.BATCH_IMAGES`` is restored for every stage instead of compounding."""
import argparse
import logging
import os

from mx_rcnn_amd.config import config
from mx_rcnn_amd.core import launch
from mx_rcnn_amd.data.load_data import load_gt_roidb, load_rpn_roidb
from mx_rcnn_amd.data.roidb import prepare_roidb, add_bbox_regression_targets
from mx_rcnn_amd.parallel import dist as pdist
from mx_rcnn_amd.utils.combine_model import combine_model
from tools.test_rpn import test_rpn
from tools.train_rcnn import train_rcnn
from tools.train_rpn import train_rpn


def alternate_train(image_set, test_image_set, year, root_path, devkit_path, pretrained, epoch, ctx, begin_epoch,
                    rpn_epoch, rcnn_epoch, frequent, kv_store, work_load_list=None, network='vgg16',
                    model_dir='model', synthetic=None, max_steps=None, rank=0, world=1):
    config.TRAIN.BG_THRESH_LO = 0.0
    batch_images = config.TRAIN.BATCH_IMAGES
    p = lambda n: os.path.join(model_dir, n)  # noqa: E731
    os.makedirs(model_dir, exist_ok=True)

    def gt():
        if synthetic is not None:
            return synthetic
        return load_gt_roidb(image_set, year, root_path, devkit_path)

    def rpn_roidb(boxes):
        if synthetic is None:
            return load_rpn_roidb(image_set, year, root_path, devkit_path, flip=True)
        imdb, roidb0 = synthetic
        base = [{k: r[k] for k in ('boxes', 'gt_classes', 'gt_overlaps', 'flipped', 'height', 'width',
                                   'synthetic_seed')} for r in roidb0]
        roidb = imdb.merge_roidbs(base, imdb.create_roidb_from_box_list(boxes, base))
        prepare_roidb(imdb, roidb)
        means, stds = add_bbox_regression_targets(roidb)
        return imdb, roidb, means, stds

    logging.info('########## TRAIN RPN WITH IMAGENET INIT')
    config.TRAIN.BATCH_IMAGES = batch_images
    train_rpn(image_set, year, root_path, devkit_path, pretrained, epoch, p('rpn1'), ctx, begin_epoch, rpn_epoch,
              frequent, kv_store, work_load_list, network=network,
              synthetic=None if synthetic is None else (synthetic[1], synthetic[0]), max_steps=max_steps,
              rank=rank, world=world)
    pdist.barrier()
    logging.info('########## GENERATE RPN DETECTION')
    boxes = test_rpn(image_set, year, root_path, devkit_path, p('rpn1'), rpn_epoch, ctx, network=network, imdb_roidb=gt(),
                     dtype=_dump_dtype())
    logging.info('########## TRAIN RCNN WITH IMAGENET INIT AND RPN DETECTION')
    config.TRAIN.BATCH_SIZE = 128
    config.TRAIN.BATCH_IMAGES = batch_images
    train_rcnn(image_set, year, root_path, devkit_path, pretrained, epoch, p('rcnn1'), ctx, begin_epoch,
               rcnn_epoch, frequent, kv_store, work_load_list, network=network, roidb_override=rpn_roidb(boxes),
               max_steps=max_steps, rank=rank, world=world)
    pdist.barrier()
    logging.info('########## TRAIN RPN WITH RCNN INIT')
    config.TRAIN.FINETUNE = True
    config.TRAIN.BATCH_IMAGES = batch_images
    train_rpn(image_set, year, root_path, devkit_path, p('rcnn1'), rcnn_epoch, p('rpn2'), ctx, begin_epoch,
              rpn_epoch, frequent, kv_store, work_load_list, network=network,
              synthetic=None if synthetic is None else (synthetic[1], synthetic[0]), max_steps=max_steps,
              rank=rank, world=world)
    pdist.barrier()
    logging.info('########## GENERATE RPN DETECTION')
    boxes = test_rpn(image_set, year, root_path, devkit_path, p('rpn2'), rpn_epoch, ctx, network=network, imdb_roidb=gt(),
                     dtype=_dump_dtype())
    logging.info('########## COMBINE RPN2 WITH RCNN1')
    if rank == 0:
        combine_model(p('rpn2'), rpn_epoch, p('rcnn1'), rcnn_epoch, p('rcnn2'), 0)
    pdist.barrier()
    logging.info('########## TRAIN RCNN WITH RPN INIT AND DETECTION')
    config.TRAIN.BATCH_SIZE = 128
    config.TRAIN.BATCH_IMAGES = batch_images
    train_rcnn(image_set, year, root_path, devkit_path, p('rcnn2'), 0, p('rcnn2'), ctx, begin_epoch, rcnn_epoch,
               frequent, kv_store, work_load_list, network=network, roidb_override=rpn_roidb(boxes),
               max_steps=max_steps, rank=rank, world=world)
    pdist.barrier()
    logging.info('########## COMBINE RPN2 WITH RCNN2')
    if rank == 0:
        combine_model(p('rpn2'), rpn_epoch, p('rcnn2'), rcnn_epoch, p('final'), 0)
    pdist.barrier()
    return p('final')


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description='Train Faster R-CNN Network with alternate training')
    ap.add_argument('--image_set', default='trainval')
    ap.add_argument('--test_image_set', default='test')
    ap.add_argument('--year', default='2007')
    ap.add_argument('--root_path', default='data')
    ap.add_argument('--devkit_path', default='data/VOCdevkit')
    ap.add_argument('--pretrained', default='model/vgg16')
    ap.add_argument('--epoch', type=int, default=1)
    ap.add_argument('--gpus', default='0')
    ap.add_argument('--begin_epoch', type=int, default=0)
    ap.add_argument('--rpn_epoch', type=int, default=8)
    ap.add_argument('--rcnn_epoch', type=int, default=8)
    ap.add_argument('--frequent', type=int, default=20)
    ap.add_argument('--kv_store', default='device')
    ap.add_argument('--work_load_list', default=None)
    ap.add_argument('--model-dir', dest='model_dir', default='model')
    launch.add_common_args(ap)
    return ap.parse_args(argv)


def _dump_dtype():
    """Precision of the proposal dumps: bf16 when training in bf16, else the reference's fp32."""
    from mx_rcnn_amd.ops import precision
    return 'bf16' if precision.default_name() == 'bf16' else 'fp32'


def main(args):
    rank, world, dev = launch.init_runtime(args)
    syn = None
    if args.synthetic:
        imdb, roidb = launch.synthetic_roidb(args, 21)
        imdb.root_path = args.root_path
        syn = (imdb, roidb)
    return alternate_train(args.image_set, args.test_image_set, args.year, args.root_path, args.devkit_path,
                           args.pretrained, args.epoch, dev, args.begin_epoch, args.rpn_epoch, args.rcnn_epoch,
                           args.frequent, args.kv_store, network=args.network, model_dir=args.model_dir,
                           synthetic=syn, max_steps=args.max_steps, rank=rank, world=world)


if __name__ == '__main__':
    main(parse_args())
