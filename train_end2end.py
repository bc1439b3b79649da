#!/usr/bin/env python
"""Approximate-joint end-to-end Faster R-CNN training (reference `train_end2end.py`).

    python train_end2end.py --image_set trainval --year 2007 --prefix model/e2e --network vgg16
    torchrun --nproc-per-node 8 train_end2end.py --network resnet101 ...   # one process per GPU
    python train_end2end.py --synthetic 64 --network resnet50 --max-steps 20   # no dataset needed
"""
import argparse
import logging

from mx_rcnn_amd.config import config
from mx_rcnn_amd.core import launch
from mx_rcnn_amd.core.callback import Speedometer
from mx_rcnn_amd.core.metric import e2e_metrics
from mx_rcnn_amd.core.module import MutableModule
from mx_rcnn_amd.data.load_data import load_gt_roidb
from mx_rcnn_amd.data.loader import AnchorLoader
from mx_rcnn_amd.parallel import dist as pdist
from mx_rcnn_amd.utils.load_model import do_checkpoint, states_file
from mx_rcnn_amd.utils.monitor import Monitor


def end2end_train(args):
    rank, world, device = launch.init_runtime(args)
    logging.info('########## TRAIN FASTER-RCNN WITH APPROXIMATE JOINT END2END #############')
    launch.e2e_config()
    model, arg_params, aux_params = launch.build_model(args.network, args.num_classes, args.pretrained,
                                                       args.load_epoch, args.resume, train_mode='e2e')
    # the graph was built with per-image sizes; the global counts scale with #GPUs (train_end2end.py:37-38)
    config.TRAIN.IMS_PER_BATCH = args.ims_per_gpu
    if args.synthetic:
        imdb, roidb = launch.synthetic_roidb(args, args.num_classes, flip=not args.no_flip)
    else:
        imdb, roidb = load_gt_roidb(args.image_set, args.year, args.root_path, args.devkit_path,
                                    flip=not args.no_flip)
    fam = launch.family(args.network)
    scales = model.anchor_scales
    # pixel means subtracted for every backbone, as the reference's AnchorLoader default does
    # (`train_end2end.py:56`, `rcnn/loader.py:148`) and as the test loaders do
    train_data = AnchorLoader(model, roidb, batch_size=args.ims_per_gpu, shuffle=True, mode='train',
                              anchor_scales=scales, rank=rank, world_size=world, seed=args.seed,
                              work_load_list=args.work_load_list,
                              raw_images=launch.raw_images(device))
    launch.calibrate_if_random(model, train_data, arg_params)
    mod = MutableModule(model, data_names=['data', 'im_info'], label_names=['gt_boxes'], context=device,
                        fixed_param_prefix=launch.FIXED_PREFIX[fam], mode='e2e', use_graph=not args.eager)
    monitor = Monitor(100) if args.monitor else None
    mod.fit(train_data, eval_metric=e2e_metrics(), epoch_end_callback=do_checkpoint(args.prefix), monitor=monitor,
            batch_end_callback=Speedometer(train_data.global_batch_size, frequent=args.frequent),
            kvstore=args.kv_store, optimizer='sgd',
            optimizer_params=launch.optimizer_params(args.lr, args.mom, args.wd, args.factor_step, args.resume),
            arg_params=arg_params, aux_params=aux_params, begin_epoch=args.load_epoch, num_epoch=args.num_epoch,
            max_steps=args.max_steps, states_prefix=args.prefix,
            resume_states=states_file(args.pretrained, args.load_epoch) if args.resume else None)
    pdist.destroy()
    return mod


def parse_args(argv=None):
    p = argparse.ArgumentParser(description='Train Faster R-CNN network end to end')
    p.add_argument('--image_set', default='trainval')
    p.add_argument('--num-classes', dest='num_classes', type=int, default=21)
    p.add_argument('--test_image_set', default='test')
    p.add_argument('--year', default='2007')
    p.add_argument('--root_path', default='data')
    p.add_argument('--devkit_path', default='data/VOCdevkit')
    p.add_argument('--no-flip', dest='no_flip', action='store_true')
    p.add_argument('--pretrained', default='model/vgg16')
    p.add_argument('--load-epoch', dest='load_epoch', type=int, default=0)
    p.add_argument('--prefix', default='model/faster-rcnn')
    p.add_argument('--gpus', default='0', help='GPU list "0,1,2,3" or count: one process per GPU (or use torchrun)')
    p.add_argument('--num_epoch', type=int, default=7)
    p.add_argument('--frequent', type=int, default=20)
    p.add_argument('--kv_store', default='device')
    p.add_argument('--work_load_list', default=None, help='per-GPU share of the global batch, e.g. "1,1,2,2"')
    p.add_argument('--lr', type=float, default=0.001)
    p.add_argument('--mom', type=float, default=0.9)
    p.add_argument('--wd', type=float, default=0.0005)
    p.add_argument('--resume', action='store_true')
    p.add_argument('--factor-step', dest='factor_step', type=int, default=50000)
    p.add_argument('--monitor', action='store_true')
    launch.add_common_args(p)
    return p.parse_args(argv)


if __name__ == '__main__':
    end2end_train(parse_args())
