#!/usr/bin/env python
"""Headline benchmark: images/s of end-to-end (approximate-joint) Faster R-CNN training.

BASELINE.json metric "imgs/sec e2e train ResNet-101 Faster R-CNN at 1/2/4/8 MI355X": ResNet-101
C4 Faster R-CNN, COCO-shaped synthetic images 800x1333 (81 classes), random-init weights,
1 image per GPU per step (the reference's only mode), at the reference's precision by default
(--dtype fp32: every tensor between kernels is the exact fp32 value as a (mid, hi, lo) bf16 triple,
products as six bf16 MFMAs hh+hm+mh+hl+lh+mm with fp32 accumulation, fp32 gradients / BN statistics
/ masters / SGD, mx_rcnn_amd/ops/precision.py); the faster, lower-precision modes are timed after it
and reported as extra fields: ``config.bf16x3`` (16-bit hi / lo pairs, three products) and
``config.bf16`` (bf16 operands) (--dtype bf16x3 / bf16: that mode alone),
full step timed: trunk+RPN fwd/bwd, anchor target, proposal (sort + NMS 12000->6000),
proposal target (128 RoIs), RoIPool, stage-4 head, losses, bucketed RCCL all-reduce (N>1),
fused SGD update.  Weak scaling (fixed per-GPU work).

    python bench.py --gpus N --steps K --warmup W      # spawns N ranks itself (one per GPU)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Rank 0 prints ONE JSON line.  Reference publishes no numbers, so vs_baseline=null.
With N>1 the line also carries the measured per-bucket all-reduce time (``config.allreduce``:
each gradient bucket's collective timed in isolation with HIP events after the timed region).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--network', default='resnet101')
    ap.add_argument('--num-classes', type=int, default=81)
    ap.add_argument('--image', default='800x1333')
    ap.add_argument('--ims-per-gpu', type=int, default=1)
    ap.add_argument('--mode', default='graph', choices=['graph', 'eager'])
    ap.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16x3', 'bf16'],
                    help='fp32 (default): the reference precision (exact fp32 triples), followed by bf16x3 and bf16 '
                         'runs reported as config.bf16x3 / config.bf16; bf16x3 / bf16: that mode alone')
    ap.add_argument('--no-bf16-extra', action='store_true', help='fp32 only: skip the extra bf16x3 / bf16 runs')
    ap.add_argument('--bucket-mb', type=float, default=25)
    ap.add_argument('--grad-comm', default='fp32', choices=['fp32', 'bf16'],
                    help='all-reduce wire dtype of the gradient buckets (fp32 = the reference kvstore sum)')
    ap.add_argument('--pool', type=int, default=4, help='distinct synthetic batches cycled')
    ap.add_argument('--host-float-data', action='store_true',
                    help='feed float network input (converted to the compute dtype outside the step) instead of '
                         'the loaders\' raw uint8 images (converted inside the captured step)')
    ap.add_argument('--train-mode', default='e2e', choices=['e2e', 'rpn', 'rcnn'],
                    help='e2e (headline) or one stage of 4-step alternate training (BASELINE config 4): '
                         'rpn = RPN-only step, rcnn = Fast R-CNN step on 128 given RoIs per image')
    return ap.parse_args(argv)


if __name__ == '__main__':
    # before anything touches the GPU: --gpus N without a launcher -> N fresh rank processes
    from mx_rcnn_amd.parallel.spawn import maybe_spawn
    maybe_spawn(parse_args().gpus, os.path.abspath(__file__), sys.argv[1:])

import torch  # noqa: E402

from mx_rcnn_amd.config import snapshot  # noqa: E402
from mx_rcnn_amd.models import FasterRCNN  # noqa: E402
from mx_rcnn_amd.parallel import dist as pdist  # noqa: E402
from mx_rcnn_amd.core.trainer import Trainer, GraphedStep  # noqa: E402

METRIC = 'imgs/sec e2e train ResNet-101 Faster R-CNN'
PRECISION_NOTE = {
    'fp32': 'fp32: every tensor between kernels is the exact fp32 value as a (mid, hi, lo) bf16 triple (24 '
            'significant bits), products hh+hm+mh+hl+lh+mm on the bf16 MFMA with fp32 accumulation, fp32 '
            'grads/BN statistics/masters/SGD',
    'bf16x3': 'bf16x3: MFMA operands and stored tensors as bf16 hi/lo pairs (16 significant bits), '
              'hi*hi+hi*lo+lo*hi with fp32 accumulation, fp32 grads/masters/SGD',
    'bf16': 'bf16 operands, fp32 accumulation and masters',
}


def synthetic_batch(n_img, h, w, num_classes, device, gen, max_gt=20, raw=False, pixel_means=None):
    """raw=True: the training loaders' raw-image form (uint8 BGR (n, h, w, 3) + pixel_means,
    data/loader.py raw_images), converted inside the captured step by csrc/hip/image.hip; else
    float (n, 3, h, w) network input."""
    if raw:
        data = torch.randint(0, 256, (n_img, h, w, 3), generator=gen, dtype=torch.uint8)
    else:
        data = torch.randn(n_img, 3, h, w, generator=gen) * 50.0
    G = max_gt
    gt = torch.full((n_img, G, 5), -1.0)
    n_gt = torch.randint(1, G + 1, (n_img,), generator=gen).to(torch.int32)
    for b in range(n_img):
        k = int(n_gt[b])
        bw = torch.randint(32, 400, (k,), generator=gen).float()
        bh = torch.randint(32, 400, (k,), generator=gen).float()
        x1 = (torch.rand(k, generator=gen) * (w - bw - 1)).floor()
        y1 = (torch.rand(k, generator=gen) * (h - bh - 1)).floor()
        cls = torch.randint(1, num_classes, (k,), generator=gen).float()
        gt[b, :k] = torch.stack([x1, y1, x1 + bw, y1 + bh, cls], dim=1)
    im_info = torch.tensor([[float(h), float(w), 1.0]] * n_img)
    out = {'data': data.to(device), 'im_info': im_info.to(device), 'gt_boxes': gt.to(device), 'n_gt': n_gt.to(device)}
    if raw:
        pm = (0.0, 0.0, 0.0) if pixel_means is None else torch.as_tensor(pixel_means, dtype=torch.float64).reshape(-1)[:3]
        out['pixel_means'] = tuple(float(m) for m in pm)
    return out


def network_input(b):
    """The float (n, 3, h, w) image a batch feeds the network (raw batches converted as in the step)."""
    if b['data'].dtype != torch.uint8:
        return b['data']
    from mx_rcnn_amd.ops.image import image_prep
    return image_prep(b['data'], b['im_info'], b['pixel_means'], torch.float32, channels_last=False)


def rcnn_batch(b, num_classes, rois_per_image, gen, fg_fraction=0.25):
    """A Fast R-CNN step input of the alternate scheme's shape (tools/train_rcnn.py): per image
    ``rois_per_image`` RoIs (the proposal-target sample of precomputed proposals), fg first with
    one class-specific regression target each, background after."""
    n, h, w = network_input(b).shape[0], b['im_info'][0, 0], b['im_info'][0, 1]
    h, w = int(h), int(w)
    R = n * rois_per_image
    wh = torch.rand(R, 2, generator=gen) * min(300.0, 0.5 * min(h, w)) + 16
    x1 = torch.rand(R, generator=gen) * (w - wh[:, 0] - 1)
    y1 = torch.rand(R, generator=gen) * (h - wh[:, 1] - 1)
    img = torch.arange(n).repeat_interleave(rois_per_image).float()
    rois = torch.stack([img, x1, y1, x1 + wh[:, 0], y1 + wh[:, 1]], 1)
    label = torch.zeros(n, rois_per_image, dtype=torch.int32)
    nfg = int(rois_per_image * fg_fraction)
    label[:, :nfg] = torch.randint(1, num_classes, (n, nfg), generator=gen).to(torch.int32)
    label = label.reshape(-1)
    tgt = torch.zeros(R, 4 * num_classes)
    inside = torch.zeros(R, 4 * num_classes)
    fg = (label > 0).nonzero().reshape(-1)
    cols = (4 * label[fg].long()).unsqueeze(1) + torch.arange(4)
    tgt[fg.unsqueeze(1), cols] = torch.randn(len(fg), 4, generator=gen) * 0.5
    inside[fg.unsqueeze(1), cols] = 1.0
    dev = b['data'].device
    extra = {k: b[k] for k in ('im_info', 'pixel_means') if b['data'].dtype == torch.uint8}
    return {**extra, 'data': b['data'], 'rois': rois.to(dev), 'label': label.to(dev), 'bbox_target': tgt.to(dev),
            'bbox_inside_weight': inside.to(dev), 'bbox_outside_weight': inside.clone().to(dev)}


def main():
    args = parse_args()
    rank, world, local_rank, device = pdist.init_distributed()
    if world != args.gpus:
        raise SystemExit('--gpus %d but %d ranks were launched' % (args.gpus, world))
    rec = run(args, args.dtype, rank, world, device)
    if args.dtype == 'fp32' and not args.no_bf16_extra and device.type == 'cuda':
        for name in ('bf16x3', 'bf16'):
            torch.cuda.empty_cache()
            extra = run(args, name, rank, world, device)
            rec['config'][name] = {'value': extra['value'], 'ms_per_step': extra['ms_per_step'],
                                   'exec': extra['config']['exec'],
                                   'objective_first_last': extra['config']['objective_first_last']}
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if os.environ.get('MXR_BENCH_DUMP_TUNE') and device.type == 'cuda':
        from mx_rcnn_amd.ops import need_ext
        for key, tile, sp in need_ext().conv_tune_table():
            print('[tune] %-48s tile %d splits %d' % (key, tile, sp), file=sys.stderr)
    if device.type == 'cuda' and rank == 0:  # persist the conv plan for the next run (ops/tune_plan.py)
        from mx_rcnn_amd.ops import tune_plan
        tune_plan.save()
    pdist.destroy()


def run(args, precision, rank, world, device):
    """One timed run at ``precision`` ('fp32' triples, 'bf16x3' pairs, 'bf16') -> the JSON record."""
    h, w = [int(v) for v in args.image.lower().split('x')]
    cfg = snapshot()
    # end2end config mutation (train_end2end.py:25-32)
    if args.train_mode == 'e2e':
        cfg.TRAIN.BG_THRESH_LO = 0.0
        cfg.TRAIN.HAS_RPN = True
        cfg.END2END = 1
        cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    elif args.train_mode == 'rpn':  # tools/train_rpn.py
        cfg.TRAIN.HAS_RPN = True
        cfg.END2END = 0
    cfg.TRAIN.IMS_PER_BATCH = args.ims_per_gpu
    torch.manual_seed(1234 + rank)
    model = FasterRCNN(args.network, args.num_classes, cfg=cfg)
    gen = torch.Generator().manual_seed(4321 + rank)
    raw = not args.host_float_data
    pool = [synthetic_batch(args.ims_per_gpu, h, w, args.num_classes, device, gen, raw=raw,
                            pixel_means=cfg.PIXEL_MEANS) for _ in range(args.pool)]
    if args.train_mode == 'rcnn':
        pool = [rcnn_batch(b, args.num_classes, cfg.TRAIN.BATCH_SIZE, gen) for b in pool]
    if args.network.startswith('resnet'):
        model.to(device).calibrate_bn(network_input(pool[0]))  # stand-in for pretrained BN statistics
    else:
        model.to(device).calibrate_vgg(network_input(pool[0]))  # stand-in for pretrained filters (LSUV scale)
    fixed = ['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'] if args.network.startswith('resnet') else ['conv1', 'conv2']
    trainer = Trainer(model, args.train_mode, fixed_param_prefix=fixed, lr=0.001, momentum=0.9, wd=0.0005, clip_gradient=1.0,
                      rescale_grad=1.0, device=device, bucket_mb=args.bucket_mb, precision=precision,
                      grad_comm_dtype=torch.float32 if args.grad_comm == 'fp32' else torch.bfloat16)

    mode = args.mode if device.type == 'cuda' else 'eager'
    step_fn = None
    if mode == 'graph':
        ok = 1.0
        try:
            g = GraphedStep(trainer, pool[0], warmup=3)
            step_fn = g
        except Exception as e:  # reported, never silent
            ok = 0.0
            print('[bench] rank %d: hipGraph capture failed (%s: %s)' % (rank, type(e).__name__, str(e)[:300]),
                  file=sys.stderr)
            torch.cuda.synchronize()
        # every rank must take the same path (collectives are inside the captured step)
        if -pdist.all_reduce_max(-ok, device) < 1.0:
            if rank == 0:
                print('[bench] falling back to eager execution on all ranks', file=sys.stderr)
            mode, step_fn = 'eager', None
    if step_fn is None:
        step_fn = trainer.step

    def sync():
        if device.type == 'cuda':
            torch.cuda.synchronize()

    for i in range(args.warmup):
        out = step_fn(pool[i % len(pool)])
    sync()
    loss0 = float(out['objective'].float().item()) if args.warmup else float('nan')
    pdist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        out = step_fn(pool[i % len(pool)])
    sync()
    pdist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    elapsed = pdist.all_reduce_max(elapsed, device)
    loss1 = float(out['objective'].float().item())
    plan = None
    if device.type == 'cuda':  # the conv plan the timed step ran with, and whether the ranks agree
        from mx_rcnn_amd.ops import tune_plan
        ph = int(tune_plan.plan_hash(), 16)
        plan = {'hash': '%08x' % ph, 'entries': len(tune_plan.table()),
                'ranks_agree': pdist.all_reduce_max(float(ph), device) == -pdist.all_reduce_max(-float(ph), device)}
    # after the timed region: each gradient bucket's collective in isolation (HIP events)
    comm = trainer.reducer.measure_collectives() if world > 1 else None
    replicas = None
    if world > 1:  # data-parallel replicas must hold bitwise-equal weights after the timed steps
        dg = float(trainer.store.weights_digest())
        replicas = {'digest': '%08x' % int(dg),
                    'agree': pdist.all_reduce_max(dg, device) == -pdist.all_reduce_max(-dg, device)}
    ms = elapsed / max(args.steps, 1) * 1e3
    imgs = args.ims_per_gpu * world * args.steps
    value = imgs / elapsed
    metric = METRIC if args.network == 'resnet101' else 'imgs/sec e2e train %s Faster R-CNN' % args.network
    if args.train_mode != 'e2e':
        metric = 'imgs/sec alternate-stage %s train %s' % (args.train_mode, args.network)
    rec = {'metric': metric, 'value': round(value, 3), 'unit': 'images/s', 'n_gpus': world,
           'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms, 3),
           'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
           'dtype': trainer.precision,
           'data': 'synthetic (random %dx%d %s images, 1-20 random gt boxes, random-init weights)' % (
               h, w, 'float' if args.host_float_data else 'uint8 BGR (raw-loader form, converted in the step)'),
           'config': {'model': '%s-faster-rcnn%s' % (args.network, '-c4' if args.network.startswith('resnet') else ''), 'global_batch': args.ims_per_gpu * world,
                      'seq_len': None, 'image_hw': [h, w], 'num_classes': args.num_classes,
                      'ims_per_gpu': args.ims_per_gpu, 'train_mode': args.train_mode, 'parallelism': 'dp%d' % world,
                      'precision': PRECISION_NOTE.get(trainer.precision, trainer.precision),
                      'rpn_pre_post_nms': [cfg.TRAIN.RPN_PRE_NMS_TOP_N, cfg.TRAIN.RPN_POST_NMS_TOP_N],
                      'rois_per_image': cfg.TRAIN.BATCH_SIZE, 'exec': mode,
                      'objective_first_last': [round(loss0, 4), round(loss1, 4)],
                      'backend': pdist.backend_name(), 'allreduce': comm, 'conv_plan': plan,
                      'replicas': replicas,
                      'rccl': pdist.rccl_env() if pdist.backend_name() == 'nccl' else None,
                      'hip_runtime': __import__('mx_rcnn_amd').runtime_settings()}}
    del step_fn, trainer
    return rec


if __name__ == '__main__':
    main()
