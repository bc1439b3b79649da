#!/usr/bin/env python
"""Training-loss curve of the headline configuration on a fixed synthetic set (precision / learning
check behind BASELINE.md; SURVEY §7.3 success criterion "loss decreasing over ~100 steps").

ResNet-101 C4 Faster R-CNN end-to-end, 800x1333, 81 classes, bf16 compute with fp32 masters and
fp32 gradient sums, graph-replayed steps -- the bench.py step -- on N fixed synthetic images whose
gt boxes are drawn into the image (data/synthetic.py: brighter box regions on textured noise), so
objectness and box regression have signal.  Random-init weights, BN statistics calibrated on the
first image.  Per-step losses stay on the device and are read once at the end.

    python tools/loss_curve.py [--steps 200] [--images 8] [--lr 0.001] [--dtype fp32] [--out profiles/....jsonl]
    python tools/loss_curve.py --train-mode rcnn ...   # Fast R-CNN head on FIXED RoIs per image

``--train-mode rcnn`` isolates the detection head: every image gets a fixed set of 128 RoIs (32
jittered copies of its gt boxes, IoU >= 0.5 with their box, and 96 background boxes) with their
labels and normalised class-specific regression targets, so the head's cls / bbox losses can
only fall if its gradients are right.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mx_rcnn_amd.config import config, snapshot  # noqa: E402
from mx_rcnn_amd.core.trainer import GraphedStep, Trainer  # noqa: E402
from mx_rcnn_amd.data.loader import AnchorLoader  # noqa: E402
from mx_rcnn_amd.data.synthetic import SyntheticDetection  # noqa: E402
from mx_rcnn_amd.models import FasterRCNN  # noqa: E402

KEYS = ('objective', 'rpn_cls_loss', 'rpn_bbox_loss', 'cls_loss', 'bbox_loss')


def _fixed_rois(b, num_classes, cfg, seed, R=128, n_fg=32):
    """A fixed Fast R-CNN minibatch for one loader batch: gt-jittered fg RoIs, random bg RoIs."""
    from mx_rcnn_amd.ops.boxes import bbox_transform, box_iou
    g = torch.Generator().manual_seed(100 + seed)
    dev = b['data'].device
    gt = b['gt_boxes'][0].cpu()
    gt = gt[:int(b['n_gt'][0])] if 'n_gt' in b else gt[gt[:, 4] > 0]
    H, W = int(b['im_info'][0, 0]), int(b['im_info'][0, 1])
    pick = torch.randint(0, len(gt), (n_fg,), generator=g)
    base = gt[pick, :4]
    wh = (base[:, 2:] - base[:, :2]).repeat(1, 2)
    fg = base + (torch.rand(n_fg, 4, generator=g) - 0.5) * 0.15 * wh
    lab_fg = gt[pick, 4].long()
    bg = []
    while len(bg) < R - n_fg:
        xy = torch.rand(2, generator=g) * torch.tensor([W - 40.0, H - 40.0])
        box = torch.cat([xy, xy + torch.rand(2, generator=g) * 160 + 24]).clamp(max=max(W, H) - 1.0)
        if float(box_iou(box[None], gt[:, :4]).max()) < 0.3:
            bg.append(box)
    rois = torch.cat([fg, torch.stack(bg)], 0)
    rois = torch.cat([torch.zeros(R, 1), rois], 1)
    label = torch.cat([lab_fg, torch.zeros(R - n_fg, dtype=torch.long)]).to(torch.int32)
    tg = bbox_transform(fg, base)
    means = torch.tensor(cfg.TRAIN.BBOX_MEANS, dtype=torch.float32)
    stds = torch.tensor(cfg.TRAIN.BBOX_STDS, dtype=torch.float32)
    tg = (tg - means) / stds
    tgt = torch.zeros(R, 4 * num_classes)
    inside = torch.zeros(R, 4 * num_classes)
    cols = (4 * lab_fg).unsqueeze(1) + torch.arange(4)
    tgt[torch.arange(n_fg).unsqueeze(1), cols] = tg
    inside[torch.arange(n_fg).unsqueeze(1), cols] = 1.0
    return {'data': b['data'], 'rois': rois.to(dev), 'label': label.to(dev), 'bbox_target': tgt.to(dev),
            'bbox_inside_weight': inside.to(dev), 'bbox_outside_weight': inside.clone().to(dev)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--images', type=int, default=8)
    ap.add_argument('--network', default='resnet101')
    ap.add_argument('--num-classes', type=int, default=81)
    ap.add_argument('--image', default='800x1333')
    ap.add_argument('--lr', type=float, default=0.001)
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'bf16x3', 'fp32'])
    ap.add_argument('--out', default='')
    ap.add_argument('--train-mode', default='e2e', choices=['e2e', 'rcnn'])
    args = ap.parse_args()
    dev = torch.device('cuda', 0) if torch.cuda.is_available() else torch.device('cpu')
    h, w = [int(v) for v in args.image.split('x')]
    cfg = snapshot()
    cfg.TRAIN.BG_THRESH_LO = 0.0
    cfg.TRAIN.HAS_RPN = True
    cfg.END2END = 1
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    config.SCALES = (min(h, w),)
    config.MAX_SIZE = max(h, w)
    imdb = SyntheticDetection(args.images, h, w, args.num_classes, max_gt=20, seed=7)
    loader = AnchorLoader(None, imdb.gt_roidb(), 1, shuffle=False, pad_shape=(h, w), max_gt=32, prefetch=1,
                          workers=1, need_mean=False)
    batches = [{k: v.to(dev) for k, v in b.items()} for b in loader]
    loader.close()
    if args.train_mode == 'rcnn':
        batches = [_fixed_rois(b, args.num_classes, cfg, i) for i, b in enumerate(batches)]
    torch.manual_seed(0)
    model = FasterRCNN(args.network, args.num_classes, cfg=cfg)
    if args.network.startswith('resnet'):
        model.to(dev).calibrate_bn(batches[0]['data'])
    fixed = ['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'] if args.network.startswith('resnet') else ['conv1', 'conv2']
    tr = Trainer(model, args.train_mode, fixed_param_prefix=fixed, lr=args.lr, momentum=0.9, wd=0.0005,
                 clip_gradient=1.0, device=dev, precision=args.dtype)
    dtype = tr.precision
    keys = KEYS if args.train_mode == 'e2e' else ('objective', 'cls_loss', 'bbox_loss')
    step = GraphedStep(tr, batches[0], warmup=2) if dev.type == 'cuda' else tr.step
    hist = []
    for i in range(args.steps):
        out = step(batches[i % len(batches)])
        hist.append(torch.stack([out[k].float().sum() for k in keys]).clone())
    vals = torch.stack(hist).cpu().tolist()
    recs = [dict(step=i + 1, **{k: round(v[j], 5) for j, k in enumerate(keys)}) for i, v in enumerate(vals)]
    n = max(1, min(20, len(recs) // 5))

    def avg(rs, k):
        return sum(r[k] for r in rs) / len(rs)
    summary = {'network': args.network, 'image_hw': [h, w], 'images': args.images, 'steps': args.steps,
               'lr': args.lr, 'dtype': dtype, 'train_mode': args.train_mode,
               'first%d' % n: {k: round(avg(recs[:n], k), 4) for k in keys},
               'last%d' % n: {k: round(avg(recs[-n:], k), 4) for k in keys}}
    if args.out:
        os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
        with open(args.out, 'w') as f:
            f.write(json.dumps({'summary': summary}) + '\n')
            for r in recs:
                f.write(json.dumps(r) + '\n')
    print(json.dumps(summary), flush=True)


if __name__ == '__main__':
    main()
