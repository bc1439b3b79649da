#!/usr/bin/env python
"""Training-loss curve of the headline configuration on a fixed synthetic set (precision / learning
check behind BASELINE.md; SURVEY §7.3 success criterion "loss decreasing over ~100 steps").

ResNet-101 C4 Faster R-CNN end-to-end, 800x1333, 81 classes, bf16 compute with fp32 masters and
fp32 gradient sums, graph-replayed steps -- the bench.py step -- on N fixed synthetic images whose
gt boxes are drawn into the image (data/synthetic.py: brighter box regions on textured noise), so
objectness and box regression have signal.  Random-init weights, BN statistics calibrated on the
first image.  Per-step losses stay on the device and are read once at the end.

    python tools/loss_curve.py [--steps 200] [--images 8] [--lr 0.001] [--out profiles/r2_loss_curve.jsonl]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--images', type=int, default=8)
    ap.add_argument('--network', default='resnet101')
    ap.add_argument('--num-classes', type=int, default=81)
    ap.add_argument('--image', default='800x1333')
    ap.add_argument('--lr', type=float, default=0.001)
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'fp32'])
    ap.add_argument('--out', default='')
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
    torch.manual_seed(0)
    model = FasterRCNN(args.network, args.num_classes, cfg=cfg)
    if args.network.startswith('resnet'):
        model.to(dev).calibrate_bn(batches[0]['data'])
    fixed = ['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'] if args.network.startswith('resnet') else ['conv1', 'conv2']
    dtype = torch.bfloat16 if (args.dtype == 'bf16' and dev.type == 'cuda') else torch.float32
    tr = Trainer(model, 'e2e', fixed_param_prefix=fixed, lr=args.lr, momentum=0.9, wd=0.0005, clip_gradient=1.0,
                 compute_dtype=dtype, device=dev)
    step = GraphedStep(tr, batches[0], warmup=2) if dev.type == 'cuda' else tr.step
    hist = []
    for i in range(args.steps):
        out = step(batches[i % len(batches)])
        hist.append(torch.stack([out[k].float().sum() for k in KEYS]).clone())
    vals = torch.stack(hist).cpu().tolist()
    recs = [dict(step=i + 1, **{k: round(v[j], 5) for j, k in enumerate(KEYS)}) for i, v in enumerate(vals)]
    n = max(1, min(20, len(recs) // 5))

    def avg(rs, k):
        return sum(r[k] for r in rs) / len(rs)
    summary = {'network': args.network, 'image_hw': [h, w], 'images': args.images, 'steps': args.steps,
               'lr': args.lr, 'dtype': str(dtype).replace('torch.', ''),
               'first%d' % n: {k: round(avg(recs[:n], k), 4) for k in KEYS},
               'last%d' % n: {k: round(avg(recs[-n:], k), 4) for k in KEYS}}
    if args.out:
        os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
        with open(args.out, 'w') as f:
            f.write(json.dumps({'summary': summary}) + '\n')
            for r in recs:
                f.write(json.dumps(r) + '\n')
    print(json.dumps(summary), flush=True)


if __name__ == '__main__':
    main()
