#!/usr/bin/env python
"""BASELINE.json config 1: VGG16 RPN-only forward on the CPU, one synthetic 600x1000 image
(the reference's plumbing configuration, `rcnn/symbol.py` get_vgg_rpn_test + `tools/test_rpn.py`:
trunk conv1_1..conv5_3 -> RPN head -> Proposal with TEST settings 6000 -> NMS 0.7 -> 300 RoIs).
fp32, random-init weights, no GPU.

    python bench_rpn_cpu.py [--steps K --warmup W --threads T]

Prints one JSON line; the metric is time-like (ms per image, lower is better).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from mx_rcnn_amd.config import snapshot  # noqa: E402
from mx_rcnn_amd.models import FasterRCNN  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--threads', type=int, default=0, help='intra-op threads (0 = torch default)')
    ap.add_argument('--image', default='600x1000')
    ap.add_argument('--channels-last', type=int, default=1)
    args = ap.parse_args()
    if args.threads:
        torch.set_num_threads(args.threads)
    h, w = [int(v) for v in args.image.lower().split('x')]
    torch.manual_seed(0)
    model = FasterRCNN('vgg16', 21, cfg=snapshot()).eval()
    x = torch.randn(1, 3, h, w)
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
    info = torch.tensor([[float(h), float(w), 1.0]])
    with torch.no_grad():
        for _ in range(args.warmup):
            rois, scores = model.rpn_test(x, info)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            rois, scores = model.rpn_test(x, info)
        el = time.perf_counter() - t0
    ms = el / max(args.steps, 1) * 1e3
    print(json.dumps({'metric': 'ms/image VGG16 RPN-only forward CPU', 'value': round(ms, 2), 'unit': 'ms/image',
                      'n_gpus': 0, 'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms, 2),
                      'higher_is_better': False, 'scaling': None, 'vs_baseline': None, 'dtype': 'fp32',
                      'data': 'synthetic (random %dx%d image, random-init weights)' % (h, w),
                      'config': {'model': 'vgg16-rpn', 'image_hw': [h, w], 'threads': torch.get_num_threads(),
                                 'channels_last': bool(args.channels_last), 'rois': list(rois.shape)}}),
          flush=True)


if __name__ == '__main__':
    main()
