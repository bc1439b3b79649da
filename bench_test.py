#!/usr/bin/env python
"""Inference benchmark: test-time images/s (FPS) of Faster R-CNN (BASELINE.json headline
"...; test FPS").  ResNet-101 C4 by default, COCO-shaped 800x1333 synthetic images, 81 classes,
random-init weights (BN statistics calibrated on the data), bf16 (--dtype fp32: the reference's
precision as exact three-plane bf16 operands on our kernels; fp16), batch 1 per GPU, TEST config
(RPN 6000 -> 300 proposals, NMS 0.7; per-class score > 0.05, NMS 0.3, top-100).

Timed per image: trunk + RPN + proposal + RoIPool + head (one replayed hipGraph by default)
+ box decode / clip / per-class threshold / batched NMS / top-k on the device, i.e. everything
``tester.pred_eval`` does except image decoding and file IO.  N>1: one process per GPU
(torchrun), each runs its own image stream; value = total images/s over all ranks.

    python bench_test.py [--gpus N --steps K --warmup W --mode graph|eager --network resnet101]
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
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--network', default='resnet101')
    ap.add_argument('--num-classes', type=int, default=81)
    ap.add_argument('--image', default='800x1333')
    ap.add_argument('--mode', default='graph', choices=['graph', 'eager'])
    ap.add_argument('--batch', type=int, default=1, help='images per forward per GPU (BASELINE config 5: 8)')
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'fp16', 'fp32'],
                    help='precision of the test graph (fp16: BASELINE config 5; fp32: the reference\'s, three '
                         'bf16 planes per operand on the MFMA kernels)')
    ap.add_argument('--plant', type=int, default=10,
                    help='classes whose cls_score bias is raised so random-init weights produce detections above '
                         'the 0.05 threshold (the NMS / top-k post-process then has real work); 0 = off')
    return ap.parse_args(argv)


if __name__ == '__main__':
    from mx_rcnn_amd.parallel.spawn import maybe_spawn
    maybe_spawn(parse_args().gpus, os.path.abspath(__file__), sys.argv[1:])

import torch  # noqa: E402

from mx_rcnn_amd.config import config, snapshot  # noqa: E402
from mx_rcnn_amd.core.detector import Detector  # noqa: E402
from mx_rcnn_amd.models import FasterRCNN  # noqa: E402
from mx_rcnn_amd.parallel import dist as pdist  # noqa: E402

METRIC = 'test FPS ResNet-101 Faster R-CNN'


class GraphedDetect:
    """model.detect captured once for a fixed input shape and replayed."""

    def __init__(self, det, data, im_info, warmup=2):
        self.det = det
        self.data = data.clone()
        self.info = im_info.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), torch.no_grad():
            for _ in range(warmup):
                det.detect(self.data, self.info)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph), torch.no_grad():
            self.out = det.detect(self.data, self.info)
        torch.cuda.synchronize()

    def __call__(self, data, im_info):
        self.data.copy_(data, non_blocking=True)
        self.info.copy_(im_info, non_blocking=True)
        self.graph.replay()
        return self.out


def main():
    args = parse_args()
    rank, world, local_rank, device = pdist.init_distributed()
    if world != args.gpus:
        raise SystemExit('--gpus %d but %d ranks were launched' % (args.gpus, world))
    h, w = [int(v) for v in args.image.lower().split('x')]
    torch.manual_seed(1234 + rank)
    model = FasterRCNN(args.network, args.num_classes, cfg=snapshot(), train_mode='test')
    gen = torch.Generator().manual_seed(99 + rank)
    nb = args.batch
    pool = [(torch.randn(nb, 3, h, w, generator=gen) * 50.0) for _ in range(4)]
    info = torch.tensor([[float(h), float(w), 1.0]] * nb)
    if args.network.startswith('resnet'):
        model.to(device).calibrate_bn(pool[0][:1].to(device))
    if args.plant:
        with torch.no_grad():  # synthetic "confident" classes: softmax mass well above 0.05 on them
            model.head.cls_score.bias[1:1 + args.plant] += 6.0
    cdt = args.dtype if device.type == 'cuda' else 'fp32'
    det = Detector(model, device, compute_dtype=cdt)
    dev_pool = [det._prep(x) for x in pool]
    dinfo = info.to(device)
    run = None
    mode = args.mode if device.type == 'cuda' else 'eager'
    if mode == 'graph':
        try:
            run = GraphedDetect(det, dev_pool[0], dinfo)
        except Exception as e:  # reported, never silent
            print('[bench_test] graph capture failed (%s): %s' % (type(e).__name__, str(e)[:300]), file=sys.stderr)
            mode = 'eager'
    if run is None:
        def run(x, i):
            with torch.no_grad():
                return det.detect(x, i)

    use_dev = device.type == 'cuda'

    def one(i):
        r, scores, deltas = run(dev_pool[i % len(dev_pool)], dinfo)
        if use_dev and det.device_postprocess_ok(r, scores, dinfo):
            # decode + clip + threshold + per-class NMS + top-100 as two launches, no host sync
            return det.postprocess_raw(r, scores, deltas, dinfo, config.TEST.NMS, 0.05, 100)
        return det.postprocess(r, scores, deltas, dinfo, config.TEST.NMS, 0.05, 100)

    def sync():
        if device.type == 'cuda':
            torch.cuda.synchronize()

    for i in range(args.warmup):
        res = one(i)
    sync()
    pdist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        res = one(i)
    sync()
    pdist.barrier()
    sync()
    elapsed = pdist.all_reduce_max(time.perf_counter() - t0, device)
    if isinstance(res, (tuple, list)) and len(res) == 2 and torch.is_tensor(res[1]) and res[1].dim() == 1 and \
            res[1].dtype == torch.int32:
        n_det = int(res[1][-1].item())  # detections of the last image of the last batch
    else:
        n_det = int(res[-1][1].numel())
    if rank == 0:
        value = world * nb * args.steps / elapsed
        print(json.dumps({
            'metric': METRIC if args.network == 'resnet101' else 'test FPS %s Faster R-CNN' % args.network, 'value': round(value, 3), 'unit': 'images/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': args.dtype if device.type == 'cuda' else 'fp32',
            'data': 'synthetic (random %dx%d images, random-init weights, BN calibrated, %d planted classes)' % (
                h, w, args.plant),
            'config': {'model': '%s-faster-rcnn%s' % (args.network, '-c4' if args.network.startswith('resnet') else ''), 'global_batch': world * nb, 'ims_per_gpu': nb,
                       'image_hw': [h, w],
                       'num_classes': args.num_classes, 'parallelism': 'dp%d' % world, 'exec': mode,
                       'rpn_pre_post_nms': [config.TEST.RPN_PRE_NMS_TOP_N, config.TEST.RPN_POST_NMS_TOP_N],
                       'detections_last_image': n_det}}), flush=True)
    if os.environ.get('MXR_BENCH_DUMP_TUNE') and device.type == 'cuda':
        from mx_rcnn_amd.ops import need_ext
        for key, tile, sp in need_ext().conv_tune_table():
            print('[tune] %-48s tile %d splits %d' % (key, tile, sp), file=sys.stderr)
    if device.type == 'cuda' and rank == 0:  # persist the conv plan for the next run (ops/tune_plan.py)
        from mx_rcnn_amd.ops import tune_plan
        tune_plan.save()
    pdist.destroy()


if __name__ == '__main__':
    main()
