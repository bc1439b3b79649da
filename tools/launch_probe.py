"""Is the graphed training step bound by the GPU or by the host's graph submission?

Times, for the bench.py ResNet-101 step under GraphedStep:
  * gpu     -- ms/step of back-to-back replays (synchronised once at the end);
  * host    -- ms/step the host spends inside the replay calls of that same loop;
  * single  -- ms of one replay synchronised on its own (launch latency + GPU time);
  * enqueue_behind_busy -- host ms of one replay call issued while the GPU is busy (submission
    cost alone, no back-pressure from the previous replay).
A host time close to the gpu time means the step is submission-bound.

    python tools/launch_probe.py [--steps 50] [--precision fp32|bf16]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from mx_rcnn_amd.config import snapshot  # noqa: E402
from mx_rcnn_amd.core.trainer import GraphedStep, Trainer  # noqa: E402
from mx_rcnn_amd.models.faster_rcnn import FasterRCNN  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--network', default='resnet101')
    ap.add_argument('--precision', default='fp32', choices=['fp32', 'bf16'],
                    help="'fp32': the fp32-class x2 step (bench.py's default), 'bf16'")
    args = ap.parse_args()
    dev = torch.device('cuda:0')
    cfg = snapshot()
    cfg.TRAIN.BG_THRESH_LO = 0.0
    cfg.TRAIN.HAS_RPN = True
    cfg.END2END = 1
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    torch.manual_seed(1234)
    model = FasterRCNN(args.network, 81, cfg=cfg)
    gen = torch.Generator().manual_seed(4321)
    batch = bench.synthetic_batch(1, 800, 1333, 81, dev, gen)
    model.to(dev).calibrate_bn(batch['data'])
    tr = Trainer(model, 'e2e', fixed_param_prefix=['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'], lr=0.001,
                 momentum=0.9, wd=0.0005, clip_gradient=1.0, rescale_grad=1.0, device=dev, precision=args.precision)
    g = GraphedStep(tr, batch, warmup=3)
    for _ in range(5):
        g(batch)
    torch.cuda.synchronize()
    host = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = time.perf_counter()
        g(batch)
        host += time.perf_counter() - a
    torch.cuda.synchronize()
    gpu = (time.perf_counter() - t0) / args.steps
    singles = []
    for _ in range(10):
        torch.cuda.synchronize()
        a = time.perf_counter()
        g(batch)
        torch.cuda.synchronize()
        singles.append(time.perf_counter() - a)
    # bare graph replay (no input copies)
    torch.cuda.synchronize()
    h2 = 0.0
    t1 = time.perf_counter()
    for _ in range(args.steps):
        a = time.perf_counter()
        g.graph.replay()
        h2 += time.perf_counter() - a
    torch.cuda.synchronize()
    gpu2 = (time.perf_counter() - t1) / args.steps
    # pure submission cost: one replay enqueued behind a long spin kernel (the GPU is busy, so
    # the call cannot block on the previous replay's completion)
    enq = []
    for _ in range(5):
        torch.cuda.synchronize()
        torch.cuda._sleep(50_000_000)
        a = time.perf_counter()
        g.graph.replay()
        enq.append(time.perf_counter() - a)
        torch.cuda.synchronize()
    print(json.dumps({'precision': args.precision, 'enqueue_behind_busy_ms': round(min(enq) * 1e3, 3),
                      'gpu_ms': round(gpu * 1e3, 3), 'host_ms': round(host / args.steps * 1e3, 3),
                      'single_ms': round(min(singles) * 1e3, 3), 'replay_only_gpu_ms': round(gpu2 * 1e3, 3),
                      'replay_only_host_ms': round(h2 / args.steps * 1e3, 3),
                      'env': {k: v for k, v in os.environ.items() if k.startswith(('DEBUG_', 'HIP_', 'MXR_'))}}))


if __name__ == '__main__':
    main()
