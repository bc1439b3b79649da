"""Two data-parallel ranks on ONE GPU -- the worker of tests/test_dist_gpu.py
test_two_ranks_on_one_gpu_* (ResNet-50 Fast R-CNN).  RCCL refuses two ranks on one device, so the ranks talk over gloo,
which carries the device-resident gradient buckets through host memory; everything else is the
production DP path: the flat-buffer gradient hooks, bucketed async all-reduce (SUM, fp32 wire),
bucket-wise SGD, on the GPU kernels.  Without WORLD_SIZE the same script runs one plain process.

    python tools/dp_two_rank_check.py OUT.pt [--precision fp32|bf16] [--steps 2] [--same-batch]
        [--rescale 1.0] [--mode e2e --network resnet101 --image 800x1333 --bucket-mb 25]

``--mode e2e``: the headline step's shape -- approximate-joint e2e training (anchor targets, the
proposal chain 12000 -> 6000 with its sampling, RoI pooling, the stage-4 head) on a synthetic
800x1333 image with random gt boxes, production bucket sizes (eager; gloo carries the buckets).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import mx_rcnn_amd  # noqa: E402,F401  (runtime defaults before the GPU initialises)
import torch  # noqa: E402

from mx_rcnn_amd.config import snapshot  # noqa: E402
from mx_rcnn_amd.core.trainer import Trainer  # noqa: E402
from mx_rcnn_amd.models import FasterRCNN  # noqa: E402
from mx_rcnn_amd.parallel import dist as pdist  # noqa: E402


def batch(seed, device):
    """A Fast R-CNN (rcnn mode) batch: one 224x320 image and 4 fixed RoIs, per-seed pixels / targets."""
    g = torch.Generator().manual_seed(100 + seed)
    rois = torch.tensor([[0., 10, 20, 80, 100], [0., 30, 30, 90, 120], [0., 5, 5, 60, 60], [0., 40, 8, 150, 110]])
    b = {'data': torch.randn(1, 3, 224, 320, generator=g) * 50, 'rois': rois,
         'label': torch.tensor([3, 0, 5, 1], dtype=torch.int32),
         'bbox_target': torch.randn(4, 24, generator=g) * 0.1,
         'bbox_inside_weight': torch.ones(4, 24), 'bbox_outside_weight': torch.ones(4, 24)}
    return {k: v.to(device) for k, v in b.items()}


def e2e_batch(seed, device, h, w, num_classes):
    from bench import synthetic_batch
    return synthetic_batch(1, h, w, num_classes, device, torch.Generator().manual_seed(100 + seed))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('out')
    ap.add_argument('--precision', default='fp32')
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--same-batch', action='store_true', help='every rank trains on the batch of rank 0')
    ap.add_argument('--rescale', type=float, default=1.0)
    ap.add_argument('--mode', default='rcnn', choices=['rcnn', 'e2e'])
    ap.add_argument('--network', default='resnet50')
    ap.add_argument('--image', default='800x1333')
    ap.add_argument('--bucket-mb', type=float, default=0.05)
    args = ap.parse_args()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = 0
    if world > 1:
        rank, world, _, _ = pdist.init_distributed(backend='gloo')
    dev = torch.device('cuda', 0) if torch.cuda.is_available() else torch.device('cpu')  # (CPU: a dry run)
    if dev.type == 'cuda':
        torch.cuda.set_device(dev)
    torch.manual_seed(0)
    if args.mode == 'e2e':
        h, w = [int(v) for v in args.image.split('x')]
        cfg = snapshot()
        cfg.TRAIN.BG_THRESH_LO = 0.0
        cfg.END2END = 1
        cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
        model = FasterRCNN(args.network, 81, cfg=cfg)
        model.to(dev).calibrate_bn(e2e_batch(0, dev, h, w, 81)['data'])  # rank 0 broadcasts its statistics
        make = lambda s: e2e_batch(s, dev, h, w, 81)  # noqa: E731
        fixed, clip = ['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'], 1.0
    else:
        model = FasterRCNN(args.network, 6, cfg=snapshot())
        make = lambda s: batch(s, dev)  # noqa: E731
        fixed, clip = ['conv0', 'stage1', 'bn_data', 'bn0'], -1
    tr = Trainer(model, args.mode, fixed_param_prefix=fixed, lr=0.01, momentum=0.9,
                 wd=0.0005, clip_gradient=clip, rescale_grad=args.rescale, device=dev, bucket_mb=args.bucket_mb,
                 precision=args.precision)
    assert tr.reducer.dp == (world > 1)
    objs = []
    for s in range(args.steps):
        torch.manual_seed(1000 + s)  # the samplers' draws: the same on every rank and in the plain run
        out = tr.step(make((0 if args.same_batch else rank) + 10 * s))
        objs.append(float(out['objective'].float().item()))
    if dev.type == 'cuda':
        torch.cuda.synchronize()
    state = {k: v.detach().cpu().clone() for k, v in tr.store.state_arrays().items()}
    state['_info'] = torch.tensor([int(tr.reducer.dp), len(tr.reducer.buckets), world, rank])
    state['_objective'] = torch.tensor(objs)
    torch.save(state, args.out)
    print('rank %d/%d saved %d arrays, dp=%d buckets=%d backend=%s objectives=%s' % (
        rank, world, len(state), tr.reducer.dp, len(tr.reducer.buckets), pdist.backend_name(), objs), flush=True)
    if world > 1:
        pdist.barrier()
        pdist.destroy()


if __name__ == '__main__':
    main()
