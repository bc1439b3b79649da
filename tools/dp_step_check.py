"""Run K graph-replayed training steps and save the resulting state (flat fp32 masters, momentum,
shadows) -- the worker of tests/test_dist_gpu.py.  With ``MXR_FORCE_DIST=1 WORLD_SIZE=1`` the step
runs under a 1-rank RCCL process group: every gradient bucket goes through the reducer's
all-reduce, captured inside the hipGraph, so comparing against a run without the group checks the
DP path end to end on one GPU.

    python tools/dp_step_check.py OUT.pt [--precision bf16|fp32] [--steps 3] [--mode rcnn|e2e] [--network vgg16]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import mx_rcnn_amd  # noqa: E402,F401  (runtime defaults before the GPU initialises)
import torch  # noqa: E402

from bench import rcnn_batch, synthetic_batch  # noqa: E402
from mx_rcnn_amd.config import snapshot  # noqa: E402
from mx_rcnn_amd.core.trainer import GraphedStep, Trainer  # noqa: E402
from mx_rcnn_amd.models import FasterRCNN  # noqa: E402
from mx_rcnn_amd.parallel import dist as pdist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('out')
    ap.add_argument('--precision', default='bf16')
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--mode', default='rcnn', choices=['rcnn', 'e2e'])
    ap.add_argument('--network', default='resnet50')
    ap.add_argument('--image', default='320x480')
    ap.add_argument('--dirty-gb', type=float, default=0.0,
                    help='before anything else, fill this many GB of the caching allocator with NaN and free it: '
                         'a kernel that reads memory it never wrote then sees NaN instead of the zeros of fresh VRAM')
    ap.add_argument('--dirty-keep', action='store_true',
                    help='keep the dirty blocks in the caching allocator (no empty_cache): eager allocations '
                         'then reuse them')
    ap.add_argument('--dirty-val', type=float, default=float('nan'), help='fill value of --dirty-gb')
    args = ap.parse_args()
    rank, world, _, device = pdist.init_distributed()
    if args.dirty_gb > 0:
        blocks = []
        for sz in (1 << 28, 1 << 24, 1 << 20, 1 << 16):  # large and small allocator pools
            for _ in range(max(1, int(args.dirty_gb * (1 << 30) / 4 / sz / 4))):
                blocks.append(torch.full((sz,), args.dirty_val, device=device))
        torch.cuda.synchronize()
        del blocks
        if not args.dirty_keep:
            torch.cuda.empty_cache()  # back to the driver: the graph pool's fresh segments may get these pages
    h, w = [int(v) for v in args.image.split('x')]
    cfg = snapshot()
    if args.mode == 'e2e':
        cfg.TRAIN.BG_THRESH_LO = 0.0
        cfg.END2END = 1
        cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    torch.manual_seed(7)
    model = FasterRCNN(args.network, 21, cfg=cfg)
    gen = torch.Generator().manual_seed(11)
    pool = [synthetic_batch(1, h, w, 21, device, gen) for _ in range(2)]
    if args.mode == 'rcnn':
        pool = [rcnn_batch(b, 21, cfg.TRAIN.BATCH_SIZE, gen) for b in pool]
    vgg = args.network.startswith('vgg')
    if vgg:
        model.to(device).calibrate_vgg(pool[0]['data'])
    else:
        model.to(device).calibrate_bn(pool[0]['data'])
    fixed = ['conv1', 'conv2'] if vgg else ['conv0', 'stage1', 'bn_data', 'bn0']
    tr = Trainer(model, args.mode, fixed_param_prefix=fixed, lr=0.01, momentum=0.9,
                 wd=0.0005, clip_gradient=1.0, device=device, precision=args.precision)
    g = GraphedStep(tr, pool[0], warmup=2)
    for i in range(args.steps):
        out = g(pool[i % 2])
    torch.cuda.synchronize()
    state = {k: v.detach().cpu().clone() for k, v in tr.store.state_arrays().items()}
    state['_objective'] = out['objective'].detach().float().cpu().reshape(1)
    state['_dp'] = torch.tensor([int(tr.reducer.dp), len(tr.reducer.buckets), world, len(tr.reducer.early_names),
                                 len(tr.fused_fc_sgd)])
    torch.save(state, args.out)
    print('saved %d arrays, dp=%d buckets=%d backend=%s' % (len(state), tr.reducer.dp, len(tr.reducer.buckets),
                                                           pdist.backend_name()))
    pdist.barrier()
    pdist.destroy()


if __name__ == '__main__':
    main()
