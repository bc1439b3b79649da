"""Attribute the step's non-HIP-extension GPU kernels (torch elementwise / copy / fill, vendor
library kernels) to the Python lines that launch them.

Runs the bench.py training step eagerly under torch.profiler (with_stack) and prints, for every
kernel whose name is not one of ours (``mxr::``), its duration and the innermost repo frame of the
op that launched it, aggregated over the profiled steps.

    python tools/glue_trace.py --steps 3 [--network resnet101] > gpurun_out/glue.txt
"""
import argparse
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from mx_rcnn_amd.config import snapshot  # noqa: E402
from mx_rcnn_amd.core.trainer import Trainer  # noqa: E402
from mx_rcnn_amd.models.faster_rcnn import FasterRCNN  # noqa: E402


def list_sites(tr, batch, ops):
    """One eager step under a TorchDispatchMode: every listed aten op on a GPU tensor with its
    shapes and the innermost repo frames of the Python stack that issued it."""
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode

    sites = defaultdict(int)

    class Mode(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = func.__name__.split('.')[0]
            if name in ops:
                shapes = [tuple(a.shape) for a in args if isinstance(a, torch.Tensor)][:2]
                fr = [f for f in traceback.extract_stack() if 'mx_rcnn_amd' in f.filename or 'bench' in f.filename]
                where = ' <- '.join('%s:%d' % (f.filename.split('mx_rcnn_amd/')[-1], f.lineno) for f in fr[-3:][::-1])
                sites[(name, str(shapes)[:60], where or '(autograd engine)')] += 1
            return func(*args, **(kwargs or {}))

    with Mode():
        tr.step(batch)
    torch.cuda.synchronize()
    print('--- aten call sites in one eager step (count, op, shapes, repo frames innermost first)')
    for (name, shapes, where), n in sorted(sites.items(), key=lambda kv: kv[0][2]):
        print('%3d %-16s %-60s %s' % (n, name, shapes, where))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--network', default='resnet101')
    ap.add_argument('--image', default='800x1333')
    ap.add_argument('--top', type=int, default=60)
    ap.add_argument('--ops', default='copy_,fill_,zero_,add_,add,sort,clone,_to_copy,slice_backward,zeros,'
                    'zeros_like,gather,sum,gt,uniform_,convolution,contiguous,cat,index,new_zeros,ones_like',
                    help='aten ops whose Python call sites are listed (one eager step under a dispatch mode)')
    args = ap.parse_args()
    dev = torch.device('cuda:0')
    h, w = [int(v) for v in args.image.split('x')]
    cfg = snapshot()
    cfg.TRAIN.BG_THRESH_LO = 0.0
    cfg.TRAIN.HAS_RPN = True
    cfg.END2END = 1
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    torch.manual_seed(1234)
    model = FasterRCNN(args.network, 81, cfg=cfg)
    gen = torch.Generator().manual_seed(4321)
    batch = bench.synthetic_batch(1, h, w, 81, dev, gen)
    if args.network.startswith('resnet'):
        model.to(dev).calibrate_bn(batch['data'])
    fixed = ['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'] if args.network.startswith('resnet') else ['conv1', 'conv2']
    tr = Trainer(model, 'e2e', fixed_param_prefix=fixed, lr=0.001, momentum=0.9, wd=0.0005, clip_gradient=1.0,
                 rescale_grad=1.0, compute_dtype=torch.bfloat16, device=dev)
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    list_sites(tr, batch, set(args.ops.split(',')))
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(args.steps):
            tr.step(batch)
        torch.cuda.synchronize()
    # correlate each device kernel with the CPU op (and its Python stack) that launched it
    events = prof.events()
    by_id = {}
    for e in events:
        by_id[e.id] = e
    agg = defaultdict(lambda: [0, 0.0])
    for e in events:
        if e.device_type != torch.autograd.DeviceType.CPU:
            continue
        for k in e.kernels:
            name = k.name
            if 'mxr::' in name:
                continue
            site, chain, p = '?', [], e
            while p is not None:
                st = [s for s in (p.stack or []) if 'mx_rcnn_amd' in s]
                if st:
                    site = st[0]
                    break
                if len(chain) < 3:
                    chain.append(p.name[:28])
                p = p.cpu_parent
            site = '/'.join(chain[1:]) + ' @ ' + site
            short = name.split('(')[0].replace('void ', '')
            for tag in ('direct_copy', 'FillFunctor', 'CUDAFunctor_add', 'copyBuffer', 'fillBuffer', 'reduce_kernel',
                        'gather', 'distribution', 'rocprim', 'Cijk', 'igemm', 'SubTensor', 'MulFunctor', 'compare',
                        'bfloat16_copy', 'index', 'where', 'cat'):
                if tag in name:
                    short = tag
                    break
            key = (short[:40], e.name[:32], site[-110:])
            agg[key][0] += 1
            agg[key][1] += k.duration_us() if callable(getattr(k, 'duration_us', None)) else k.duration
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    tot = sum(v[1] for v in agg.values()) / args.steps
    print('non-mxr kernel time per step: %.1f us' % tot)
    for (kern, op, site), (n, us) in rows[:args.top]:
        print('%8.1f us %4.1f/step  %-22s %-30s %s' % (us / args.steps, n / args.steps, kern, op, site))


if __name__ == '__main__':
    main()
