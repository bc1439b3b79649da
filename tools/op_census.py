"""Census of the ATen ops one eager training step dispatches, grouped by the framework source
line that issued them (every ATen op on a GPU tensor is at least one kernel launch in the
captured step).  Used to find per-layer glue that should be fused into our kernels.

    python tools/op_census.py [--network resnet101] [--image 800x1333] [--top 60]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from bench import synthetic_batch  # noqa: E402
from mx_rcnn_amd.config import snapshot  # noqa: E402
from mx_rcnn_amd.core.trainer import Trainer  # noqa: E402
from mx_rcnn_amd.models import FasterRCNN  # noqa: E402

SKIP = {'aten::detach', 'aten::view', 'aten::_unsafe_view', 'aten::as_strided', 'aten::t', 'aten::permute',
        'aten::reshape', 'aten::expand', 'aten::slice', 'aten::select', 'aten::unsqueeze', 'aten::squeeze',
        'aten::transpose', 'aten::alias', 'aten::empty', 'aten::empty_strided', 'aten::empty_like', 'aten::lift_fresh',
        'aten::_to_copy' if False else 'aten::__none__', 'prim::device', 'aten::is_nonzero', 'aten::item',
        'aten::_local_scalar_dense', 'aten::split', 'aten::unbind', 'aten::chunk', 'aten::narrow', 'aten::diagonal'}


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.count = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = 'aten::' + func.__name__.split('.')[0]
        if name not in SKIP:
            f = sys._getframe(0).f_back
            site = '<autograd engine: built-in backward>'
            while f is not None:
                fn = f.f_code.co_filename
                if ('mx_rcnn_amd' in fn or fn.endswith('bench.py')) and 'op_census' not in fn:
                    site = '%s:%d %s' % (os.path.relpath(fn, os.path.dirname(os.path.dirname(__file__))), f.f_lineno,
                                         f.f_code.co_name)
                    break
                f = f.f_back
            self.count[(name, site)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--network', default='resnet101')
    ap.add_argument('--image', default='800x1333')
    ap.add_argument('--top', type=int, default=70)
    args = ap.parse_args()
    dev = torch.device('cuda')
    h, w = [int(v) for v in args.image.split('x')]
    cfg = snapshot()
    cfg.TRAIN.BG_THRESH_LO = 0.0
    cfg.TRAIN.HAS_RPN = True
    cfg.END2END = 1
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    torch.manual_seed(0)
    model = FasterRCNN(args.network, 81, cfg=cfg)
    gen = torch.Generator().manual_seed(1)
    batch = synthetic_batch(1, h, w, 81, dev, gen)
    model.to(dev).calibrate_bn(batch['data'])
    tr = Trainer(model, 'e2e', fixed_param_prefix=['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'], device=dev,
                 compute_dtype=torch.bfloat16)
    for _ in range(2):
        tr.step(batch)
    torch.cuda.synchronize()
    c = Census()
    with c:
        tr.step(batch)
    torch.cuda.synchronize()
    total = sum(c.count.values())
    print('ATen ops per eager step (excluding views/empties): %d' % total)
    for (name, site), n in c.count.most_common(args.top):
        print('%5d  %-34s %s' % (n, name, site))


if __name__ == '__main__':
    main()
