"""Tile sweep of the fp32 (x3 triple) implicit-GEMM conv forward on the ResNet-101 C4 @800x1333
shapes: graph-replayed timing per launch, numerics against the fp32 conv of the joined triples.

    python tools/microbench/conv_x3_tiles.py [--shapes s3_1x1a,s3_3x3] [--tiles 23,30,33,34]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mx_rcnn_amd.ops import need_ext  # noqa: E402
from mx_rcnn_amd.ops.precision import split, join  # noqa: E402
from tools.microbench.conv_tiles import SHAPES, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shapes', default='s3_1x1a,s3_3x3,s3_1x1b,s4_3x3,s4_1x1a,s4_1x1b,rpn_3x3')
    ap.add_argument('--tiles', default='23,30')
    ap.add_argument('--splits', default='1')
    args = ap.parse_args()
    ext = need_ext()
    torch.manual_seed(0)
    for name in args.shapes.split(','):
        n, cin, h, w, cout, k, s, p = SHAPES[name]
        xf = torch.randn(n, cin, h, w, device='cuda').contiguous(memory_format=torch.channels_last)
        wf = (torch.randn(cout, cin, k, k, device='cuda') / (cin * k * k) ** 0.5).contiguous(
            memory_format=torch.channels_last)
        xp = split(xf, 3)
        wp = split(wf, 3)
        ref = F.conv2d(join(xp, 3).double(), join(wp, 3).double(), stride=s, padding=p)
        ho, wo = ref.shape[2], ref.shape[3]
        flops = 2.0 * n * ho * wo * cout * cin * k * k
        for t in [int(v) for v in args.tiles.split(',')]:
            for sp in [int(v) for v in args.splits.split(',')]:
                def run():
                    return ext.conv_igemm_fwd(xp, wp[:cout], None, s, p, False, t, sp, x2=3,
                                              w_plane=wp.numel() // 3)[0]
                try:
                    y = run()
                    torch.cuda.synchronize()
                except Exception as e:  # unsupported combination
                    print(json.dumps({'shape': name, 'tile': t, 'splits': sp, 'error': str(e)[:80]}), flush=True)
                    continue
                err = ((join(y, 3).double() - ref).abs().max() / ref.abs().max()).item()
                us = timeit(run)
                print(json.dumps({'shape': name, 'tile': t, 'splits': sp, 'us': round(us, 2),
                                  'tflops_eq6': round(6 * flops / us / 1e6, 1), 'rel_err': float('%.2e' % err)}),
                      flush=True)


if __name__ == '__main__':
    main()
