"""Buffer-kernel tile / depth sweep for bf16 and fp32-class (x2) pairs on the ResNet-101 C4
@800x1333 shapes: device time per call (graph-replayed) and bitwise agreement between tiles (the
same K order).  Tiles: 23 = 64x64 depth 3, 33 = 64x64 depth 4, 22 / 32 = 128x64 depth 3 / 4,
21 = 128x128 depth 3.

Round-3 finding kept here: a register-pipelined variant (each wave loading its MFMA fragments
straight from memory, 3-6 K-steps in VGPRs, no LDS) ran 2.5-3x slower than tile 23 on every
shape -- the scattered 16-B-per-lane row loads cost far more L1 / L2 throughput than one LDS-DMA
stage shared by four waves.

    python tools/microbench/conv_reg.py [--shapes s3_1x1a,s3_3x3] [--tiles 23,33] [--splits 1]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from mx_rcnn_amd.ops import need_ext, precision  # noqa: E402
from tools.microbench.conv_tiles import SHAPES, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shapes', default='s3_1x1a,s3_3x3,s3_1x1b,s2_1x1a,s2_3x3,rpn_3x3,s4_1x1a,s4_3x3')
    ap.add_argument('--tiles', default='23,33,22,32,21')
    ap.add_argument('--splits', default='1')
    args = ap.parse_args()
    ext = need_ext()
    dev = torch.device('cuda', 0)
    cl = torch.channels_last
    for name in args.shapes.split(','):
        N, Cin, H, W, Cout, k, stride, pad = SHAPES[name]
        g = torch.Generator().manual_seed(0)
        xf = torch.randn(N, Cin, H, W, generator=g).to(dev).contiguous(memory_format=cl)
        wf = (torch.randn(Cout, Cin, k, k, generator=g) * 0.05).to(dev).contiguous(memory_format=cl)
        for mode in ('bf16', 'x2'):
            if mode == 'x2':
                xp = precision.split(xf).contiguous(memory_format=cl)
                wp = precision.split(wf).contiguous(memory_format=cl)
                xa, wa, kw = xp, wp[:Cout], dict(x2=True, w_plane=wp.numel() // 2)
            else:
                xa, wa, kw = xf.to(torch.bfloat16), wf.to(torch.bfloat16), {}
            ref = None
            row = {'shape': name, 'mode': mode}
            for t in [int(v) for v in args.tiles.split(',')]:
                for sp in [int(v) for v in args.splits.split(',')]:
                    try:
                        fn = lambda: ext.conv_igemm_fwd(xa, wa, None, stride, pad, False, t, sp, **kw)  # noqa: E731
                        out = fn()[0]
                    except RuntimeError as e:
                        row['t%d_s%d' % (t, sp)] = 'n/a'
                        continue
                    if ref is None:
                        ref = out
                    same = bool(torch.equal(out, ref))
                    row['t%d_s%d' % (t, sp)] = '%.1f%s' % (timeit(fn), '' if same else ' DIFF')
            print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
