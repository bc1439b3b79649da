"""Run ONE conv_igemm_fwd configuration repeatedly (for rocprofv3 --pmc passes).

    python tools/microbench/conv_one.py s3_3x3 TILE SPLITS [ITERS]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from mx_rcnn_amd.ops import need_ext  # noqa: E402
from tools.microbench.conv_tiles import SHAPES  # noqa: E402


def main():
    name, tile, sp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 50
    n, cin, h, w, cout, k, s, p = SHAPES[name]
    ext = need_ext()
    x = torch.randn(n, cin, h, w, device='cuda').bfloat16().contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cout, cin, k, k, device='cuda') / (cin * k * k) ** 0.5).bfloat16().contiguous(
        memory_format=torch.channels_last)
    for _ in range(iters):
        ext.conv_igemm_fwd(x, wt, None, s, p, False, tile, sp)
    torch.cuda.synchronize()
    print('done', name, tile, sp)


if __name__ == '__main__':
    main()
