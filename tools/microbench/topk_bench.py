"""Proposal top-k: HIP radix-select + rank kernels vs torch stable sort + gather (graph-timed).

    python tools/microbench/topk_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from mx_rcnn_amd.ops import need_ext  # noqa: E402
from tools.microbench.conv_tiles import timeit  # noqa: E402


def main():
    ext = need_ext()
    for (B, N, P, kind) in [(1, 50400, 12000, 'uniform'), (1, 50400, 6000, 'uniform'), (8, 50400, 6000, 'uniform'),
                            (1, 50400, 12000, 'rpn'), (8, 50400, 12000, 'rpn'), (8, 50400, 6000, 'rpn')]:
        g = torch.Generator().manual_seed(0)
        if kind == 'rpn':  # softmax foreground probabilities: most near 0, clustered top bytes
            keys = torch.softmax(torch.randn(B, N, 2, generator=g) * 3, 2)[..., 1].cuda()
        else:
            keys = torch.rand(B, N, generator=g).cuda()
        keys[torch.rand(B, N, generator=g).cuda() < 0.2] = float('-inf')
        boxes = (torch.rand(B, N, 4, generator=g) * 500).cuda()

        def hip():
            return ext.proposal_topk(keys, boxes, P)

        def ref():
            sk, order = torch.sort(keys, dim=1, descending=True, stable=True)
            sk, order = sk[:, :P].contiguous(), order[:, :P]
            sb = torch.gather(boxes, 1, order[..., None].expand(-1, -1, 4)).contiguous()
            return sk, sb, (sk > float('-inf')).sum(1).to(torch.int32)
        print('%-7s B=%d N=%d P=%d  hip %.1f us  torch %.1f us' % (kind, B, N, P, timeit(hip), timeit(ref)),
              flush=True)


if __name__ == '__main__':
    main()
