"""Is the stage-3 implicit-GEMM conv latency- or bandwidth-bound?  Runs k independent copies of
the same conv (plan-chosen tile) concurrently on k streams and reports the time per batch of k
against k x the single-stream time: ~1x means the CUs sit idle waiting on memory latency (more
concurrent work per CU would help), ~k x means a per-CU fill or HBM bandwidth limit.

    python tools/microbench/conv_concurrency.py [--shapes s3_1x1a,s3_3x3] [--k 1,2,4]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from mx_rcnn_amd.ops import need_ext  # noqa: E402
from tools.microbench.conv_tiles import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shapes', default='s3_1x1a,s3_3x3,s3_1x1b,s2_3x3,s4_3x3')
    ap.add_argument('--k', default='1,2,4')
    ap.add_argument('--iters', type=int, default=50)
    args = ap.parse_args()
    ext = need_ext()
    torch.manual_seed(0)
    for name in args.shapes.split(','):
        n, cin, h, w, cout, k, s, p = SHAPES[name]
        res = {'name': name}
        for kk in [int(v) for v in args.k.split(',')]:
            xs = [torch.randn(n, cin, h, w, device='cuda').bfloat16().contiguous(memory_format=torch.channels_last)
                  for _ in range(kk)]
            ws = [(torch.randn(cout, cin, k, k, device='cuda') / (cin * k * k) ** 0.5).bfloat16().contiguous(
                memory_format=torch.channels_last) for _ in range(kk)]
            streams = [torch.cuda.Stream() for _ in range(kk)]
            main = torch.cuda.current_stream()

            def run(reps):
                # each stream runs `reps` convs back to back: no cross-stream sync inside the timed
                # region except the fork and the join
                for i in range(kk):
                    streams[i].wait_stream(main)
                    with torch.cuda.stream(streams[i]):
                        for _ in range(reps):
                            ext.conv_igemm_fwd(xs[i], ws[i], None, s, p, False, 0, 0)
                for i in range(kk):
                    main.wait_stream(streams[i])

            run(3)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(args.iters)
            e1.record()
            torch.cuda.synchronize()
            res['k%d_us' % kk] = round(e0.elapsed_time(e1) / args.iters * 1e3, 1)  # per conv per stream
        if 'k1_us' in res:
            for kk in [int(v) for v in args.k.split(',')]:
                if kk > 1:
                    res['k%d_vs_serial' % kk] = round(res['k%d_us' % kk] / (kk * res['k1_us']), 2)
        print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
