"""Tile / pipeline / split-K sweep of the MFMA implicit-GEMM conv (conv_igemm_fwd) on the
ResNet-101 C4 @800x1333 shapes (forward and the stride-1 dgrad form), one process, CUDA-event
timing, numerics checked against torch's conv (fp32 accumulate of the same bf16 operands).

    python tools/microbench/conv_tiles.py [--shapes s3_3x3,s3_1x1a] [--tiles 0,11,12,13] [--splits 1,2,4]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mx_rcnn_amd.ops import need_ext  # noqa: E402

SHAPES = {
    # name: (N, Cin, H, W, Cout, k, stride, pad)
    's1_3x3': (1, 64, 200, 334, 64, 3, 1, 1),
    's2_3x3': (1, 128, 100, 167, 128, 3, 1, 1),
    's2_1x1a': (1, 512, 100, 167, 128, 1, 1, 0),
    's3_3x3': (1, 256, 50, 84, 256, 3, 1, 1),
    # grid-fill study: the stage-3 3x3 / 1x1 at M giving 200, 256, 264 (= s3_*) and 512 64x64 tiles
    'g200_3x3': (1, 256, 40, 80, 256, 3, 1, 1),
    'g256_3x3': (1, 256, 64, 64, 256, 3, 1, 1),
    'g512_3x3': (1, 256, 64, 128, 256, 3, 1, 1),
    'g200_1x1a': (1, 1024, 40, 80, 256, 1, 1, 0),
    'g256_1x1a': (1, 1024, 64, 64, 256, 1, 1, 0),
    'g512_1x1a': (1, 1024, 64, 128, 256, 1, 1, 0),
    's3_1x1a': (1, 1024, 50, 84, 256, 1, 1, 0),
    's3_1x1b': (1, 256, 50, 84, 1024, 1, 1, 0),
    'rpn_3x3': (1, 1024, 50, 84, 512, 3, 1, 1),
    'rpn_dgrad': (1, 512, 50, 84, 1024, 3, 1, 1),  # the dgrad of rpn_3x3 as a forward conv
    's4_3x3': (128, 512, 7, 7, 512, 3, 1, 1),
    's4_1x1a': (128, 2048, 7, 7, 512, 1, 1, 0),
    's4_1x1b': (128, 512, 7, 7, 2048, 1, 1, 0),
    's1_1x1a': (1, 256, 200, 334, 64, 1, 1, 0),
    's1_1x1b': (1, 64, 200, 334, 256, 1, 1, 0),
    's2_1x1b': (1, 128, 100, 167, 512, 1, 1, 0),
    # the stage-3 shapes at M = 4096 (exactly 256 64x64 blocks): wave-quantisation probe
    's3_3x3_sq': (1, 256, 64, 64, 256, 3, 1, 1),
    's3_1x1a_sq': (1, 1024, 64, 64, 256, 1, 1, 0),
    # batch-8 inference (BASELINE config 5) and VGG16 600x1000 trunk: the large-M GEMMs
    'b8_s3_1x1a': (8, 1024, 50, 84, 256, 1, 1, 0),
    'b8_s3_3x3': (8, 256, 50, 84, 256, 3, 1, 1),
    'b8_s3_1x1b': (8, 256, 50, 84, 1024, 1, 1, 0),
    'b8_rpn_3x3': (8, 1024, 50, 84, 512, 3, 1, 1),
    'vgg_c3': (1, 256, 150, 250, 256, 3, 1, 1),
    'vgg_c2': (1, 128, 300, 500, 128, 3, 1, 1),
}


def timeit(fn, iters=20, warm=3):
    """Device time per call (us): ``iters`` calls captured in one hipGraph and replayed, so host
    launch / binding overhead (~10 us per Python call) does not floor the small kernels."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        run = g.replay
        per = iters
    except Exception:  # not capturable: eager timing
        run = fn
        per = 1
    run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = max(1, 5 if per > 1 else iters)
    s.record()
    for _ in range(reps):
        run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (reps * per) * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shapes', default=','.join(SHAPES))
    ap.add_argument('--tiles', default='0,1,2,3,11,12,13,14,15,16')
    ap.add_argument('--splits', default='0,1,2,4,8')
    ap.add_argument('--wgrad', action='store_true', help='sweep conv_wgrad (variant x splits) instead')
    ap.add_argument('--epi', action='store_true', help='forward with the bottleneck epilogue: bias + residual + ReLU')
    ap.add_argument('--bias-relu', action='store_true',
                    help='forward with the inference BN-fold epilogue: fp32 bias + ReLU, one output (ops/fused.py _folded)')
    args = ap.parse_args()
    ext = need_ext()
    torch.manual_seed(0)
    for name in args.shapes.split(','):
        n, cin, h, w, cout, k, s, p = SHAPES[name]
        x = torch.randn(n, cin, h, w, device='cuda').bfloat16().contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, k, k, device='cuda') / (cin * k * k) ** 0.5).bfloat16().contiguous(
            memory_format=torch.channels_last)
        ref = F.conv2d(x.float(), wt.float(), stride=s, padding=p)
        fl = 2.0 * ref.numel() * cin * k * k
        if args.wgrad:
            dy = torch.randn_like(ref).bfloat16().contiguous(memory_format=torch.channels_last)
            wref = torch.ops.aten.convolution_backward(dy.float(), x.float(), wt.float(), None, [s, s], [p, p], [1, 1],
                                                       False, [0, 0], 1, [False, True, False])[1]
            res = {'name': name, 'gflop': round(fl / 1e9, 2), 'miopen_us': round(timeit(
                lambda: torch.ops.aten.convolution_backward(dy, x, wt, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                            [False, True, False])), 1)}
            best = None
            for var in (0, 1):
                for sp in [int(v) for v in args.splits.split(',')]:
                    dw = ext.conv_wgrad(dy, x, k, k, s, p, sp, variant=var)
                    err = (dw.float() - wref).abs().max().item() / (wref.abs().max().item() + 1e-6)
                    key = 'v%d_s%d' % (var, sp)
                    if err > 2e-2:
                        res[key] = 'BAD %.3g' % err
                        continue
                    us = timeit(lambda: ext.conv_wgrad(dy, x, k, k, s, p, sp, variant=var))
                    res[key] = round(us, 1)
                    if best is None or us < best[0]:
                        best = (us, var, sp)
            res['best'] = '%.1fus v%d s%d %.0f TF/s' % (best[0], best[1], best[2], fl / best[0] / 1e6)
            print(json.dumps(res), flush=True)
            continue
        res = {'name': name, 'gflop': round(fl / 1e9, 2), 'miopen_us': round(timeit(lambda: F.conv2d(x, wt, stride=s, padding=p)), 1)}
        if k == 1 and s == 1:
            x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
            w2 = wt.reshape(cout, cin)
            res['hipblaslt_us'] = round(timeit(lambda: F.linear(x2, w2)), 1)
        best = None
        ekw = {}
        if args.epi:  # the inference bottleneck's last conv: folded-BN bias, identity residual, ReLU
            bias = torch.randn(cout, device='cuda').bfloat16()
            resid = torch.randn_like(ref).bfloat16().contiguous(memory_format=torch.channels_last)
            ref = torch.relu(ref + bias.float().view(1, -1, 1, 1) + resid.float())
            ekw = {'bias': bias, 'relu': True, 'residual': resid}
        if args.bias_relu:
            bias = torch.randn(cout, device='cuda')
            ref = torch.relu(ref + bias.view(1, -1, 1, 1))
            ekw = {'bias': bias, 'relu': True, 'residual': None}
        for tile in [int(t) for t in args.tiles.split(',')]:
            for sp in [int(v) for v in args.splits.split(',')]:
                if tile == 0 and sp != 0:
                    continue
                def call():
                    if ekw:
                        return ext.conv_igemm_fwd(x, wt, ekw['bias'], s, p, True, tile, sp, residual=ekw['residual'])
                    return ext.conv_igemm_fwd(x, wt, None, s, p, False, tile, sp)
                try:
                    y = call()[0]
                except RuntimeError as e:
                    res['t%d_s%d' % (tile, sp)] = 'err'
                    continue
                err = (y.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
                if err > 2e-2:
                    res['t%d_s%d' % (tile, sp)] = 'BAD %.3g' % err
                    continue
                us = timeit(call)
                res['t%d_s%d' % (tile, sp)] = round(us, 1)
                if best is None or us < best[0]:
                    best = (us, tile, sp)
        if best:
            res['best'] = '%.1fus t%d s%d %.0f TF/s' % (best[0], best[1], best[2], fl / best[0] / 1e6)
        print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
