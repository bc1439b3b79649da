"""Microbenchmark: MIOpen conv fwd+bwd in bf16, NCHW vs NHWC, on the ResNet-101 C4 /
VGG16 shapes of SURVEY §2.14 (800x1333 input).  Decides the activation layout."""
import json
import time

import torch
import torch.nn.functional as F


def bench(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def case(name, n, cin, h, w, cout, k, s, p, fmt, dtype=torch.bfloat16, bwd=True):
    x = torch.randn(n, cin, h, w, device='cuda', dtype=dtype)
    wt = torch.randn(cout, cin, k, k, device='cuda', dtype=dtype) * 0.05
    if fmt == 'nhwc':
        x = x.contiguous(memory_format=torch.channels_last)
        wt = wt.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(bwd)
    wt.requires_grad_(bwd)

    def f():
        y = F.conv2d(x, wt, stride=s, padding=p)
        if bwd:
            y.backward(torch.ones_like(y))
        return y
    ms = bench(f)
    y = F.conv2d(x, wt, stride=s, padding=p)
    flops = 2 * y.numel() * cin * k * k * (3 if bwd else 1)
    return {'name': name, 'fmt': fmt, 'ms': round(ms, 4), 'tflops': round(flops / ms / 1e9, 1)}


def main():
    torch.backends.cudnn.benchmark = True
    shapes = [
        # name, n, cin, h, w, cout, k, s, p
        ('r101_conv0', 1, 3, 800, 1333, 64, 7, 2, 3),
        ('r101_s1_1x1', 1, 64, 200, 334, 64, 1, 1, 0),
        ('r101_s1_3x3', 1, 64, 200, 334, 64, 3, 1, 1),
        ('r101_s1_1x1up', 1, 64, 200, 334, 256, 1, 1, 0),
        ('r101_s3_1x1a', 1, 1024, 50, 84, 256, 1, 1, 0),
        ('r101_s3_3x3', 1, 256, 50, 84, 256, 3, 1, 1),
        ('r101_s3_1x1b', 1, 256, 50, 84, 1024, 1, 1, 0),
        ('rpn_3x3', 1, 1024, 50, 84, 512, 3, 1, 1),
        ('r101_s4_3x3_rois', 128, 512, 7, 7, 512, 3, 2, 1),
        ('r101_s4_1x1_rois', 128, 512, 4, 4, 2048, 1, 1, 0),
        ('vgg_conv1_2', 1, 64, 600, 1000, 64, 3, 1, 1),
        ('vgg_conv3_x', 1, 256, 150, 250, 256, 3, 1, 1),
        ('vgg_conv5_x', 1, 512, 37, 62, 512, 3, 1, 1),
    ]
    out = []
    for s in shapes:
        for fmt in ('nchw', 'nhwc'):
            try:
                r = case(*s, fmt=fmt)
            except Exception as e:  # record and continue
                r = {'name': s[0], 'fmt': fmt, 'error': str(e)[:200]}
            print(json.dumps(r), flush=True)
            out.append(r)
    # GEMM reference point (fc6-like)
    a = torch.randn(128, 25088, device='cuda', dtype=torch.bfloat16)
    b = torch.randn(4096, 25088, device='cuda', dtype=torch.bfloat16)
    ms = bench(lambda: a @ b.t())
    print(json.dumps({'name': 'fc6_gemm_128x4096x25088', 'ms': round(ms, 4),
                      'tflops': round(2 * 128 * 4096 * 25088 / ms / 1e9, 1)}))
    a = torch.randn(8192, 8192, device='cuda', dtype=torch.bfloat16)
    ms = bench(lambda: a @ a)
    print(json.dumps({'name': 'gemm_8192', 'ms': round(ms, 4), 'tflops': round(2 * 8192 ** 3 / ms / 1e9, 1)}))


if __name__ == '__main__':
    main()
