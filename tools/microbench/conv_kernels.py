"""Per-shape A/B of the hand-written MFMA conv kernels vs MIOpen / hipBLASLt (one process,
interleaved, bf16 NHWC), for the ResNet-101 C4 @800x1333 and VGG16 shapes."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mx_rcnn_amd.ops import need_ext  # noqa: E402


def t_ms(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    ext = need_ext()
    shapes = [
        ('s1_3x3', 1, 64, 200, 334, 64, 3, 1, 1),
        ('s2_3x3', 1, 128, 100, 167, 128, 3, 1, 1),
        ('s3_3x3', 1, 256, 50, 84, 256, 3, 1, 1),
        ('rpn_3x3', 1, 1024, 50, 84, 512, 3, 1, 1),
        ('s4_3x3_rois', 128, 512, 4, 4, 512, 3, 1, 1),
        ('s4u1_3x3s2_rois', 128, 512, 7, 7, 512, 3, 2, 1),
        ('s3_1x1a', 1, 1024, 50, 84, 256, 1, 1, 0),
        ('s3_1x1b', 1, 256, 50, 84, 1024, 1, 1, 0),
        ('s4_1x1a_rois', 128, 2048, 4, 4, 512, 1, 1, 0),
        ('s4_1x1b_rois', 128, 512, 4, 4, 2048, 1, 1, 0),
        ('s1_1x1up', 1, 64, 200, 334, 256, 1, 1, 0),
        ('vgg_conv3', 1, 256, 150, 250, 256, 3, 1, 1),
        ('vgg_conv5', 1, 512, 37, 62, 512, 3, 1, 1),
    ]
    for name, n, cin, h, w, cout, k, s, p in shapes:
        x = torch.randn(n, cin, h, w, device='cuda').bfloat16().contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, k, k, device='cuda') * 0.05).bfloat16().contiguous(
            memory_format=torch.channels_last)
        y = F.conv2d(x, wt, stride=s, padding=p)
        dy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
        fl = 2 * y.numel() * cin * k * k
        r = {'name': name}
        r['fwd_miopen'] = t_ms(lambda: F.conv2d(x, wt, stride=s, padding=p))
        r['fwd_ours'] = t_ms(lambda: ext.conv_igemm_fwd(x, wt, None, s, p, False)[0])
        if k == 1 and s == 1:
            x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
            r['fwd_gemm'] = t_ms(lambda: F.linear(x2, wt.reshape(cout, cin)))
        r['wgrad_miopen'] = t_ms(lambda: torch.ops.aten.convolution_backward(
            dy, x, wt, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [False, True, False]))
        r['wgrad_ours'] = t_ms(lambda: ext.conv_wgrad(dy, x, k, k, s, p))
        if k == 1 and s == 1:
            dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
            x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
            r['wgrad_gemm'] = t_ms(lambda: dy2.t() @ x2)
        r['dgrad_miopen'] = t_ms(lambda: torch.ops.aten.convolution_backward(
            dy, x, wt, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [True, False, False]))
        if s == 1 and cout % 64 == 0:
            wf = wt.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
            r['dgrad_ours'] = t_ms(lambda: ext.conv_igemm_fwd(dy, wf, None, 1, k - 1 - p, False)[0])
        for kk in list(r):
            if kk != 'name':
                r[kk] = round(r[kk] * 1000, 1)  # us
        r['gflop_fwd'] = round(fl / 1e9, 2)
        print(json.dumps(r), flush=True)


if __name__ == '__main__':
    main()
