"""Fixed (K-independent) cost of one conv launch: the stage-3 1x1 shape at K = 64 (two K stages)
in several epilogue / precision forms, each launched 30 times (run under rocprofv3 --kernel-trace
and read the per-kernel durations).

    rocprofv3 --kernel-trace -d out -o run -- python tools/microbench/conv_fixed_cost.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from mx_rcnn_amd.ops import need_ext  # noqa: E402
from mx_rcnn_amd.ops.precision import split  # noqa: E402


def main():
    ext = need_ext()
    torch.manual_seed(0)
    cin = int(os.environ.get('CIN', '64'))
    xf = torch.randn(1, cin, 50, 84, device='cuda').contiguous(memory_format=torch.channels_last)
    wf = (torch.randn(256, cin, 1, 1, device='cuda') / cin ** 0.5).contiguous(memory_format=torch.channels_last)
    xp, wp = split(xf), split(wf)
    xb, wb = xf.bfloat16(), wf.bfloat16()
    cases = [
        ('bf16', lambda: ext.conv_igemm_fwd(xb, wb, None, 1, 0, False, 23, 1)),
        ('bf16_relu', lambda: ext.conv_igemm_fwd(xb, wb, None, 1, 0, True, 23, 1)),
        ('x2', lambda: ext.conv_igemm_fwd(xp, wp[:256], None, 1, 0, False, 23, 1, x2=True, w_plane=wp.numel() // 2)),
        ('x2_f32out', lambda: ext.conv_igemm_fwd(xp, wp[:256], None, 1, 0, False, 23, 1, x2=True,
                                                 w_plane=wp.numel() // 2, out_f32=True)),
        ('x2_split2', lambda: ext.conv_igemm_fwd(xp, wp[:256], None, 1, 0, False, 23, 2, x2=True,
                                                 w_plane=wp.numel() // 2)),
    ]
    for name, fn in cases:
        for _ in range(30):
            fn()
        torch.cuda.synchronize()
        torch.cuda._sleep(2000000)  # a visible gap between the cases in the trace
        torch.cuda.synchronize()
        print('case', name, flush=True)


if __name__ == '__main__':
    main()
