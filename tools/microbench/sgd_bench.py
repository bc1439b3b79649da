"""Fused SGD-momentum bandwidth on flat buffers of the two models' trainable sizes.

    MXR_SGD=0|1|2 python tools/microbench/sgd_bench.py
(0: 4-wide kernel, 1: 8-wide, 2: 8-wide with nontemporal master / momentum / gradient access.)
Bytes per element: fp32-class 24 (w, mom, grad read; w, mom, hi, lo written), bf16 20."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from mx_rcnn_amd.ops import need_ext  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    ext = need_ext()
    for name, n in (('vgg16', 136_800_000), ('resnet101', 42_200_000)):
        for mode in ('x2', 'bf16'):
            w = torch.randn(n, device=dev)
            mom = torch.zeros(n, device=dev)
            grad = torch.randn(n, device=dev) if mode == 'x2' else torch.randn(n, device=dev).bfloat16()
            sh = torch.empty((2 if mode == 'x2' else 1) * n, dtype=torch.bfloat16, device=dev)
            lr = torch.full((1,), 1e-3, device=dev)
            for _ in range(3):
                ext.sgd_momentum(w, mom, grad, lr, 0.9, 5e-4, 1.0, 1.0, sh)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            it = 20
            a.record()
            for _ in range(it):
                ext.sgd_momentum(w, mom, grad, lr, 0.9, 5e-4, 1.0, 1.0, sh)
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / it * 1e3
            nbytes = n * (24 if mode == 'x2' else 20)
            print(json.dumps({'variant': os.environ.get('MXR_SGD', '0'), 'model': name, 'mode': mode, 'n': n,
                              'us': round(us, 1), 'TBps': round(nbytes / us / 1e6, 2)}), flush=True)
            del w, mom, grad, sh


if __name__ == '__main__':
    main()
