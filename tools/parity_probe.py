#!/usr/bin/env python
"""Gradient-parity probe behind tests/test_parity.py: how far is each training path from the fp32
CPU reference, per layer (cosine, relative norm)?

Arms (same weights, same deterministic samples as the test):
  gpu_bf16      the production path (HIP kernels, bf16 activations / weights, fp32 accumulation)
  gpu_fp32      the same model in fp32 on the GPU (PyTorch / MIOpen ops: order-of-summation noise only)
  cpu_bf16in    fp32 CPU math on bf16-ROUNDED input image and weights (sensitivity of the random-init
                network to input rounding alone)
  cpu_bf16act   cpu_bf16in plus every layer output and every layer-output gradient rounded to bf16
                (forward / tensor hooks on the leaf modules): what bf16 STORAGE of activations and
                gradients costs with exact fp32 arithmetic in between -- the floor of any bf16 path
  gpu_bf16x3    bf16 hi / lo pairs between kernels, three MFMAs per product (16 significant bits)
  gpu_fp32x3    the fp32 mode: exact (mid, hi, lo) bf16 triples, six MFMAs per product (24 bits)

    python tools/parity_probe.py [--mode rpn|rcnn]
"""
import argparse
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

import torch  # noqa: E402

import test_parity as tp  # noqa: E402
from mx_rcnn_amd.core.trainer import Trainer  # noqa: E402
from mx_rcnn_amd.models import FasterRCNN  # noqa: E402


def stats(ref, got):
    norms = {n: float(v.norm()) for n, v in ref.items()}
    big = max(norms.values())
    rows = []
    for n, v in ref.items():
        if norms[n] < 1e-3 * big:
            continue
        w = got[n]
        cos = float(torch.dot(v, w) / (v.norm() * w.norm() + 1e-30))
        rows.append((cos, abs(float(w.norm()) - norms[n]) / norms[n], n))
    near = [r for r in rows if r[2].split('_')[0] in ('rpn', 'cls', 'bbox') or r[2].startswith('stage4_unit3') or
            r[2].startswith('bn1_')]
    rows.sort()
    cs = sorted(r[0] for r in rows)
    return cs[len(cs) // 2], rows[:4], sorted(near)


def _bf(t):
    return t.to(torch.bfloat16).float() if torch.is_tensor(t) and t.is_floating_point() else t


def _round_storage(model):
    """Round every leaf module's output (forward) and the gradient arriving at it (backward) to
    bf16, as bf16 activation / gradient storage between kernels would."""
    def fwd_hook(mod, inp, out):
        def one(t):
            if not (torch.is_tensor(t) and t.is_floating_point()):
                return t
            r = _bf(t)
            if r.requires_grad:
                r.register_hook(_bf)
            return r
        if isinstance(out, tuple):
            return tuple(one(t) for t in out)
        return one(out)
    for mod in model.modules():
        if len(list(mod.children())) == 0:
            mod.register_forward_hook(fwd_hook)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--mode', default='rpn', choices=['rpn', 'rcnn'])
    args = ap.parse_args()
    mode = args.mode
    batch = tp._image()[0] if mode == 'rpn' else tp._rcnn_batch()
    torch.manual_seed(0)
    m = FasterRCNN('resnet50', 21, cfg=tp._cfg(), train_mode=mode)
    m.calibrate_bn(tp._image()[0]['data'])
    base = copy.deepcopy(m)
    ref = Trainer(m, mode, fixed_param_prefix=tp.FIXED, lr=0.0, device='cpu')
    _, g_ref = tp._fwd_bwd(ref, batch)
    arms = {}
    if torch.cuda.is_available():
        dev = torch.device('cuda', 0)
        arms['gpu_bf16'] = Trainer(copy.deepcopy(base), mode, fixed_param_prefix=tp.FIXED, lr=0.0, device=dev)
        arms['gpu_fp32'] = Trainer(copy.deepcopy(base), mode, fixed_param_prefix=tp.FIXED, lr=0.0, device=dev,
                                   channels_last=False, precision='torch')
        arms['gpu_bf16x3'] = Trainer(copy.deepcopy(base), mode, fixed_param_prefix=tp.FIXED, lr=0.0, device=dev,
                                     precision='bf16x3')
        arms['gpu_fp32x3'] = Trainer(copy.deepcopy(base), mode, fixed_param_prefix=tp.FIXED, lr=0.0, device=dev,
                                     precision='fp32')
    q = copy.deepcopy(base)
    with torch.no_grad():
        for p in q.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    arms['cpu_bf16in'] = Trainer(q, mode, fixed_param_prefix=tp.FIXED, lr=0.0, device='cpu')
    qa = copy.deepcopy(q)
    _round_storage(qa)
    arms['cpu_bf16act'] = Trainer(qa, mode, fixed_param_prefix=tp.FIXED, lr=0.0, device='cpu')
    for name, tr in arms.items():
        b = dict(batch)
        if name.startswith('cpu_bf16'):
            b['data'] = b['data'].to(torch.bfloat16).float()
        _, g = tp._fwd_bwd(tr, b)
        med, worst, near = stats(g_ref, g)
        print('%-12s median cos %.4f  worst %s' % (name, med, [(round(c, 3), round(r, 3), n) for c, r, n in worst]),
              flush=True)
        print('%-12s near-loss layers %s' % (name, [(round(c, 4), round(r, 3), n) for c, r, n in near]), flush=True)


if __name__ == '__main__':
    main()
