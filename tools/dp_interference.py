"""How much does a data-parallel all-reduce's CU share cost the compute stream?  

An RCCL ring all-reduce runs one workgroup per channel on every GPU for as long as a gradient
bucket reduces -- about 1.1 ms per step for ResNet-101's 184 MB fp32 gradients on 8 GPUs over
xGMI (SURVEY §5.8's ring estimate) -- and those workgroups occupy compute units that the
overlapped backward wants.  This probe replays the graphed single-GPU training step while a side
stream holds k compute units for the same time (csrc/hip/probe.hip):

  spin  k workgroups of 512 threads waiting on the real-time counter (channels waiting on
        flags / the link: occupancy only)
  copy  k workgroups streaming a buffer copy sized to last about as long (occupancy + HBM
        traffic of the reduce / copy steps)

and reports the step time against the step alone, for k in {0, 8, 16, 32, 64}.  The side work is
issued right after each replay (host order), so it overlaps the whole step, like a bucket
all-reduce that starts early in the backward.

    python tools/dp_interference.py [--dtype fp32] [--steps 30] [--us 1100]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16x3', 'bf16'])
    ap.add_argument('--network', default='resnet101')
    ap.add_argument('--steps', type=int, default=30)
    ap.add_argument('--us', type=float, default=1100.0, help='side-work duration per step (us)')
    ap.add_argument('--ks', default='0,8,16,32,64')
    a = ap.parse_args()
    from bench import synthetic_batch
    from mx_rcnn_amd.config import snapshot
    from mx_rcnn_amd.core.trainer import Trainer, GraphedStep
    from mx_rcnn_amd.models import FasterRCNN
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    dev = torch.device('cuda', 0)
    cfg = snapshot()
    cfg.TRAIN.BG_THRESH_LO = 0.0
    cfg.END2END = 1
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    torch.manual_seed(0)
    model = FasterRCNN(a.network, 81, cfg=cfg)
    gen = torch.Generator().manual_seed(1)
    batch = synthetic_batch(1, 800, 1333, 81, dev, gen)
    model.to(dev).calibrate_bn(batch['data'])
    tr = Trainer(model, 'e2e', fixed_param_prefix=['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'], lr=0.001,
                 momentum=0.9, wd=0.0005, clip_gradient=1.0, device=dev, precision=a.dtype)
    step = GraphedStep(tr, batch, warmup=3)
    side = torch.cuda.Stream(device=dev)
    # copy buffers: size the copy so k = 16 workgroups take about --us alone
    n = 1 << 24
    src = torch.randn(n, device=dev)
    dst = torch.empty_like(src)

    def copy_time(k, elems):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        ext.cu_copy(src[:elems], dst[:elems], k)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) * 1e3

    def run(mode, k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step(batch)
            if k > 0:
                with torch.cuda.stream(side):
                    if mode == 'spin':
                        ext.cu_spin(k, a.us)
                    else:
                        ext.cu_copy(src[:elems[k]], dst[:elems[k]], k)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3

    ks = [int(v) for v in a.ks.split(',')]
    elems = {}
    for k in ks:
        if k > 0:  # elements that k workgroups copy in about --us
            t = copy_time(k, n)
            elems[k] = max(4, min(n, int(n * a.us / max(t, 1e-3)) // 4 * 4))
    for _ in range(3):
        step(batch)
    base = run('spin', 0)
    rows = []
    for k in ks:
        for mode in ('spin', 'copy'):
            if k == 0 and mode == 'copy':
                continue
            ms = run(mode, k) if k else base
            rec = {'dtype': a.dtype, 'mode': mode, 'k_cus': k, 'side_us': a.us if k else 0,
                   'step_ms': round(ms, 3), 'slowdown_pct': round(100 * (ms / base - 1), 2)}
            if mode == 'copy' and k:
                rec['copy_mb'] = round(elems[k] * 4 * 2 / 1e6, 1)
            rows.append(rec)
            print(json.dumps(rec), flush=True)
    # interleaved repeat of the baseline (box noise)
    print(json.dumps({'dtype': a.dtype, 'mode': 'spin', 'k_cus': 0, 'step_ms': round(run('spin', 0), 3),
                      'repeat': True}), flush=True)


if __name__ == '__main__':
    main()
