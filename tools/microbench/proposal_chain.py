"""Isolated timing of the proposal chain's serial-looking kernels on one GPU: the NMS reduce
(csrc/hip/nms.hip; mask prebuilt, so only the reducer is timed) on proposal-shaped boxes at the
training (12000 -> 2000) and test (6000 -> 300) sizes, and the R-CNN proposal-target sampler
(csrc/hip/sample.hip proposal_sample, 2000 RoIs + gt, 128 samples, 81 classes).

    python tools/microbench/proposal_chain.py            # multi-workgroup NMS (default)
    MXR_NMS_SERIAL=1 python tools/microbench/proposal_chain.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _time(fn, reps=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def probe_summary(mask, P, per, tick_ns=10.0):
    """The reducer's MXR_NMS_PROBE timeline (B = 1; wall clock at 100 MHz): per workgroup the wait
    in phase A, phase B, and the hand-off from the previous workgroup's last publish; per block
    the resolve time and fixpoint rounds."""
    nb = (P + 63) // 64
    pp = ((nb + 1) // 2) * 128
    base = nb * pp + nb * 2 + 1
    pr = mask[base:base + nb * 8].cpu().view(-1)
    blk, wg = pr[:nb * 4].view(nb, 4), pr[nb * 4:].view(nb, 4)
    G = (nb + per - 1) // per
    t0 = int(wg[:G, 0].min())
    us = lambda v: round((int(v) - t0) * tick_ns / 1e3, 2)
    done = [t for t in range(nb) if int(blk[t, 1]) > 0]
    last = max(done) if done else -1
    rows = []
    for w in range(G):
        lo = w * per
        if lo > last:
            break
        hand = None
        if lo > 0:
            hand = round((int(blk[lo, 0]) - int(blk[lo - 1, 1])) * tick_ns / 1e3, 2)
        rows.append({'wg': w, 'start': us(wg[w, 0]), 'phaseA_done': us(wg[w, 1]), 'phaseB_done': us(wg[w, 2]),
                     'end': us(wg[w, 3]), 'handoff_us': hand})
    res = [(int(blk[t, 1]) - int(blk[t, 0])) * tick_ns / 1e3 for t in done]
    rounds = [int(blk[t, 2]) for t in done]
    inner = [(int(blk[t + 1, 0]) - int(blk[t, 1])) * tick_ns / 1e3 for t in done if t + 1 in done and (t + 1) % per]
    return {'probe': 'nms_reduce_mc', 'P': P, 'per': per, 'blocks': len(done),
            'resolve_us_mean': round(sum(res) / max(len(res), 1), 3), 'resolve_us_max': round(max(res or [0]), 3),
            'next_block_gap_us_mean': round(sum(inner) / max(len(inner), 1), 3),
            'fixpoint_rounds_mean': round(sum(rounds) / max(len(rounds), 1), 2), 'fixpoint_rounds_max': max(rounds or [0]),
            'last_publish_us': us(blk[last, 1]) if last >= 0 else None, 'workgroups': rows}


def main():
    from mx_rcnn_amd.ops import need_ext
    from tests.test_detection_ops import rpn_like_boxes
    C = need_ext()
    dev = torch.device('cuda', 0)
    g = torch.Generator().manual_seed(0)
    mode = 'serial' if os.environ.get('MXR_NMS_SERIAL') == '1' else 'multi_wg_per%s' % os.environ.get('MXR_NMS_PER', '8')
    for P, post in [(12000, 2000), (12000, 6000), (6000, 300), (12000, 12000)]:
        b = rpn_like_boxes(g, P)[None].to(dev)
        s = torch.sort(torch.rand(1, P, generator=g), dim=1, descending=True).values.to(dev)
        nv = torch.tensor([P], dtype=torch.int32, device=dev)
        u = torch.rand(1, post, generator=g).to(dev)
        mask = C.nms_mask_build(b, nv, 0.7)
        us_mask = _time(lambda: C.nms_mask_build(b, nv, 0.7))
        us = _time(lambda: C.nms_proposals(b, s, nv, 0.7, post, u, mask))
        nk = int(C.nms_proposals(b, s, nv, 0.7, post, u, mask)[3][0])
        print(json.dumps({'op': 'nms_reduce', 'mode': mode, 'P': P, 'post': post, 'n_keep': nk,
                          'reduce_us': round(us, 1), 'mask_us': round(us_mask, 1)}), flush=True)
        if os.environ.get('MXR_NMS_PROBE') == '1' and mode != 'serial':
            print(json.dumps(probe_summary(mask, P, int(os.environ.get('MXR_NMS_PER', '8')))), flush=True)
    # proposal-target sampler at the e2e training shape
    P, G, R, F, NC = 2000, 8, 128, 32, 81
    rois = torch.zeros(1, P, 5)
    rois[0, :, 1:] = rpn_like_boxes(g, P)
    gt = torch.full((1, G, 5), -1.0)
    gt[0, :5, :4] = rpn_like_boxes(g, 5)
    gt[0, :5, 4] = torch.randint(1, NC, (5,), generator=g).float()
    n_gt = torch.tensor([5], dtype=torch.int32)
    ov = torch.rand(1, P, generator=g)
    am = torch.randint(0, 5, (1, P), generator=g, dtype=torch.int32)
    rnd = torch.rand(1, 2 * (P + G) + R, generator=g)
    args = [t.to(dev) for t in (rois, gt, n_gt, ov, am, rnd)]
    us = _time(lambda: C.proposal_sample(*args, R, F, NC, 0.5, 0.5, 0.0, True, True, [0.0] * 4, [0.1, 0.1, 0.2, 0.2],
                                         [1.0] * 4))
    print(json.dumps({'op': 'proposal_sample', 'P': P, 'R': R, 'C': NC, 'us': round(us, 1)}), flush=True)


if __name__ == '__main__':
    main()
