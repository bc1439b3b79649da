"""Find which op of the training step refuses hipGraph stream capture."""
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from mx_rcnn_amd import ops
from mx_rcnn_amd.config import snapshot


def try_capture(name, fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g):
            fn()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        print('[capture] OK   ', name, flush=True)
    except Exception as e:
        print('[capture] FAIL ', name, type(e).__name__, str(e).splitlines()[0][:200], flush=True)
        traceback.print_exc(limit=6)
        torch.cuda.synchronize()


def main():
    dev = torch.device('cuda')
    cfg = snapshot()
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    A, H, W = 12, 50, 84
    cls = torch.randn(1, 2 * A, H, W, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    dlt = (torch.randn(1, 4 * A, H, W, device=dev) * 0.1).bfloat16().contiguous(memory_format=torch.channels_last)
    im_info = torch.tensor([[800., 1333., 1.]], device=dev)
    gt = torch.tensor([[[20., 30, 200, 220, 3], [100, 50, 400, 300, 17]]], device=dev)
    n_gt = torch.tensor([2], dtype=torch.int32, device=dev)
    keys = torch.rand(1, 50400, device=dev)
    try_capture('sort', lambda: torch.sort(keys, dim=1, descending=True, stable=True))
    try_capture('rand', lambda: torch.rand(1, 6000, device=dev))
    try_capture('proposal_decode', lambda: ops.need_ext().proposal_decode(
        cls, dlt, im_info, ops.base_anchors(16, (4, 8, 16, 32), (0.5, 1, 2), dev), 16.0, 16.0, True, False))
    try_capture('proposal', lambda: ops.proposal(cls, dlt, im_info, 16, (4, 8, 16, 32), (0.5, 1, 2), 12000, 6000,
                                                 0.7, 16, is_train=True))
    try_capture('anchor_target', lambda: ops.anchor_target((H, W), gt, n_gt, im_info, scales=(4, 8, 16, 32),
                                                           cfg=cfg))
    rois = torch.cat([torch.zeros(1, 6000, 1, device=dev), torch.rand(1, 6000, 4, device=dev).mul(400).sort(-1)[0]],
                     -1)
    try_capture('proposal_target', lambda: ops.proposal_target(rois, gt, n_gt, 81, cfg=cfg))
    feat = torch.randn(1, 1024, H, W, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    feat.requires_grad_()
    r = rois[0, :128].contiguous()

    def rp():
        out = ops.roi_pool(feat, r, (7, 7), 1 / 16)
        out.sum().backward()
    try_capture('roi_pool fwd+bwd', rp)
    lab = torch.randint(-1, 2, (1, A * H * W), device=dev)
    clsr = cls.clone().requires_grad_()

    def ce():
        ops.rpn_softmax_ce(clsr, lab).backward()
    try_capture('rpn_ce', ce)
    x = torch.randn(1, 256, H, W, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    gmm = torch.ones(256, device=dev, requires_grad=True)
    bt = torch.zeros(256, device=dev, requires_grad=True)
    mu, var = torch.zeros(256, device=dev), torch.ones(256, device=dev)
    x.requires_grad_()

    def bn():
        ops.frozen_bn_relu(x, gmm, bt, mu, var).sum().backward()
    try_capture('bn_relu', bn)
    w = torch.randn(256, 256, 3, 3, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    w.requires_grad_()
    from mx_rcnn_amd.ops.conv import conv2d

    def cv():
        conv2d(x, w, None, 1, 1).sum().backward()
    try_capture('conv_igemm fwd+bwd', cv)
    xs = x.detach().clone().requires_grad_()

    def tbn():
        torch.nn.functional.batch_norm(xs, torch.zeros(256, device=dev), torch.ones(256, device=dev),
                                       gmm.bfloat16(), bt.bfloat16(), training=True).sum().backward()
    try_capture('train-mode batch_norm', tbn)


if __name__ == '__main__':
    main()
