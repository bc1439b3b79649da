"""Run-twice repeatability of the detection hot paths (SURVEY 5.2 determinism tests).

Proposal (decode + top-k + NMS), the proposal NMS kernel and the RoI max-pool forward are
run twice on the same inputs and compared bitwise: none of them may depend on wave
scheduling (the NMS bitmask reduce, the keyed sort and the first-maximum RoI pool are all
order-independent by construction).  The RNG-dependent tail (random padding of the post-NMS
list in training mode) is pinned by re-seeding before each call.
"""
import pytest
import torch

from mx_rcnn_amd import ops
from tests.test_detection_ops import LARGE_NMS, _rpn_inputs, rand_boxes, rpn_like_boxes
from tests.test_kernels import _rois

KW = dict(feat_stride=16, scales=(8, 16, 32), ratios=(0.5, 1, 2), pre_nms_top_n=6000, post_nms_top_n=300,
          nms_thresh=0.7, min_size=16)


def _twice(fn):
    torch.manual_seed(123)
    a = fn()
    torch.manual_seed(123)
    b = fn()
    return a, b


@pytest.mark.parametrize('train', [True, False])
def test_proposal_cpu_repeatable(train):
    cls, dlt = _rpn_inputs(3, 9, 30, 40)
    im_info = torch.tensor([[480.0, 640.0, 1.0]])
    (r1, s1), (r2, s2) = _twice(lambda: ops.proposal(cls, dlt, im_info, is_train=train, **KW))
    assert torch.equal(r1, r2) and torch.equal(s1, s2)


def test_roi_pool_cpu_repeatable():
    g = torch.Generator().manual_seed(5)
    feat = torch.randn(2, 16, 30, 40, generator=g)
    rois = _rois(g, 128, 2, 30, 40)
    o1, o2 = _twice(lambda: ops.roi_pool(feat, rois, (7, 7), 1 / 16))
    assert torch.equal(o1, o2)


@pytest.mark.gpu
@pytest.mark.parametrize('train', [True, False])
def test_proposal_gpu_repeatable(cuda, train):
    cls, dlt = _rpn_inputs(4, 9, 38, 63, B=2)
    cl = cls.to(cuda).contiguous(memory_format=torch.channels_last)
    dl = dlt.to(cuda).contiguous(memory_format=torch.channels_last)
    im_info = torch.tensor([[600.0, 1000.0, 1.0], [590.0, 950.0, 1.5]], device=cuda)
    (r1, s1), (r2, s2) = _twice(lambda: ops.proposal(cl, dl, im_info, is_train=train, **KW))
    torch.cuda.synchronize()
    assert torch.equal(r1, r2) and torch.equal(s1, s2)


@pytest.mark.gpu
def test_nms_proposals_gpu_repeatable(cuda):
    from mx_rcnn_amd.ops import need_ext
    C = need_ext()
    g = torch.Generator().manual_seed(21)
    P, post = 12000, 6000
    b = rand_boxes(g, P, 1300)[None].to(cuda)
    s = torch.sort(torch.rand(P, generator=g), descending=True).values[None].to(cuda).contiguous()
    nv = torch.tensor([P], dtype=torch.int32, device=cuda)
    u = torch.rand(1, post, generator=g).to(cuda)
    out1 = [t.clone() for t in C.nms_proposals(b, s, nv, 0.7, post, u)]
    out2 = C.nms_proposals(b, s, nv, 0.7, post, u)
    torch.cuda.synchronize()
    for x, y in zip(out1, out2):
        assert torch.equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize('P,post', LARGE_NMS)
def test_nms_proposals_gpu_repeatable_large(cuda, P, post):
    """The RPN-dump shapes (tools/test_rpn.py: pre-NMS = all anchors) reach the reducer's
    beyond-window fold and, with post < kept, its early exit: run twice, bitwise equal."""
    from mx_rcnn_amd.ops import need_ext
    C = need_ext()
    g = torch.Generator().manual_seed(7 * P + post)
    pst = P if post < 0 else post
    b = rpn_like_boxes(g, P)[None].to(cuda)
    s = torch.sort(torch.rand(P, generator=g), descending=True).values[None].to(cuda).contiguous()
    nv = torch.tensor([P], dtype=torch.int32, device=cuda)
    u = torch.rand(1, pst, generator=g).to(cuda)
    out1 = [t.clone() for t in C.nms_proposals(b, s, nv, 0.7, pst, u)]
    out2 = C.nms_proposals(b, s, nv, 0.7, pst, u)
    torch.cuda.synchronize()
    for x, y in zip(out1, out2):
        assert torch.equal(x, y)


@pytest.mark.gpu
def test_roi_pool_gpu_repeatable(cuda):
    g = torch.Generator().manual_seed(6)
    feat = torch.randn(2, 256, 38, 50, generator=g).to(cuda, torch.bfloat16)
    feat = feat.contiguous(memory_format=torch.channels_last)
    rois = _rois(g, 256, 2, 38, 50).to(cuda)
    o1, o2 = _twice(lambda: ops.roi_pool(feat, rois, (7, 7), 1 / 16))
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
