"""Multi-workgroup NMS reducer (csrc/hip/nms.hip nms_reduce_mc_kernel): a chain of workgroups,
each owning 8 column blocks, handing kept words to later workgroups through per-block records.
Checked on batches whose images have different valid counts (0, under one block, block-aligned,
odd), with and without early exit at `post`, against the device flag-loop oracle and the fp32
CPU greedy loop; and with one mask buffer reduced twice (the records clean themselves)."""
import pytest
import torch

from tests.test_detection_ops import nms_mismatch_report, rpn_like_boxes


def _batch(g, B, P):
    boxes = torch.stack([rpn_like_boxes(g, P) for _ in range(B)])
    scores = torch.sort(torch.rand(B, P, generator=g), dim=1, descending=True).values
    return boxes.contiguous(), scores.contiguous()


def _check(C, cuda, boxes, scores, nv, post, out, thresh=0.7):
    from mx_rcnn_amd.ops.nms import _greedy_ref
    _, _, keep, n_keep = out
    bd = boxes.to(cuda)
    nvd = nv.to(cuda)
    res = C.nms_check(bd, nvd, thresh, post, keep, n_keep).cpu()
    for b in range(boxes.shape[0]):
        nk = int(n_keep[b])
        assert int(res[b, 0]) == -1 and int(res[b, 1]) == nk, (b, res[b].tolist(), nk)
        n = int(nv[b])
        ref = torch.tensor(_greedy_ref(boxes[b, :max(n, 1)], n, thresh, post, fp32=True), dtype=torch.long)
        got = keep[b, :nk].cpu()
        assert torch.equal(ref, got), nms_mismatch_report(boxes[b], ref, got, thresh, (b, n, post))
        if nk:  # padded slots repeat kept boxes
            pad = keep[b, nk:].cpu()
            assert bool(torch.isin(pad, got).all())


@pytest.mark.gpu
@pytest.mark.parametrize('P,post', [(12000, 2000), (12000, 12000), (6000, 300), (3000, 3000), (1100, 2000)])
def test_multi_workgroup_nms_batched(cuda, P, post):
    from mx_rcnn_amd.ops import need_ext
    C = need_ext()
    g = torch.Generator().manual_seed(P + post)
    B = 5
    boxes, scores = _batch(g, B, P)
    nv = torch.tensor([P, 0, 37, min(P, 1024), P - 65], dtype=torch.int32)
    u = torch.rand(B, post, generator=g).to(cuda)
    out = C.nms_proposals(boxes.to(cuda), scores.to(cuda), nv.to(cuda), 0.7, post, u)
    torch.cuda.synchronize()
    _check(C, cuda, boxes, scores, nv, post, out)
    assert int(out[3][1]) == 0


@pytest.mark.gpu
def test_multi_workgroup_nms_mask_reused(cuda):
    """The two-phase path (nms_mask_build, then nms_proposals with that mask) run twice on one
    mask buffer: the second reduce must not see the first one's records."""
    from mx_rcnn_amd.ops import need_ext
    C = need_ext()
    g = torch.Generator().manual_seed(5)
    P, post = 9000, 9000
    boxes, scores = _batch(g, 2, P)
    nv = torch.tensor([P, 4000], dtype=torch.int32)
    bd, sd, nvd = boxes.to(cuda), scores.to(cuda), nv.to(cuda)
    u = torch.rand(2, post, generator=g).to(cuda)
    mask = C.nms_mask_build(bd, nvd, 0.7)
    first = [t.clone() for t in C.nms_proposals(bd, sd, nvd, 0.7, post, u, mask)]
    second = C.nms_proposals(bd, sd, nvd, 0.7, post, u, mask)
    torch.cuda.synchronize()
    for a, b in zip(first, second):
        assert torch.equal(a, b)
    _check(C, cuda, boxes, scores, nv, post, second)


@pytest.mark.gpu
def test_multi_workgroup_nms_give_up_is_reported(cuda, monkeypatch):
    """MXR_NMS_SPIN=0: a workgroup whose first poll finds an earlier workgroup's record unwritten
    gives up at once.  The kernel must still drain, add to the caller's fault counter (the Trainer
    passes its non-finite counter, so check_finite raises), and leave the records clean: the next
    reduce on the same mask with the default poll budget is exact and reports nothing."""
    from mx_rcnn_amd.ops import need_ext
    C = need_ext()
    g = torch.Generator().manual_seed(9)
    P, post = 12000, 12000
    boxes, scores = _batch(g, 1, P)
    nv = torch.tensor([P], dtype=torch.int32)
    bd, sd, nvd = boxes.to(cuda), scores.to(cuda), nv.to(cuda)
    u = torch.rand(1, post, generator=g).to(cuda)
    mask = C.nms_mask_build(bd, nvd, 0.7)
    fault = torch.zeros(1, dtype=torch.int32, device=cuda)
    monkeypatch.setenv('MXR_NMS_SPIN', '0')
    C.nms_proposals(bd, sd, nvd, 0.7, post, u, mask, fault)
    torch.cuda.synchronize()
    assert int(fault.item()) > 0  # 24 workgroups in a chain, none allowed to wait
    monkeypatch.delenv('MXR_NMS_SPIN')
    fault.zero_()
    out = C.nms_proposals(bd, sd, nvd, 0.7, post, u, mask, fault)
    torch.cuda.synchronize()
    assert int(fault.item()) == 0
    _check(C, cuda, boxes, scores, nv, post, out)
