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
def test_multi_workgroup_nms_give_up_falls_back_to_serial(cuda, monkeypatch):
    """MXR_NMS_SPIN=0: a workgroup whose first poll finds an earlier workgroup's record unwritten
    gives up at once.  The chain must still drain and leave its records clean, and the serial
    reducer launched behind it must finish the image: the output is the oracle's keep list, and the
    caller's give-up counter says how many images were redone.  The next reduce on the same mask
    with the default poll budget is exact and redoes nothing."""
    from mx_rcnn_amd.ops import need_ext
    C = need_ext()
    g = torch.Generator().manual_seed(9)
    P, post = 12000, 12000
    boxes, scores = _batch(g, 2, P)
    nv = torch.tensor([P, P - 700], dtype=torch.int32)
    bd, sd, nvd = boxes.to(cuda), scores.to(cuda), nv.to(cuda)
    u = torch.rand(2, post, generator=g).to(cuda)
    mask = C.nms_mask_build(bd, nvd, 0.7)
    gave_up = torch.zeros(1, dtype=torch.int32, device=cuda)
    monkeypatch.setenv('MXR_NMS_SPIN', '0')
    out = C.nms_proposals(bd, sd, nvd, 0.7, post, u, mask, gave_up)
    torch.cuda.synchronize()
    assert int(gave_up.item()) >= 1  # 24 workgroups per image in a chain, none allowed to wait
    _check(C, cuda, boxes, scores, nv, post, out)
    monkeypatch.delenv('MXR_NMS_SPIN')
    gave_up.zero_()
    out2 = C.nms_proposals(bd, sd, nvd, 0.7, post, u, mask, gave_up)
    torch.cuda.synchronize()
    assert int(gave_up.item()) == 0
    for a, b in zip(out, out2):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_training_step_survives_nms_give_up(cuda, monkeypatch):
    """A whole graphed training step with every NMS chain giving up (MXR_NMS_SPIN=0) runs to the
    end without raising, counts the redone images, and trains to the same weights as the default
    step (the serial fallback reproduces the chain's keep list bit for bit)."""
    from mx_rcnn_amd.core.trainer import GraphedStep, Trainer
    from mx_rcnn_amd.models import FasterRCNN
    from tests.test_model import _batch, _cfg
    cfg = _cfg()
    cfg.TRAIN.RPN_PRE_NMS_TOP_N = 6000  # 94 column blocks: a chain of 12 workgroups
    cfg.TRAIN.RPN_POST_NMS_TOP_N = 2000
    b = {k: v.to(cuda) for k, v in _batch(320, 480).items()}

    def run(spin):
        if spin is None:
            monkeypatch.delenv('MXR_NMS_SPIN', raising=False)
        else:
            monkeypatch.setenv('MXR_NMS_SPIN', str(spin))
        torch.manual_seed(0)
        m = FasterRCNN('resnet50', 21, cfg=cfg)
        tr = Trainer(m, 'e2e', fixed_param_prefix=['conv0', 'stage1', 'bn_data', 'bn0'], lr=0.01, device=cuda)
        torch.manual_seed(10)
        tr.step(b)
        g = GraphedStep(tr, b, warmup=1)
        for _ in range(2):
            g(b)
        tr.check_finite()  # the give-up is not a failure any more
        torch.cuda.synchronize()
        return {'gave_up': int(m.nms_gave_up.item()),
                'weights': {k: v.detach().clone() for k, v in tr.store.state_arrays().items()}}

    base = run(None)
    got = run(0)
    assert base['gave_up'] == 0
    assert got['gave_up'] > 0
    for k in base['weights']:
        assert torch.equal(base['weights'][k], got['weights'][k]), k
