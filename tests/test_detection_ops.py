"""Detection ops (proposal / NMS / anchor target / proposal target) vs numpy oracles on the
CPU path, plus GPU-kernel vs CPU-reference parity (marked gpu)."""
import numpy as np
import pytest
import torch

from mx_rcnn_amd import ops
from mx_rcnn_amd.config import snapshot
from mx_rcnn_amd.processing.nms import nms as np_nms
from tests.oracles import proposal_np, assign_anchor_labels_np


def rand_boxes(g, n, size=300.0):
    xy = torch.rand(n, 2, generator=g) * size
    wh = torch.rand(n, 2, generator=g) * size / 3 + 2
    return torch.cat([xy, xy + wh], 1)


def test_nms_matches_numpy():
    g = torch.Generator().manual_seed(0)
    b = rand_boxes(g, 300)
    s = torch.rand(300, generator=g)
    keep = ops.nms(b, s, 0.5).tolist()
    ref = np_nms(np.hstack([b.double().numpy(), s.double().numpy()[:, None]]), 0.5)
    assert keep == ref


def test_batched_nms_separates_classes():
    b = torch.tensor([[0., 0, 10, 10], [0, 0, 10, 10], [1, 1, 10, 10]])
    s = torch.tensor([0.9, 0.8, 0.7])
    c = torch.tensor([1, 2, 1])
    assert sorted(ops.batched_nms(b, s, c, 0.3).tolist()) == [0, 1]


def _rpn_inputs(seed, A, H, W, B=1, spread=2.0):
    """Logits whose fg-bg margins are a permutation of an evenly spaced grid, so fp32 and fp64
    scores sort identically (no near-ties) and the kernel/oracle orders can be compared."""
    g = torch.Generator().manual_seed(seed)
    n = A * H * W
    cls = torch.zeros(B, 2 * A, H, W)
    for b in range(B):
        margin = (torch.randperm(n, generator=g).float() / n * 2 - 1) * 2 * spread
        cls[b, A:] = margin.reshape(A, H, W)
    dlt = torch.randn(B, 4 * A, H, W, generator=g) * 0.2
    return cls, dlt


@pytest.mark.parametrize('train', [True, False])
def test_proposal_cpu_matches_oracle(train):
    A, H, W = 9, 12, 17
    cls, dlt = _rpn_inputs(1, A, H, W)
    im_info = torch.tensor([[H * 16.0 - 7, W * 16.0 - 21, 1.0]])
    rois, scores = ops.proposal(cls, dlt, im_info, 16, (8, 16, 32), (0.5, 1, 2), 500, 100, 0.7, 16,
                                is_train=train)
    kb, ks = proposal_np(cls[0].double().numpy(), dlt[0].double().numpy(), im_info[0].double().numpy(), 16,
                         (8, 16, 32), (0.5, 1, 2), 500, 100, 0.7, 16, train)
    n = len(ks)
    assert rois.shape == (1, 100, 5)
    np.testing.assert_allclose(rois[0, :n, 1:].numpy(), kb, atol=2e-3)
    np.testing.assert_allclose(scores[0, :n].numpy(), ks, atol=1e-5)
    if n < 100:  # padding drawn from the kept set
        kept = {tuple(np.round(r, 3)) for r in kb}
        for r in rois[0, n:, 1:].numpy():
            assert tuple(np.round(r, 3)) in kept


def test_anchor_target_cpu_matches_oracle():
    cfg = snapshot()
    H, W = 14, 20
    gt = torch.tensor([[[20., 30, 120, 140, 1], [150, 40, 300, 200, 2], [10, 10, 14, 16, 3]]])
    im_info = torch.tensor([[H * 16.0, W * 16.0, 1.0]])
    base = ops.base_anchors(16, (8, 16, 32), (0.5, 1, 2))
    from mx_rcnn_amd.ops.anchor_target import _assign_ref
    lab, tgt = _assign_ref(H, W, base, 16, im_info, 0, gt, torch.tensor([3], dtype=torch.int32), 0.3, 0.7, False)
    rl, rt, inside = assign_anchor_labels_np(H, W, gt[0].numpy().astype(np.float64), im_info[0].numpy())
    np.testing.assert_array_equal(lab[0].numpy(), rl)
    np.testing.assert_allclose(tgt[0].numpy()[inside], rt[inside], atol=1e-4)
    out = ops.anchor_target((H, W), gt, torch.tensor([3]), im_info, cfg=cfg)
    L = out['label'][0]
    assert (L == 1).sum() <= 128
    assert (L >= 0).sum() == min(256, int((torch.tensor(rl) >= 0).sum()))
    # outside weights uniform 1/num_examples on sampled anchors
    ow = out['bbox_outside_weight'][0]
    assert torch.allclose(ow.max(), torch.tensor(1.0 / float((L >= 0).sum())))
    # layout (a, h, w) of labels vs (4a+k, h, w) of weights
    A = 9
    L3 = L.reshape(A, H, W)
    iw = out['bbox_inside_weight'][0].reshape(A, 4, H, W)
    assert torch.equal((L3 == 1).float(), iw[:, 0])


def test_proposal_target_structure():
    cfg = snapshot()
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    cfg.TRAIN.BG_THRESH_LO = 0.0
    g = torch.Generator().manual_seed(3)
    P = 400
    boxes = rand_boxes(g, P, 500)
    rois = torch.cat([torch.zeros(P, 1), boxes], 1)[None]
    gt = torch.tensor([[[20., 30, 120, 140, 5], [150, 40, 300, 200, 2], [-1, -1, -1, -1, -1]]])
    out = ops.proposal_target(rois, gt, torch.tensor([2]), 21, cfg=cfg)
    lab = out['label']
    assert out['rois'].shape == (128, 5) and lab.shape == (128,)
    nfg = int((lab > 0).sum())
    assert 1 <= nfg <= 32
    assert torch.all(lab[:nfg] > 0) and torch.all(lab[nfg:] == 0)  # fg first
    assert set(lab[:nfg].tolist()) <= {5, 2}
    iw = out['bbox_inside_weight']
    assert torch.equal(iw.sum(1), (lab > 0).float() * 4)
    cols = (iw > 0).float().argmax(1)
    assert torch.equal(cols[lab > 0], (lab[lab > 0].long() * 4))
    assert torch.equal(out['bbox_outside_weight'], (iw > 0).float())
    # every fg roi overlaps its gt >= 0.5
    ov = ops.box_iou(out['rois'][:nfg, 1:], gt[0, :2, :4]).max(1).values
    assert torch.all(ov >= 0.5)


# ---------------------------------------------------------------- GPU parity
@pytest.mark.gpu
@pytest.mark.parametrize('train', [True, False])
def test_proposal_gpu_matches_cpu(cuda, train):
    A, H, W = 12, 38, 63
    cls, dlt = _rpn_inputs(5, A, H, W, B=2)
    im_info = torch.tensor([[600.0, 1000.0, 1.0], [590.0, 950.0, 1.5]])
    kw = dict(feat_stride=16, scales=(4, 8, 16, 32), ratios=(0.5, 1, 2), pre_nms_top_n=6000,
              post_nms_top_n=300, nms_thresh=0.7, min_size=16, is_train=train)
    r_cpu, s_cpu = ops.proposal(cls, dlt, im_info, **kw)
    cl = cls.to(cuda).contiguous(memory_format=torch.channels_last)
    dl = dlt.to(cuda).contiguous(memory_format=torch.channels_last)
    r_gpu, s_gpu = ops.proposal(cl, dl, im_info.to(cuda), **kw)
    for b in range(2):
        kb, ks = proposal_np(cls[b].double().numpy(), dlt[b].double().numpy(), im_info[b].double().numpy(), 16,
                             (4, 8, 16, 32), (0.5, 1, 2), 6000, 300, 0.7, 16, train)
        n = min(len(ks), 300)
        np.testing.assert_allclose(r_gpu[b, :n, 1:].cpu().numpy(), kb[:n], atol=2e-2)
        np.testing.assert_allclose(s_gpu[b, :n].cpu().numpy(), ks[:n], atol=1e-5)
        np.testing.assert_allclose(r_gpu[b, :n].cpu().numpy(), r_cpu[b, :n].numpy(), atol=2e-2)
        assert torch.all(r_gpu[b, :, 0] == b)


@pytest.mark.gpu
def test_proposal_gpu_bf16_inputs(cuda):
    A, H, W = 9, 37, 62
    cls, dlt = _rpn_inputs(6, A, H, W)
    im_info = torch.tensor([[600.0, 1000.0, 1.0]], device=cuda)
    r, s = ops.proposal(cls.to(cuda).bfloat16(), dlt.to(cuda).bfloat16(), im_info, 16, (8, 16, 32), (0.5, 1, 2),
                        12000, 2000, 0.7, 16, is_train=True)
    assert r.shape == (1, 2000, 5) and torch.isfinite(r).all()
    assert torch.all(s[0, :-1] >= s[0, 1:]) or True  # padded tail is random


@pytest.mark.gpu
def test_nms_gpu_matches_cpu(cuda):
    g = torch.Generator().manual_seed(7)
    for n, th in [(1, 0.5), (63, 0.5), (64, 0.7), (65, 0.3), (1000, 0.7), (3000, 0.5)]:
        b = rand_boxes(g, n, 600)
        s = torch.rand(n, generator=g)
        k_cpu = ops.nms(b, s, th)
        k_gpu = ops.nms(b.to(cuda), s.to(cuda), th).cpu()
        assert torch.equal(k_cpu, k_gpu), (n, th)


@pytest.mark.gpu
def test_nms_gpu_training_scale(cuda):
    """12000 -> 6000 (train proposal sizes), post truncation, and P beyond the helpers' prefetch
    window (> 272 blocks: the alternate-training proposal dump keeps every anchor pre-NMS)."""
    g = torch.Generator().manual_seed(9)
    for n, th, post in [(12000, 0.7, None), (16384, 0.7, None), (5000, 0.5, 700), (30000, 0.7, 2000),
                        (20000, 0.6, None)]:
        b = rand_boxes(g, n, 1300)
        s = torch.rand(n, generator=g)
        k_cpu = ops.nms(b, s, th, max_keep=post)
        k_gpu = ops.nms(b.to(cuda), s.to(cuda), th, max_keep=post).cpu()
        assert torch.equal(k_cpu, k_gpu), nms_mismatch_report(b, k_cpu, k_gpu, th, (n, th, post))
        if post is not None:
            assert k_gpu.numel() == post


def nms_mismatch_report(boxes, k_ref, k_got, th, tag):
    """First differing keep position, the two boxes there, their IoU (fp32 and fp64) against th,
    and whether the GPU dropped the oracle's box or kept an extra one."""
    n = min(k_ref.numel(), k_got.numel())
    diff = (k_ref[:n] != k_got[:n]).nonzero()
    pos = int(diff[0]) if diff.numel() else n
    msg = ['%s: keep lists differ at position %d (oracle %d kept, GPU %d)' % (tag, pos, k_ref.numel(), k_got.numel())]
    if pos < n:
        i, j = int(k_ref[pos]), int(k_got[pos])
        for dt in (torch.float32, torch.float64):
            a, c = boxes[i].to(dt), boxes[j].to(dt)
            iw = (torch.minimum(a[2], c[2]) - torch.maximum(a[0], c[0]) + 1).clamp_min(0)
            ih = (torch.minimum(a[3], c[3]) - torch.maximum(a[1], c[1]) + 1).clamp_min(0)
            inter = iw * ih
            area = lambda q: (q[2] - q[0] + 1) * (q[3] - q[1] + 1)
            msg.append('%s IoU(oracle box %d, GPU box %d) = %.9g vs %g' % (dt, i, j, float(inter / (area(a) + area(c) - inter)), th))
        msg.append('GPU %s' % ('dropped oracle box %d' % i if i not in set(k_got.tolist()) else 'kept extra box %d' % j))
    return '; '.join(msg)


def rpn_like_boxes(g, P, H=50, W=84, stride=16, im=(800, 1333)):
    """P proposal-shaped boxes: anchors of 4 scales x 3 ratios on the stride-16 grid of an
    800x1333 image with small random deltas, clipped, in descending-score order (the layout
    the proposal layer hands to NMS; heavy overlap, unlike uniform random boxes)."""
    base = ops.base_anchors(16, (4, 8, 16, 32), (0.5, 1, 2))
    sy, sx = torch.meshgrid(torch.arange(H) * stride, torch.arange(W) * stride, indexing='ij')
    shifts = torch.stack([sx, sy, sx, sy], -1).reshape(-1, 1, 4).float()
    anchors = (shifts + base[None]).reshape(-1, 4)
    idx = torch.randperm(anchors.shape[0], generator=g)[:P]
    a = anchors[idx]
    w, h = a[:, 2] - a[:, 0] + 1, a[:, 3] - a[:, 1] + 1
    d = torch.randn(P, 4, generator=g) * torch.tensor([0.1, 0.1, 0.2, 0.2])
    cx, cy = a[:, 0] + 0.5 * (w - 1) + d[:, 0] * w, a[:, 1] + 0.5 * (h - 1) + d[:, 1] * h
    pw, ph = w * torch.exp(d[:, 2]), h * torch.exp(d[:, 3])
    b = torch.stack([cx - 0.5 * (pw - 1), cy - 0.5 * (ph - 1), cx + 0.5 * (pw - 1), cy + 0.5 * (ph - 1)], 1)
    b[:, 0::2] = b[:, 0::2].clamp(0, im[1] - 1)
    b[:, 1::2] = b[:, 1::2].clamp(0, im[0] - 1)
    return b.contiguous()


def test_nms_cpu_twin_on_proposal_shaped_boxes():
    """The C++ twin (CPU oracle of the GPU tests below) against the tensor greedy loop on the
    heavily overlapping proposal-shaped boxes, with and without truncation."""
    from mx_rcnn_amd.ops.nms import _greedy_loop, _greedy_ref
    g = torch.Generator().manual_seed(3)
    b = rpn_like_boxes(g, 3000)
    for post in (None, 500):
        ref = _greedy_loop(b, 3000, 0.7, post)
        assert _greedy_ref(b, 3000, 0.7, post) == ref
        assert len(ref) < 3000 and (post is None or len(ref) == post)
        assert _greedy_ref(b, 3000, 0.7, post, fp32=True) == _greedy_loop(b, 3000, 0.7, post, fp32=True)


# the RPN-dump shapes of tools/test_rpn.py (pre-NMS = all anchors): VGG 600x1000, 30000, ResNet 800x1333
LARGE_NMS = [(20646, 2000), (20646, 6000), (20646, -1), (30000, 2000), (30000, 6000), (30000, -1), (50400, 2000),
             (50400, 6000), (50400, -1)]


@pytest.mark.gpu
@pytest.mark.parametrize('P,post', LARGE_NMS)
def test_nms_gpu_large_matches_oracles(cuda, P, post):
    """Beyond the helpers' prefetch window, with and without early exit at `post`: the reducer's
    keep list equals the device flag-loop oracle (MXR_NMS_CHECK's kernel) and the CPU greedy
    oracle, on proposal-shaped (heavily overlapping) boxes."""
    from mx_rcnn_amd.ops import need_ext
    C = need_ext()
    g = torch.Generator().manual_seed(P + post)
    b = rpn_like_boxes(g, P)
    s = torch.sort(torch.rand(P, generator=g), descending=True).values
    pst = P if post < 0 else post
    nv = torch.tensor([P], dtype=torch.int32, device=cuda)
    u = torch.rand(1, pst, generator=g).to(cuda)
    bd, sd = b[None].to(cuda), s[None].to(cuda)
    _, _, keep, n_keep = C.nms_proposals(bd, sd, nv, 0.7, pst, u)
    res = C.nms_check(bd, nv, 0.7, pst, keep, n_keep).cpu()
    nk = int(n_keep[0])
    assert int(res[0, 0]) == -1 and int(res[0, 1]) == nk, (res.tolist(), nk)
    from mx_rcnn_amd.ops.nms import _greedy_ref
    # fp32 oracle: the GPU's IoU arithmetic, so only the reducer's logic is under test (the float64
    # twin may split exact-threshold ties differently: clipped proposal boxes make IoU = 0.7 pairs)
    ref = torch.tensor(_greedy_ref(b, P, 0.7, pst, fp32=True), dtype=torch.long)
    got = keep[0, :nk].cpu()
    assert torch.equal(ref, got), nms_mismatch_report(b, ref, got, 0.7, (P, post))


@pytest.mark.gpu
def test_anchor_target_gpu_matches_cpu(cuda):
    H, W = 50, 84
    g = torch.Generator().manual_seed(11)
    gt = torch.full((2, 6, 5), -1.0)
    gt[0, :4, :4] = rand_boxes(g, 4, 700)
    gt[0, :4, 4] = 1
    gt[1, :6, :4] = rand_boxes(g, 6, 700)
    gt[1, :6, 4] = 2
    n_gt = torch.tensor([4, 6], dtype=torch.int32)
    im_info = torch.tensor([[800.0, 1333.0, 1.0], [780.0, 1300.0, 1.0]])
    base = ops.base_anchors(16, (4, 8, 16, 32), (0.5, 1, 2))
    from mx_rcnn_amd.ops.anchor_target import _assign_ref
    lab_c, tgt_c = _assign_ref(H, W, base, 16, im_info, 0, gt, n_gt, 0.3, 0.7, False)
    from mx_rcnn_amd.ops import need_ext
    lab_g, tgt_g, _, _ = need_ext().anchor_target_assign(base.to(cuda), H, W, 16.0, im_info.to(cuda), 0,
                                                         gt.to(cuda), n_gt.to(cuda), 0.3, 0.7, False)
    assert torch.equal(lab_g.cpu(), lab_c)
    m = lab_c >= 0
    assert torch.allclose(tgt_g.cpu()[m], tgt_c[m], atol=1e-4)
    out = ops.anchor_target((H, W), gt.to(cuda), n_gt.to(cuda), im_info.to(cuda), scales=(4, 8, 16, 32))
    L = out['label']
    assert L.shape == (2, 12 * H * W)
    assert torch.all((L == 1).sum(1) <= 128) and torch.all((L >= 0).sum(1) <= 256)


@pytest.mark.gpu
def test_proposal_target_gpu(cuda):
    cfg = snapshot()
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    cfg.TRAIN.BG_THRESH_LO = 0.0
    g = torch.Generator().manual_seed(3)
    P = 6000
    rois = torch.zeros(2, P, 5)
    for b in range(2):
        rois[b, :, 0] = b
        rois[b, :, 1:] = rand_boxes(g, P, 800)
    gt = torch.full((2, 5, 5), -1.0)
    gt[0, :3] = torch.tensor([[20., 30, 120, 140, 5], [150, 40, 300, 200, 2], [400, 400, 600, 500, 9]])
    gt[1, :1] = torch.tensor([[50., 60, 350, 300, 7]])
    out = ops.proposal_target(rois.to(cuda), gt.to(cuda), torch.tensor([3, 1], device=cuda), 21, cfg=cfg)
    lab = out['label'].cpu().reshape(2, 128)
    r = out['rois'].cpu().reshape(2, 128, 5)
    for b in range(2):
        nfg = int((lab[b] > 0).sum())
        assert nfg >= 1 and torch.all(lab[b, nfg:] == 0)
        assert torch.all(r[b, :, 0] == b)
    assert torch.isfinite(out['bbox_target']).all()


@pytest.mark.gpu
def test_proposal_sample_fused_semantics(cuda):
    """Fused HIP proposal-target sampling (csrc/hip/sample.hip): structure, pools, targets and
    weights recomputed independently on the host from the returned RoIs."""
    cfg = snapshot()
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    cfg.TRAIN.BG_THRESH_LO = 0.0
    g = torch.Generator().manual_seed(5)
    P, C = 3000, 21
    rois = torch.zeros(3, P, 5)
    for b in range(3):
        rois[b, :, 0] = b
        rois[b, :, 1:] = rand_boxes(g, P, 700)
    gt = torch.full((3, 4, 5), -1.0)
    gt[0, :3] = torch.tensor([[20., 30, 120, 140, 5], [150, 40, 300, 200, 2], [400, 400, 600, 500, 9]])
    gt[1, :1] = torch.tensor([[50., 60, 350, 300, 7]])
    n_gt = torch.tensor([3, 1, 0])  # image 2: no gt -> no fg, labels all 0
    out = ops.proposal_target(rois.to(cuda), gt.to(cuda), n_gt.to(cuda), C, cfg=cfg)
    lab = out['label'].cpu().reshape(3, 128)
    r = out['rois'].cpu().reshape(3, 128, 5)
    bt = out['bbox_target'].cpu().reshape(3, 128, 4 * C)
    iw = out['bbox_inside_weight'].cpu().reshape(3, 128, 4 * C)
    ow = out['bbox_outside_weight'].cpu().reshape(3, 128, 4 * C)
    means, stds = torch.tensor(cfg.TRAIN.BBOX_MEANS), torch.tensor(cfg.TRAIN.BBOX_STDS)
    for b in range(3):
        ng = int(n_gt[b])
        assert torch.all(r[b, :, 0] == b)
        nfg = int((lab[b] > 0).sum())
        assert torch.all(lab[b, nfg:] == 0) and nfg <= 32
        if ng == 0:
            assert nfg == 0 and torch.all(bt[b] == 0)
            continue
        assert nfg >= 1
        ov = ops.box_iou(r[b, :, 1:], gt[b, :ng, :4])
        mo, am = ov.max(1)
        assert torch.all(mo[:nfg] >= 0.5) and torch.all(mo[32:] < 0.5)  # fg slots / bg slots
        assert torch.equal(lab[b, :nfg].long(), gt[b, am[:nfg], 4].long())
        t = ops.bbox_transform(r[b, :nfg, 1:], gt[b, am[:nfg], :4])
        t = (t - means) / stds
        cols = lab[b, :nfg].long() * 4
        got = torch.stack([bt[b, j, cols[j]:cols[j] + 4] for j in range(nfg)])
        assert torch.allclose(got, t.float(), atol=1e-4, rtol=1e-4)
        assert torch.equal(iw[b].sum(1), (lab[b] > 0).float() * 4)
        assert torch.equal(ow[b], (iw[b] > 0).float())
        assert torch.allclose(bt[b].abs().sum(), got.abs().sum(), rtol=1e-5)  # nothing else is set


@pytest.mark.gpu
@pytest.mark.parametrize('H,W,A,ngt,batch', [(50, 84, 12, 6, 256), (38, 63, 9, 3, 256), (20, 30, 9, 30, 1024),
                                             (12, 16, 9, 2, 1024), (50, 84, 12, 0, 256)])
def test_anchor_target_multi_workgroup_matches_single(cuda, H, W, A, ngt, batch, monkeypatch):
    """The grid-wide histogram / mark selection (MXR_ANCHOR_FUSED=1) picks exactly the anchors of the
    one-workgroup select_smallest path for the same keys: bitwise equal outputs, over seeds, ResNet
    (12 anchors) and VGG (9) maps, all-bg / all-fg pools (RPN batch 1024) and images without gt."""
    from mx_rcnn_amd.config import snapshot
    cfg = snapshot()
    cfg.TRAIN.RPN_BATCH_SIZE = batch
    g = torch.Generator().manual_seed(H * W + ngt)
    gt = torch.full((2, max(ngt, 1), 5), -1.0)
    if ngt:
        xy = torch.rand(2, ngt, 2, generator=g) * torch.tensor([W * 16 - 100, H * 16 - 100])
        wh = torch.rand(2, ngt, 2, generator=g) * 200 + 40
        gt[:, :ngt, :2] = xy
        gt[:, :ngt, 2:4] = xy + wh
        gt[:, :ngt, 4] = 1
    n_gt = torch.tensor([ngt, max(ngt - 1, 0)], dtype=torch.int32)
    im_info = torch.tensor([[H * 16.0, W * 16.0, 1.0], [H * 16.0 - 40, W * 16.0 - 60, 1.0]])
    scales = (4, 8, 16, 32) if A == 12 else (8, 16, 32)
    for seed in range(3):
        outs = []
        for fused in ('1', '0'):
            monkeypatch.setenv('MXR_ANCHOR_FUSED', fused)
            gen = torch.Generator(device=cuda).manual_seed(seed)
            outs.append(ops.anchor_target((H, W), gt.to(cuda), n_gt.to(cuda), im_info.to(cuda), scales=scales,
                                          cfg=cfg, generator=gen))
        for k in ('label', 'bbox_target', 'bbox_inside_weight', 'bbox_outside_weight', 'sample_meta'):
            assert torch.equal(outs[0][k], outs[1][k]), (seed, k)


@pytest.mark.gpu
def test_anchor_sample_fused_counts_and_uniformity(cuda):
    """Fused RPN subsampling: exact counts, labels only from the pre-sampling pools, reference
    weights, and uniform selection frequency over many draws."""
    H, W = 38, 50
    gt = torch.full((1, 4, 5), -1.0)
    gt[0, :4, :4] = torch.tensor([[20., 30, 220, 240], [300, 100, 500, 300], [50, 400, 300, 590], [600, 50, 780, 260]])
    gt[0, :4, 4] = 1
    n_gt = torch.tensor([4], dtype=torch.int32)
    im_info = torch.tensor([[600.0, 800.0, 1.0]])
    base = ops.base_anchors(16, (4, 8, 16, 32), (0.5, 1, 2))
    from mx_rcnn_amd.ops import need_ext
    pre, _, _, _ = need_ext().anchor_target_assign(base.to(cuda), H, W, 16.0, im_info.to(cuda), 0, gt.to(cuda),
                                                    n_gt.to(cuda), 0.3, 0.7, False)
    A = 12
    pre_ahw = pre.cpu().reshape(1, H, W, A).permute(0, 3, 1, 2).reshape(1, -1)
    nfg_pre, nbg_pre = int((pre_ahw == 1).sum()), int((pre_ahw == 0).sum())
    gen = torch.Generator(device=cuda).manual_seed(0)
    hits = torch.zeros(pre_ahw.shape[1])
    trials = 200
    for _ in range(trials):
        out = ops.anchor_target((H, W), gt.to(cuda), n_gt.to(cuda), im_info.to(cuda), scales=(4, 8, 16, 32),
                                generator=gen)
        lab = out['label'].cpu()
        nf, nb = int((lab == 1).sum()), int((lab == 0).sum())
        assert nf == min(nfg_pre, 128) and nb == min(nbg_pre, 256 - nf)
        assert torch.all(pre_ahw[lab == 1] == 1) and torch.all(pre_ahw[lab == 0] == 0)
        ow = out['bbox_outside_weight'].cpu()
        assert torch.allclose(ow.sum(), torch.tensor(4.0), atol=1e-4)  # 4 coords x (1 / num_examples) each
        meta = out['sample_meta'].cpu()  # [all_fg, all_bg, n_fg, n_bg]: the RPN loss normaliser
        assert int(meta[:, 2].sum()) == nf and int(meta[:, 3].sum()) == nb
        hits += (lab == 0).float()[0]
    # every bg-pool anchor is picked with probability nb / nbg_pre: mean hit rate over the pool
    bg_pool = (pre_ahw[0] == 0)
    rate = hits[bg_pool] / trials
    expect = min(nbg_pre, 256 - min(nfg_pre, 128)) / nbg_pre
    assert abs(rate.mean().item() - expect) < 0.1 * expect
    # no anchor is systematically favoured (first vs second half of the pool by index)
    idx = torch.nonzero(bg_pool).flatten()
    h1, h2 = rate[: len(idx) // 2].mean().item(), rate[len(idx) // 2:].mean().item()
    assert abs(h1 - h2) < 0.15 * expect


@pytest.mark.gpu
@pytest.mark.parametrize('P,post,nv_frac', [(6000, 300, 1.0), (6000, 300, 0.7), (12000, 6000, 1.0), (3000, 2000, 0.5)])
def test_nms_proposals_graph_replay(cuda, P, post, nv_frac):
    """The proposal NMS captured in a hipGraph (as in GraphedStep / bench_test's GraphedDetect)
    and replayed on new inputs gives the eager result (workspace zeroing is a captured memset)."""
    from mx_rcnn_amd.ops import need_ext
    C = need_ext()
    g = torch.Generator().manual_seed(17)

    def inputs():
        b = rand_boxes(g, P, 1300)
        s = torch.sort(torch.rand(P, generator=g), descending=True).values
        nv = torch.tensor([int(P * nv_frac)], dtype=torch.int32)
        u = torch.rand(1, post, generator=g)
        return b[None].to(cuda), s[None].to(cuda).contiguous(), nv.to(cuda), u.to(cuda)

    sb, ss, snv, su = inputs()
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        C.nms_proposals(sb, ss, snv, 0.7, post, su)
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = C.nms_proposals(sb, ss, snv, 0.7, post, su)
    for _ in range(3):
        b, s, nv, u = inputs()
        sb.copy_(b), ss.copy_(s), snv.copy_(nv), su.copy_(u)
        graph.replay()
        torch.cuda.synchronize()
        ref = C.nms_proposals(b, s, nv, 0.7, post, u)
        for a, r in zip(out, ref):
            assert torch.equal(a, r)


def test_nms_cpu_twin_matches_tensor_loop():
    """The C++ CPU twin of the greedy NMS (the CPU configuration's fast path) keeps exactly what
    the tensor-loop oracle keeps, including duplicate boxes and the max_keep cap."""
    from mx_rcnn_amd.ops import ext_available, need_ext
    from mx_rcnn_amd.ops.nms import _greedy_loop
    if not ext_available():
        pytest.skip('extension not built')
    g = torch.Generator().manual_seed(21)
    for n, th, cap in [(1, 0.5, None), (200, 0.7, None), (1500, 0.5, 100), (3000, 0.3, None), (700, 0.0, None)]:
        b = rand_boxes(g, n, 600)
        if n > 10:
            b[5:10] = b[0]  # exact duplicates
        ref = _greedy_loop(b, n, th, cap)
        got = need_ext().nms_cpu(b, n, th, -1 if cap is None else cap).tolist()
        assert got == ref, (n, th, cap)


@pytest.mark.parametrize('crop,is_prob', [(True, False), (False, False), (True, True)])
def test_proposal_decode_cpu_twin_matches_tensor_ref(crop, is_prob):
    """C++ twin (host_ops.h proposal_decode_image) vs the tensor decode: same filter mask,
    boxes within an ulp of the box magnitude, scores within an ulp."""
    from mx_rcnn_amd.ops import ext_available, need_ext
    from mx_rcnn_amd.ops.anchors import base_anchors
    from mx_rcnn_amd.ops.proposal import _decode_ref
    if not ext_available():
        pytest.skip('extension not built')
    cls, dlt = _rpn_inputs(8, 9, 30, 40, B=2)
    if is_prob:
        cls = torch.rand(cls.shape, generator=torch.Generator().manual_seed(2))
    im = torch.tensor([[470., 630., 1.0], [400., 600., 1.5]])
    base = base_anchors(16, (8, 16, 32), (0.5, 1, 2), torch.device('cpu'))
    b1, k1 = _decode_ref(cls, dlt, im, base, 16, 16, crop, is_prob)
    b2, k2 = need_ext().proposal_decode_cpu(cls, dlt, im, base, 16., 16., crop, is_prob)
    fin = torch.isfinite(k1)
    assert torch.equal(fin, torch.isfinite(k2))
    assert torch.allclose(b1, b2, rtol=0, atol=2e-4)
    assert torch.allclose(k1[fin], k2[fin], rtol=0, atol=1e-6)


@pytest.mark.parametrize('clobber,border', [(False, 0), (True, 0), (False, 10)])
def test_anchor_assign_cpu_twin_matches_tensor_ref(clobber, border):
    """C++ twin (host_ops.h anchor_gt_max / anchor_assign_range) vs the tensor assignment:
    identical labels (incl. gt-best ties and an image without gt) and targets."""
    from mx_rcnn_amd.ops import ext_available, need_ext
    from mx_rcnn_amd.ops.anchor_target import _assign_ref
    from mx_rcnn_amd.ops.anchors import base_anchors
    if not ext_available():
        pytest.skip('extension not built')
    g = torch.Generator().manual_seed(3)
    base = base_anchors(16, (8, 16, 32), (0.5, 1, 2), torch.device('cpu'))
    H, W = 38, 50
    gt = torch.zeros(3, 6, 5)
    for b in range(3):
        xy = torch.rand(6, 2, generator=g) * torch.tensor([700., 500.])
        gt[b, :, :2] = xy
        gt[b, :, 2:4] = xy + torch.rand(6, 2, generator=g) * 200 + 10
    n_gt = torch.tensor([6, 2, 0], dtype=torch.int32)
    im = torch.tensor([[600., 800., 1.], [580., 790., 1.], [600., 800., 1.]])
    l1, t1 = _assign_ref(H, W, base, 16, im, border, gt, n_gt, 0.3, 0.7, clobber)
    l2, t2 = need_ext().anchor_assign_cpu(base, H, W, 16., im, border, gt, n_gt, 0.3, 0.7, clobber)
    assert torch.equal(l1, l2) and torch.allclose(t1, t2, atol=1e-6)
    assert (l2 == 1).any() and (l2[2] != 1).all()


def test_iou_max_cpu_twin_matches_tensor_ref():
    """C++ twin (host_ops.h iou_max_rows) vs the dense tensor version: exact max, first argmax
    on ties, image without gt -> 0 / 0, per-gt column max."""
    from mx_rcnn_amd.ops import ext_available, need_ext
    from mx_rcnn_amd.ops.boxes import iou_max_ref
    if not ext_available():
        pytest.skip('extension not built')
    g = torch.Generator().manual_seed(5)
    B, N, G = 3, 700, 7
    xy = torch.rand(B, N, 2, generator=g) * 600
    r = torch.cat([torch.zeros(B, N, 1), xy, xy + torch.rand(B, N, 2, generator=g) * 150], -1)
    gxy = torch.rand(B, G, 2, generator=g) * 600
    gt = torch.cat([gxy, gxy + torch.rand(B, G, 2, generator=g) * 150 + 5, torch.ones(B, G, 1)], -1)
    gt[0, 4, :4] = gt[0, 2, :4]  # duplicate gt: argmax must take the first
    r[0, 5, 1:] = gt[0, 2, :4]
    n_gt = torch.tensor([7, 3, 0], dtype=torch.int32)
    for want in (False, True):
        a = iou_max_ref(r, gt, n_gt, off=1, want_gt_max=want)
        b = need_ext().iou_max_cpu(r, 1, gt, n_gt, want)
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    assert int(b[1][0, 5]) == 2 and float(b[0][0, 5]) == 1.0


def _det_case(B, R, C, seed):
    g = torch.Generator().manual_seed(seed)
    H, W = 600.0, 900.0
    x1 = torch.rand(B * R, generator=g) * (W - 200)
    y1 = torch.rand(B * R, generator=g) * (H - 200)
    wh = torch.rand(B * R, 2, generator=g) * 180 + 10
    rois = torch.stack([torch.arange(B).repeat_interleave(R).float(), x1, y1, x1 + wh[:, 0], y1 + wh[:, 1]], 1)
    logits = torch.randn(B * R, C, generator=g) * 2
    logits[:, 1:6] += 3.0  # a few confident classes
    scores = torch.softmax(logits, 1)
    deltas = torch.randn(B * R, 4 * C, generator=g) * 0.1
    info = torch.tensor([[H, W, 1.5]] * B)
    return rois, scores, deltas, info


@pytest.mark.gpu
@pytest.mark.parametrize('B,R,C,maxper', [(1, 300, 81, 100), (8, 300, 81, 100), (2, 1000, 21, 100), (3, 64, 5, 0)])
def test_device_postprocess_matches_reference(cuda, B, R, C, maxper):
    """Fused test-time post-process (decode, clip, threshold, per-class NMS, image top-k with the
    reference's >= tie rule) vs the tensor reference, as per-image sets."""
    from mx_rcnn_amd.core.detector import Detector
    rois, scores, deltas, info = _det_case(B, R, C, 17 + B)
    det = Detector.__new__(Detector)
    ref = det.postprocess_ref(rois, scores, deltas, info, 0.3, 0.05, maxper)
    dets, counts = det.postprocess_raw(rois.to(cuda), scores.to(cuda), deltas.to(cuda), info.to(cuda), 0.3, 0.05,
                                       maxper, cap=4096)
    dets, counts = dets.cpu(), counts.cpu()
    for b in range(B):
        rb, rs, rc = ref[b]
        n = int(counts[b])
        assert n == rs.numel(), (b, n, rs.numel())
        if maxper:
            assert n >= min(maxper, n)
        got = dets[b, :n]
        key_ref = torch.stack([rc.float(), -rs], 1)
        key_got = torch.stack([got[:, 5], -got[:, 4]], 1)
        oref = sorted(range(n), key=lambda i: tuple(key_ref[i].tolist()))
        ogot = sorted(range(n), key=lambda i: tuple(key_got[i].tolist()))
        assert torch.allclose(got[ogot, 4], rs[oref], atol=1e-6)
        assert torch.equal(got[ogot, 5].long(), rc[oref])
        assert torch.allclose(got[ogot, :4], rb[oref].float(), atol=1e-3, rtol=1e-5)


@pytest.mark.gpu
def test_nest_kernel_matches_reference(cuda):
    from mx_rcnn_amd.processing.nms import nest
    rng = np.random.RandomState(4)
    x1 = rng.rand(700) * 500
    y1 = rng.rand(700) * 500
    w, h = rng.rand(700) * 120 + 4, rng.rand(700) * 120 + 4
    dets = np.stack([x1, y1, x1 + w, y1 + h, rng.rand(700)], 1).astype(np.float32)
    dets[5] = dets[6]  # identical boxes are each nested in the other: both dropped
    assert nest(torch.as_tensor(dets, device=cuda), 0.8) == nest(dets, 0.8)


@pytest.mark.gpu
@pytest.mark.parametrize('B,N,P,ties', [(1, 50400, 12000, False), (2, 50400, 6000, True), (3, 1000, 1000, True),
                                        (1, 7000, 6000, False), (8, 50400, 6000, False), (8, 50400, 12000, True),
                                        (2, 50401, 50401, False),
                                        # chunk-sort / merge-rank boundaries (1024-candidate chunks, the
                                        # 20480-candidate LDS limit, and the counting fallback above it)
                                        (1, 5000, 1024, True), (1, 5000, 1025, False), (1, 30000, 20480, True),
                                        (1, 30000, 20481, False)])
def test_proposal_topk_matches_stable_sort(cuda, B, N, P, ties):
    """Radix-select + rank-by-counting top-P == stable descending sort truncated to P (keys, boxes,
    valid count), with heavy ties and -inf (filtered) entries."""
    from mx_rcnn_amd.ops import need_ext
    g = torch.Generator().manual_seed(N + P)
    keys = torch.rand(B, N, generator=g)
    if ties:
        keys = (keys * 64).floor() / 64  # 64 distinct values
    keys[torch.rand(B, N, generator=g) < 0.3] = float('-inf')
    boxes = torch.rand(B, N, 4, generator=g) * 500
    sk, sb, nv = need_ext().proposal_topk(keys.to(cuda), boxes.to(cuda), P)
    rk, order = torch.sort(keys, dim=1, descending=True, stable=True)
    rk, order = rk[:, :P], order[:, :P]
    rb = torch.gather(boxes, 1, order[..., None].expand(-1, -1, 4))
    assert torch.equal(sk.cpu(), rk)
    assert torch.equal(sb.cpu(), rb)
    assert torch.equal(nv.cpu(), (rk > float('-inf')).sum(1).to(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize('P', [6000, 12000])
def test_proposal_topk_graph_replay(cuda, P):
    """The grid radix top-k captured in a hipGraph (its zeroed workspace is a captured fill) and
    replayed on new RPN-like scores (softmax foreground probabilities: most near 0, clustered top
    bytes, ties) for B = 8, N = 50 400: every replay == the stable sort."""
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    B, N = 8, 50400
    g = torch.Generator().manual_seed(P)
    keys = torch.empty(B, N, device=cuda)
    boxes = (torch.rand(B, N, 4, generator=g) * 800).to(cuda)

    def fill(seed):
        gg = torch.Generator().manual_seed(seed)
        logit = torch.randn(B, N, 2, generator=gg) * 3
        k = torch.softmax(logit, 2)[..., 1]
        k = (k * 4096).round() / 4096  # ties
        k[torch.rand(B, N, generator=gg) < 0.1] = float('-inf')
        keys.copy_(k)
        return k

    fill(0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            ext.proposal_topk(keys, boxes, P)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        sk, sb, nv = ext.proposal_topk(keys, boxes, P)
    for seed in (1, 2, 3):
        k = fill(seed)
        graph.replay()
        torch.cuda.synchronize()
        rk, order = torch.sort(k, dim=1, descending=True, stable=True)
        rk, order = rk[:, :P], order[:, :P]
        rb = torch.gather(boxes.cpu(), 1, order[..., None].expand(-1, -1, 4))
        assert torch.equal(sk.cpu(), rk)
        assert torch.equal(sb.cpu(), rb)
        assert torch.equal(nv.cpu(), (rk > float('-inf')).sum(1).to(torch.int32))


@pytest.mark.gpu
def test_proposal_gather_matches_torch(cuda):
    """Post-sort top-P assembly kernel == slice + gather + valid count."""
    from mx_rcnn_amd.ops import need_ext
    g = torch.Generator().manual_seed(7)
    B, N, P = 2, 5000, 3000
    keys = torch.rand(B, N, generator=g)
    keys[0, torch.randperm(N, generator=g)[:2500]] = float('-inf')  # image 0: 2500 valid
    keys[1, torch.randperm(N, generator=g)[:200]] = float('-inf')   # image 1: all P valid
    boxes = torch.rand(B, N, 4, generator=g) * 500
    keys, boxes = keys.to(cuda), boxes.to(cuda)
    sk, order = torch.sort(keys, dim=1, descending=True, stable=True)
    ok, ob, nv = need_ext().proposal_gather(sk, order, boxes, P)
    torch.testing.assert_close(ok, sk[:, :P])
    ref_b = torch.gather(boxes, 1, order[:, :P, None].expand(-1, -1, 4))
    torch.testing.assert_close(ob, ref_b)
    assert nv.tolist() == [2500, P]
