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


@pytest.mark.gpu
@pytest.mark.parametrize('P', [0, 3])
def test_roi_pool_backward_gpu_bitwise(cuda, P):
    """The RoI-pool backward sums every bin's dY into its pixel in 64-bit fixed point (per-channel
    power-of-two scale): any arrival order gives the same bits, and the single rounding at the end
    keeps the fp32-class result within fp32 rounding of the fp64 scatter.  300 heavily overlapping
    RoIs (many bins per pixel), fp32 (P = 0) and fp32 triples (P = 3) with the RPN-side gradient
    added."""
    from mx_rcnn_amd.ops import need_ext, precision
    ext = need_ext()
    g = torch.Generator().manual_seed(8)
    B, C, H, W, R = 2, 256, 38, 50, 300
    feat = torch.randn(B, C, H, W, generator=g)
    rois = _rois(g, R, B, H, W)
    gout = torch.randn(R, C, 7, 7, generator=g) * torch.logspace(-3, 3, C)[None, :, None, None]
    gadd = torch.randn(B, C, H, W, generator=g)

    def enc(t):
        t = t.to(cuda).contiguous(memory_format=torch.channels_last)
        return precision.split(t, P).contiguous(memory_format=torch.channels_last) if P else t

    _, arg = ext.roi_pool_fwd(enc(feat), rois.to(cuda), 7, 7, 1 / 16, P)
    outs = [ext.roi_pool_bwd(enc(gout), arg, rois.to(cuda), B, H, W, enc(gadd), P) for _ in range(3)]
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    got = (precision.join(outs[0], P) if P else outs[0]).double().cpu().reshape(B, C, -1)
    ref = gadd.double().reshape(B, C, -1).clone()
    a = arg.cpu().reshape(R, C, -1).long()
    go = gout.double().reshape(R, C, -1)
    for r in range(R):
        b = int(rois[r, 0])
        m = a[r] >= 0
        ref[b].view(-1).index_add_(0, (torch.arange(C)[:, None] * H * W + a[r].clamp_min(0))[m], go[r][m])
    # per-channel relative error (the channels span six decades)
    err = ((got - ref).abs().amax(2) / ref.abs().amax(2).clamp_min(1e-30)).max()
    assert float(err) <= 2e-6, float(err)


@pytest.mark.gpu
def test_bn_relu_backward_gpu_bitwise(cuda):
    """BN-ReLU backward (frozen statistics) column sums: thread-ordered in-block reduce + fixed-order
    fold, bitwise across runs, and close to fp64."""
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(9)
    N, C, H, W = 2, 64, 40, 56
    x = torch.randn(N, C, H, W, generator=g)
    dy = torch.randn(N, C, H, W, generator=g)
    gam, bet, mu, var = torch.rand(C) + 0.5, torch.randn(C) * 0.1, torch.randn(C) * 0.1, torch.rand(C) + 0.5
    p = [t.to(cuda) for t in (gam, bet, mu, var)]
    xe = x.to(cuda).contiguous(memory_format=torch.channels_last)
    de = dy.to(cuda).contiguous(memory_format=torch.channels_last)
    runs = [ext.bn_relu_bwd(xe, de, *p, 2e-5, False, True, True, True, None, None, None, 0) for _ in range(3)]
    torch.cuda.synchronize()
    for r in runs[1:]:
        for u, v in zip(r, runs[0]):
            assert torch.equal(u, v)
    s = gam.double() / torch.sqrt(var.double() + 2e-5)
    pre = (x.double() - mu.double().view(1, -1, 1, 1)) * s.view(1, -1, 1, 1) + bet.double().view(1, -1, 1, 1)
    gm = dy.double() * (pre > 0)
    xhat = (x.double() - mu.double().view(1, -1, 1, 1)) / torch.sqrt(var.double() + 2e-5).view(1, -1, 1, 1)
    dg = (gm * xhat).sum((0, 2, 3))
    db = gm.sum((0, 2, 3))
    assert float((runs[0][1].double().cpu() - dg).abs().max() / dg.abs().max()) <= 1e-5
    assert float((runs[0][2].double().cpu() - db).abs().max() / db.abs().max()) <= 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize('P', [0, 3])
def test_frozen_bn_column_sums_partial_rows(cuda, P):
    """Frozen-BN backward epilogue of a dgrad conv: the deterministic partial rows (bnb_part) +
    fixed-order fold give the fp32-atomic path's dgamma / dbeta (to rounding) and the same dx bit
    for bit, and repeat bitwise."""
    from mx_rcnn_amd.ops import need_ext, precision
    ext = need_ext()
    g = torch.Generator().manual_seed(10 + P)
    C, H, W, O = 256, 25, 42, 256
    dy = torch.randn(1, O, H, W, generator=g)
    w = torch.randn(C, O, 3, 3, generator=g) * 0.03
    xbn = torch.randn(1, C, H, W, generator=g)
    bn = [t.to(cuda) for t in (torch.rand(C) + 0.5, torch.randn(C) * 0.1, torch.randn(C) * 0.1, torch.rand(C) + 0.5)]

    def enc(t):
        t = t.to(cuda).contiguous(memory_format=torch.channels_last)
        return (precision.split(t, P) if P else t.bfloat16()).contiguous(memory_format=torch.channels_last)

    we = enc(w)
    kw = {'x2': P, 'w_plane': we.numel() // P} if P else {}
    wv = we[:C] if P else we
    dge, xe = enc(dy), enc(xbn)
    tg, tb = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
    ra = ext.conv_igemm_fwd(dge, wv, None, 1, 1, False, 23, 1, None, bn, 2e-5, False, True, xe, None, tg, tb, **kw)[0]
    nparts = (H * W + 63) // 64
    outs = []
    for _ in range(2):
        part = torch.empty(nparts * 2 * C, device=cuda)
        dg, db = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
        # tile 23 like the atomic reference (the autotuned choice may sum K in another order)
        r = ext.conv_igemm_fwd(dge, wv, None, 1, 1, False, 23, 1, None, bn, 2e-5, False, True, xe, None, None, None,
                               bnb_part=part, **kw)[0]
        ext.bnb_part_fold(part, nparts, C, dg, db)
        outs.append((r, dg, db))
    torch.cuda.synchronize()
    for u, v in zip(outs[0], outs[1]):
        assert torch.equal(u, v)
    assert torch.equal(outs[0][0], ra)
    assert torch.allclose(outs[0][1], tg, rtol=1e-5, atol=1e-5 * float(tg.abs().max()))
    assert torch.allclose(outs[0][2], tb, rtol=1e-5, atol=1e-5 * float(tb.abs().max()))


@pytest.mark.gpu
def test_bnb_part_fold_multi_matches_single_folds(cuda):
    """The batched fold (one launch for many BNs, up to 32 per launch) == one fold per BN, bitwise,
    with some entries folding only dbeta (fix_gamma) and more entries than one launch holds."""
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(12)
    ents, ref = [], []
    for i in range(37):
        C = [64, 256, 1024, 512][i % 4]
        nparts = 1 + (i * 7) % 70
        part = torch.randn(nparts * 2 * C, generator=g).to(cuda)
        base_g, base_b = torch.randn(C, generator=g).to(cuda), torch.randn(C, generator=g).to(cuda)
        dg, db = base_g.clone(), base_b.clone()
        ext.bnb_part_fold(part, nparts, C, None if i % 5 == 0 else dg, db)
        ref.append((dg, db))
        mg, mb = base_g.clone(), base_b.clone()
        ents.append((part, nparts, C, None if i % 5 == 0 else mg, mb))
    ext.bnb_part_fold_multi(ents)
    torch.cuda.synchronize()
    for (p, n, C, mg, mb), (dg, db) in zip(ents, ref):
        assert torch.equal(mb, db)
        if mg is not None:
            assert torch.equal(mg, dg)


def _anchor_layouts_with_one_total_size(cuda, cfg):
    """(G = 8, 38x50 map) and (G = 16, 36x52 map) need the same anchor workspace size
    (8 + ceil(9*1900/32) == 16 + ceil(9*1872/32)) but put the histogram / mark regions at different
    offsets: alternating them must reproduce each one's first result (the workspace was
    keyed by total size only, so the second layout's histograms met the first one's mark words)."""
    from mx_rcnn_amd import ops
    runs = {}
    for rep in range(5):
        G, (H, W) = (16, (36, 52)) if rep % 2 == 0 else (8, (38, 50))
        g = torch.Generator().manual_seed(G)
        gt = torch.full((1, G, 5), -1.0)
        xy = torch.rand(1, 6, 2, generator=g) * torch.tensor([W * 16 - 220, H * 16 - 220])
        gt[:, :6, :2] = xy
        gt[:, :6, 2:4] = xy + 60 + 150 * torch.rand(1, 6, 2, generator=g)
        gt[:, :6, 4] = 1
        im_info = torch.tensor([[H * 16.0, W * 16.0, 1.0]], device=cuda)
        torch.manual_seed(91)
        o = ops.anchor_target((H, W), gt.to(cuda), torch.tensor([6], dtype=torch.int32, device=cuda), im_info,
                              scales=(4, 8, 16, 32), cfg=cfg)
        runs.setdefault(('out', G), o)
        for k in ('label', 'bbox_target', 'sample_meta'):
            assert torch.equal(o[k], runs[('out', G)][k]), (rep, G, k)


@pytest.mark.gpu
def test_self_cleaning_workspaces_repeat(cuda):
    """The anchor-sampling and proposal top-k workspaces persist across calls and are left zeroed by
    their own kernel chains (bindings.cpp clean_ws): back-to-back calls with the same draws give the
    same result five times over, and a different gt count (another workspace) in between changes
    nothing."""
    from mx_rcnn_amd.config import snapshot
    cfg = snapshot()
    H, W = 38, 50
    g = torch.Generator().manual_seed(3)
    gt = torch.full((2, 8, 5), -1.0)
    xy = torch.rand(2, 5, 2, generator=g) * torch.tensor([W * 16 - 100, H * 16 - 100])
    gt[:, :5, :2] = xy
    gt[:, :5, 2:4] = xy + 60 + torch.rand(2, 5, 2, generator=g) * 150
    gt[:, :5, 4] = 1
    n_gt = torch.tensor([5, 3], dtype=torch.int32, device=cuda)
    im_info = torch.tensor([[H * 16.0, W * 16.0, 1.0]] * 2, device=cuda)
    outs = []
    for rep in range(5):
        if rep == 2:  # another workspace size in between
            ops.anchor_target((H, W), gt[:, :4].to(cuda), n_gt.clamp(max=4), im_info, scales=(4, 8, 16, 32), cfg=cfg)
        torch.manual_seed(77)
        outs.append(ops.anchor_target((H, W), gt.to(cuda), n_gt, im_info, scales=(4, 8, 16, 32), cfg=cfg))
    for o in outs[1:]:
        for k in ('label', 'bbox_target', 'bbox_inside_weight', 'sample_meta'):
            assert torch.equal(o[k], outs[0][k]), k
    _anchor_layouts_with_one_total_size(cuda, cfg)
    cls, dlt = _rpn_inputs(4, 9, H, W, B=2)
    cl = cls.to(cuda).contiguous(memory_format=torch.channels_last)
    dl = dlt.to(cuda).contiguous(memory_format=torch.channels_last)
    res = [_twice(lambda: ops.proposal(cl, dl, im_info, is_train=True, **KW)) for _ in range(3)]
    for (r1, s1), (r2, s2) in res:
        assert torch.equal(r1, res[0][0][0]) and torch.equal(r2, res[0][0][0]) and torch.equal(s1, res[0][0][1])
