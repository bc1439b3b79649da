"""Fused conv epilogues (conv + frozen BN + ReLU + residual), the BN backward with fused
residual gradient, the one-launch dgrad filter cache, and fused-vs-unfused ResNet units.
Oracles: plain PyTorch fp32 ops on the same bf16 inputs (tests/test_kernels.py convention)."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _cl(t, dev):
    return t.to(dev).contiguous(memory_format=torch.channels_last)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _bn_ref(y, gamma, beta, mean, var, eps=2e-5):
    s = gamma * torch.rsqrt(var + eps)
    return y * s[None, :, None, None] + (beta - mean * s)[None, :, None, None]


@pytest.mark.parametrize('shape', [(1, 256, 24, 40, 256, 1, 1, 0), (1, 64, 31, 17, 64, 3, 1, 1),
                                   (2, 128, 14, 14, 512, 1, 1, 0), (1, 1024, 50, 84, 256, 1, 1, 0)])
@pytest.mark.parametrize('tile,splits', [(3, 1), (3, 4), (0, 0), (23, 1), (22, 2), (101, 1), (105, 1), (106, 1),
                                         (109, 1), (110, 1), (106, 2)])
def test_conv_epilogue_residual_bn(cuda, shape, tile, splits):
    from mx_rcnn_amd.ops import need_ext
    N, Cin, H, W, Cout, k, s, p = shape
    g = torch.Generator().manual_seed(21)
    x = torch.randn(N, Cin, H, W, generator=g).bfloat16()
    w = (torch.randn(Cout, Cin, k, k, generator=g) * 0.05).bfloat16()
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    res = torch.randn(N, Cout, Ho, Wo, generator=g).bfloat16()
    gamma, beta = torch.rand(Cout, generator=g) + 0.5, torch.randn(Cout, generator=g) * 0.1
    mean, var = torch.randn(Cout, generator=g) * 0.2, torch.rand(Cout, generator=g) + 0.5
    y, a = need_ext().conv_igemm_fwd(_cl(x, cuda), _cl(w, cuda), None, s, p, False, tile, splits, _cl(res, cuda),
                                     [t.to(cuda) for t in (gamma, beta, mean, var)], 2e-5, False, True)
    ref_y = F.conv2d(x.float(), w.float(), stride=s, padding=p) + res.float()
    ref_a = torch.relu(_bn_ref(ref_y, gamma, beta, mean, var))
    for out, ref in ((y, ref_y), (a, ref_a)):
        err = (out.float().cpu() - ref).abs().max().item()
        assert err <= 1.5e-2 * ref.abs().max().item() + 1e-2, err
    # y2 is computed from the STORED bf16 y: exactly the unfused BN of y
    a2 = need_ext().bn_relu_fwd(y, gamma.to(cuda), beta.to(cuda), mean.to(cuda), var.to(cuda), 2e-5, False, True)
    assert (a2.float() - a.float()).abs().max().item() <= 1e-2


def test_bn_relu_bwd_dres(cuda):
    from mx_rcnn_amd.ops import need_ext
    g = torch.Generator().manual_seed(22)
    C = 256
    x = torch.randn(1, C, 20, 30, generator=g).bfloat16()
    dy = torch.randn(1, C, 20, 30, generator=g).bfloat16()
    dres = torch.randn(1, C, 20, 30, generator=g).bfloat16()
    gamma, beta = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.1
    mean, var = torch.randn(C, generator=g) * 0.2, torch.rand(C, generator=g) + 0.5
    args = [t.to(cuda) for t in (gamma, beta, mean, var)]
    dx0, dg0, db0 = need_ext().bn_relu_bwd(_cl(x, cuda), _cl(dy, cuda), *args, 2e-5, False, True, True, True)
    dx1, dg1, db1 = need_ext().bn_relu_bwd(_cl(x, cuda), _cl(dy, cuda), *args, 2e-5, False, True, True, True,
                                           None, None, _cl(dres, cuda))
    ref = dx0.float() + dres.to(cuda).float()
    assert (dx1.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    assert torch.allclose(dg0, dg1, rtol=1e-4, atol=1e-3) and torch.allclose(db0, db1, rtol=1e-4, atol=1e-3)


def test_wt_flip_cache(cuda):
    from mx_rcnn_amd.ops import need_ext
    from mx_rcnn_amd.ops.conv import _flip_t
    g = torch.Generator().manual_seed(23)
    shapes = [(256, 64, 3, 3), (64, 256, 1, 1), (1024, 256, 1, 1), (512, 512, 3, 3), (72, 136, 3, 3)]
    srcs = [_cl(torch.randn(*s, generator=g).bfloat16(), cuda) for s in shapes]
    dsts = [torch.empty((s[1], s[0], s[2], s[3]), dtype=torch.bfloat16, device=cuda,
                        memory_format=torch.channels_last) for s in shapes]
    ext = need_ext()
    n, tiles = ext.wt_flip_table_info(srcs)
    table = ext.wt_flip_build(srcs, dsts)
    ext.wt_flip_run(table, n, tiles)
    for s_, d_ in zip(srcs, dsts):
        assert torch.equal(d_, _flip_t(s_))


def _unit(cin, cout, stride, dim_match, dev, bottle=True):
    from mx_rcnn_amd.models.resnet import ResidualUnit
    torch.manual_seed(5)
    u = ResidualUnit('u', cin, cout, stride, dim_match, bottle, 0.99, True)
    with torch.no_grad():
        for m in u.modules():
            if hasattr(m, 'moving_var'):
                m.moving_mean.normal_(0, 0.2)
                m.moving_var.uniform_(0.5, 1.5)
                m.gamma.uniform_(0.5, 1.5)
                m.beta.normal_(0, 0.1)
            elif hasattr(m, 'weight') and m.weight is not None:
                m.weight.normal_(0, 0.05)
    u = u.to(dev)
    for m in u.modules():
        if hasattr(m, 'weight') and m.weight is not None and m.weight.dim() == 4:
            m.weight = torch.nn.Parameter(m.weight.detach().bfloat16().contiguous(memory_format=torch.channels_last))
    return u


@pytest.mark.parametrize('cfg', [(1024, 1024, 1, True, True), (512, 1024, 2, False, True),
                                 (256, 256, 1, True, True), (256, 512, 1, False, True),
                                 (128, 128, 1, True, False), (128, 256, 2, False, False)])
@pytest.mark.parametrize('unit_op', ['1', '0'])
def test_fused_units_match_unfused(cuda, cfg, unit_op, monkeypatch):
    """Two chained units (u -> v, v's bn1 fused into u's last epilogue) vs the plain modules."""
    monkeypatch.setenv('MXR_FUSE_UNIT', unit_op)
    cin, cout, stride, dim_match, bottle = cfg
    H, W = (24, 40) if stride == 1 else (48, 80)
    u = _unit(cin, cout, stride, dim_match, cuda, bottle)
    v = _unit(cout, cout, 1, True, cuda, bottle)
    g = torch.Generator().manual_seed(6)
    x0 = torch.randn(1, cin, H, W, generator=g).bfloat16()
    results = []
    for fused in (False, True):
        x = _cl(x0, cuda).requires_grad_()
        if fused:
            assert u.can_fuse(x)
            out_u, act = u.forward_fused(x, None, v.bn1)
            out, _ = v.forward_fused(out_u, act, None)
        else:
            out = v(u(x))
        gen = torch.Generator().manual_seed(7)
        d_out = torch.randn(out.shape, generator=gen).bfloat16().to(cuda)
        for p_ in list(u.parameters()) + list(v.parameters()):
            p_.grad = None
        out.backward(d_out)
        grads = {}
        for tag, mod in (('u', u), ('v', v)):
            for n, p_ in mod.named_parameters():
                if p_.grad is not None:
                    grads[tag + '.' + n] = p_.grad.detach().float().clone()
        results.append((out.detach().float(), x.grad.detach().float(), grads))
    (o0, x0g, g0), (o1, x1g, g1) = results
    # bf16 activations: ReLU masks flip where the two paths round a pre-activation differently
    # (fused adds the residual in fp32 before rounding), so gradients are compared in relative
    # L2 with a bound of the same size as either path's distance to an fp32 oracle (~5%,
    # the fused-vs-unfused comparison); outputs must agree to bf16 rounding.
    assert _rel(o1, o0) <= 1e-2
    assert _rel(x1g, x0g) <= 0.1
    assert set(g0) == set(g1), set(g0) ^ set(g1)
    for n in g0:
        assert _rel(g1[n], g0[n]) <= 0.1, (n, _rel(g1[n], g0[n]))


def test_bnb_epilogue_vs_reference(cuda):
    """dgrad conv with the BN-ReLU backward epilogue (+dadd, +dres) vs unfused torch ops."""
    from mx_rcnn_amd.ops import need_ext
    from mx_rcnn_amd.ops.conv import _flip_t
    g = torch.Generator().manual_seed(41)
    for (Cin, Cout, k, H, W, splits, tile) in ((256, 1024, 1, 24, 40, 1, 0), (256, 1024, 1, 24, 40, 4, 0),
                                               (256, 256, 3, 20, 30, 1, 0), (256, 256, 3, 20, 30, 2, 0),
                                               (256, 1024, 1, 24, 40, 1, 105), (256, 256, 3, 20, 30, 1, 106),
                                               (256, 256, 3, 20, 30, 1, 109), (256, 1024, 1, 24, 40, 2, 106)):
        w = (torch.randn(Cout, Cin, k, k, generator=g) * 0.05).bfloat16()
        dy = torch.randn(1, Cout, H, W, generator=g).bfloat16()
        xr = torch.randn(1, Cin, H, W, generator=g).bfloat16()
        dadd = torch.randn(1, Cin, H, W, generator=g).bfloat16()
        dres = torch.randn(1, Cin, H, W, generator=g).bfloat16()
        gamma, beta = torch.rand(Cin, generator=g) + 0.5, torch.randn(Cin, generator=g) * 0.1
        mean, var = torch.randn(Cin, generator=g) * 0.2, torch.rand(Cin, generator=g) + 0.5
        p = k // 2
        # reference
        d_act = torch.ops.aten.convolution_backward(dy.float(), xr.float(), w.float(), None, [1, 1], [p, p], [1, 1],
                                                    False, [0, 0], 1, [True, False, False])[0] + dadd.float()
        s = gamma * torch.rsqrt(var + 2e-5)
        pre = xr.float() * s[None, :, None, None] + (beta - mean * s)[None, :, None, None]
        gm = d_act * (pre > 0).float()
        ref_dx = gm * s[None, :, None, None] + dres.float()
        xhat = (xr.float() - mean[None, :, None, None]) * torch.rsqrt(var + 2e-5)[None, :, None, None]
        ref_dg, ref_db = (gm * xhat).sum(dim=(0, 2, 3)), gm.sum(dim=(0, 2, 3))
        wt = _flip_t(_cl(w, cuda))
        dx, dgm, dbt = need_ext().conv_igemm_fwd(_cl(dy, cuda), wt, None, 1, k - 1 - p, False, tile, splits,
                                                 _cl(dres, cuda), [t.to(cuda) for t in (gamma, beta, mean, var)],
                                                 2e-5, False, True, _cl(xr, cuda), _cl(dadd, cuda))
        for a, r in ((dx, ref_dx), (dgm, ref_dg), (dbt, ref_db)):
            err = (a.float().cpu() - r).abs().max().item()
            assert err <= 2e-2 * r.abs().max().item() + 2e-2, (Cin, Cout, k, splits, tile, err)


@pytest.mark.gpu
def test_bnb_epilogue_subsampled_dadd(cuda):
    """A stride-s subsampled dadd (a strided projection shortcut's gradient) added by the BN-backward
    epilogue at rows (i*s, j*s) == the same dadd scattered into a zero-filled full-size map, for the
    direct, LDS, ring and split-K epilogues and the grouped dgrad+wgrad launch."""
    from mx_rcnn_amd.ops import need_ext
    from mx_rcnn_amd.ops.conv import _flip_t
    ext = need_ext()
    g = torch.Generator().manual_seed(43)
    for (Cin, Cout, k, H, W, splits, tile, st) in ((256, 1024, 1, 24, 40, 1, 0, 2), (256, 1024, 1, 23, 37, 4, 0, 2),
                                                   (256, 1024, 1, 24, 40, 1, 105, 2), (256, 256, 3, 20, 30, 1, 106, 2),
                                                   (256, 1024, 1, 25, 31, 2, 106, 2)):
        w = (torch.randn(Cout, Cin, k, k, generator=g) * 0.05).bfloat16()
        dy = _cl(torch.randn(1, Cout, H, W, generator=g).bfloat16(), cuda)
        xr = _cl(torch.randn(1, Cin, H, W, generator=g).bfloat16(), cuda)
        sub = _cl(torch.randn(1, Cin, (H + st - 1) // st, (W + st - 1) // st, generator=g).bfloat16(), cuda)
        full = torch.zeros(1, Cin, H, W, dtype=torch.bfloat16, device=cuda).contiguous(memory_format=torch.channels_last)
        full[:, :, ::st, ::st] = sub
        bn = [t.to(cuda) for t in (torch.rand(Cin, generator=g) + 0.5, torch.randn(Cin, generator=g) * 0.1,
                                   torch.randn(Cin, generator=g) * 0.2, torch.rand(Cin, generator=g) + 0.5)]
        wt = _flip_t(_cl(w, cuda))
        p = k // 2
        outs = [ext.conv_igemm_fwd(dy, wt, None, 1, k - 1 - p, False, tile, splits, None, bn, 2e-5, False, True,
                                   xr, d) for d in (sub, full)]
        # dx bitwise; dgamma / dbeta are fp32 atomic sums (summation order varies run to run)
        torch.testing.assert_close(outs[0][0].float(), outs[1][0].float(), rtol=0, atol=0)
        for a, b in zip(outs[0][1:], outs[1][1:]):
            torch.testing.assert_close(a.float(), b.float(), rtol=1e-4, atol=1e-4)


def test_fused_trunk_step_matches_unfused(cuda):
    """One full e2e step on a small ResNet-50: fused and unfused trunks give the same losses."""
    from mx_rcnn_amd.config import snapshot
    from mx_rcnn_amd.core.trainer import Trainer
    from mx_rcnn_amd.models import FasterRCNN
    import bench
    cfg = snapshot()
    cfg.TRAIN.BG_THRESH_LO = 0.0
    cfg.END2END = 1
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    losses = []
    for fuse in ('0', '1'):
        os.environ['MXR_FUSE'] = fuse
        try:
            torch.manual_seed(0)
            m = FasterRCNN('resnet50', 21, cfg=cfg)
            gen = torch.Generator().manual_seed(1)
            batch = bench.synthetic_batch(1, 320, 480, 21, cuda, gen)
            m.to(cuda).calibrate_bn(batch['data'])
            t = Trainer(m, 'e2e', fixed_param_prefix=['conv0', 'stage1', 'bn_data', 'bn0'], lr=0.001, device=cuda)
            torch.manual_seed(3)
            torch.cuda.manual_seed(3)
            out = [t.step(batch) for _ in range(2)]
            losses.append([float(o['rpn_cls_loss']) for o in out] + [float(o['cls_loss']) for o in out])
        finally:
            os.environ.pop('MXR_FUSE', None)
    for a, b in zip(*losses):
        assert abs(a - b) <= 2e-2 * abs(a) + 1e-3, losses


@pytest.mark.parametrize('C,M_hw', [(1024, (128, 7, 7)), (2048, (128, 4, 4)), (512, (64, 7, 7)), (64, (3, 5, 5))])
@pytest.mark.parametrize('relu', [True, False])
def test_train_bn_relu_vs_torch(cuda, C, M_hw, relu):
    from mx_rcnn_amd.ops.bn import train_bn_relu
    N, H, W = M_hw
    g = torch.Generator().manual_seed(31)
    x = (torch.randn(N, C, H, W, generator=g) * 2 + 0.5).bfloat16()
    gamma = (torch.rand(C, generator=g) + 0.5)
    beta = torch.randn(C, generator=g) * 0.1
    dy = torch.randn(N, C, H, W, generator=g).bfloat16()
    # reference: fp32 torch batch norm on the same bf16 input
    xr = x.float().clone().requires_grad_()
    gr, br = gamma.clone().requires_grad_(), beta.clone().requires_grad_()
    rm_r, rv_r = torch.zeros(C), torch.ones(C)
    yr = F.batch_norm(xr, rm_r, rv_r, gr, br, training=True, momentum=0.1, eps=2e-5)
    if relu:
        yr = torch.relu(yr)
    yr.backward(dy.float())
    xg = _cl(x, cuda).requires_grad_()
    gg, bg = gamma.to(cuda).requires_grad_(), beta.to(cuda).requires_grad_()
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    yg = train_bn_relu(xg, gg, bg, rm, rv, 0.9, 2e-5, False, relu)
    yg.backward(_cl(dy, cuda))
    for a, r in ((yg, yr), (xg.grad, xr.grad), (gg.grad, gr.grad), (bg.grad, br.grad), (rm, rm_r), (rv, rv_r)):
        err = (a.float().cpu() - r.detach()).abs().max().item()
        assert err <= 2e-2 * r.abs().max().item() + 2e-3, err


@pytest.mark.parametrize('N,Cin,Cout,H,W,k,s,p', [(1, 256, 256, 100, 167, 3, 2, 1), (128, 512, 512, 7, 7, 3, 2, 1),
                                                 (2, 64, 128, 15, 22, 3, 2, 1), (1, 64, 64, 9, 10, 5, 2, 2),
                                                 (1, 128, 64, 12, 13, 3, 3, 0)])
def test_strided_dgrad_parity_classes(cuda, N, Cin, Cout, H, W, k, s, p):
    """Parity-decomposed stride-s data gradient on the MFMA kernel (output row map) vs fp32 torch."""
    from mx_rcnn_amd.ops.conv import _flip_t, strided_dgrad, strided_dgrad_ok
    assert strided_dgrad_ok(k, s, p, H, W)
    g = torch.Generator().manual_seed(51)
    x = torch.randn(N, Cin, H, W, generator=g).bfloat16()
    w = (torch.randn(Cout, Cin, k, k, generator=g) * 0.05).bfloat16()
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(N, Cout, Ho, Wo, generator=g).bfloat16()
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [s, s], [p, p], [1, 1], False,
                                              [0, 0], 1, [True, False, False])[0]
    dx = strided_dgrad(_cl(dy, cuda), _flip_t(_cl(w, cuda)), H, W, k, s, p)
    err = (dx.float().cpu() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-2, err


def test_strided_dgrad_bnb_epilogue(cuda):
    """Strided dgrad fused with the BN-ReLU backward (+dadd, +residual): dx and dgamma / dbeta
    accumulated over the parity classes vs unfused fp32 ops."""
    from mx_rcnn_amd.ops.conv import _flip_t, strided_dgrad
    g = torch.Generator().manual_seed(52)
    Cin, Cout, H, W, k, s, p = 256, 256, 21, 34, 3, 2, 1
    w = (torch.randn(Cout, Cin, k, k, generator=g) * 0.05).bfloat16()
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(1, Cout, Ho, Wo, generator=g).bfloat16()
    xr = torch.randn(1, Cin, H, W, generator=g).bfloat16()
    dadd = torch.randn(1, Cin, H, W, generator=g).bfloat16()
    dres = torch.randn(1, Cin, H, W, generator=g).bfloat16()
    gamma, beta = torch.rand(Cin, generator=g) + 0.5, torch.randn(Cin, generator=g) * 0.1
    mean, var = torch.randn(Cin, generator=g) * 0.2, torch.rand(Cin, generator=g) + 0.5
    d_act = torch.ops.aten.convolution_backward(dy.float(), xr.float(), w.float(), None, [s, s], [p, p], [1, 1],
                                                False, [0, 0], 1, [True, False, False])[0] + dadd.float()
    sc = gamma * torch.rsqrt(var + 2e-5)
    pre = xr.float() * sc[None, :, None, None] + (beta - mean * sc)[None, :, None, None]
    gm = d_act * (pre > 0).float()
    ref_dx = gm * sc[None, :, None, None] + dres.float()
    xhat = (xr.float() - mean[None, :, None, None]) * torch.rsqrt(var + 2e-5)[None, :, None, None]
    ref_dg, ref_db = (gm * xhat).sum(dim=(0, 2, 3)), gm.sum(dim=(0, 2, 3))
    dx, dgm, dbt = strided_dgrad(_cl(dy, cuda), _flip_t(_cl(w, cuda)), H, W, k, s, p, residual=_cl(dres, cuda),
                                 bn=[t.to(cuda) for t in (gamma, beta, mean, var)], bnb_x=_cl(xr, cuda),
                                 dadd=_cl(dadd, cuda))
    for a, r in ((dx, ref_dx), (dgm, ref_dg), (dbt, ref_db)):
        err = (a.float().cpu() - r).abs().max().item()
        assert err <= 2e-2 * r.abs().max().item() + 2e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize('geo', [(256, 1024, 1, 24, 40, 1024, 256, 1, 1, 0), (256, 256, 3, 20, 30, 256, 256, 3, 1, 1),
                                 (1024, 256, 1, 50, 84, 256, 1024, 1, 1, 0), (256, 256, 3, 50, 84, 256, 512, 1, 1, 0)])
@pytest.mark.parametrize('with_bn,defer', [(True, False), (False, False), (True, True)])
def test_grouped_dgrad_wgrad_matches_separate(cuda, geo, with_bn, defer):
    """conv_dgrad_wgrad (one launch: BN-backward dgrad role + split-K wgrad role) against the same
    two computations as separate launches (buffer kernel tile 23, conv_wgrad): same bodies, so the
    data gradient and the weight gradient agree to rounding; dgamma / dbeta to atomic order."""
    from mx_rcnn_amd.ops import need_ext
    from mx_rcnn_amd.ops.conv import _flip_t
    Cin, Cout, k, H, W, wCo, wCi, wk, ws, wp = geo
    g = torch.Generator().manual_seed(5)
    ext = need_ext()
    w = (torch.randn(Cout, Cin, k, k, generator=g) * 0.05).bfloat16()
    dy = _cl(torch.randn(1, Cout, H, W, generator=g).bfloat16(), cuda)
    xr = _cl(torch.randn(1, Cin, H, W, generator=g).bfloat16(), cuda)
    dres = _cl(torch.randn(1, Cin, H, W, generator=g).bfloat16(), cuda)
    bn = [t.to(cuda) for t in (torch.rand(Cin, generator=g) + 0.5, torch.randn(Cin, generator=g) * 0.1,
                               torch.randn(Cin, generator=g) * 0.2, torch.rand(Cin, generator=g) + 0.5)]
    Ho, Wo = (H + 2 * wp - wk) // ws + 1, (W + 2 * wp - wk) // ws + 1
    wdy = _cl(torch.randn(1, wCo, Ho, Wo, generator=g).bfloat16(), cuda)
    wx = _cl(torch.randn(1, wCi, H, W, generator=g).bfloat16(), cuda)
    dw0 = _cl((torch.randn(wCo, wCi, wk, wk, generator=g) * 0.1).bfloat16(), cuda)
    wt = _flip_t(_cl(w, cuda))
    p = k // 2
    tg, tb = torch.zeros(Cin, device=cuda), torch.zeros(Cin, device=cuda)
    dw = dw0.clone()
    if with_bn:
        dx, dgm, dbt, slab = ext.conv_dgrad_wgrad(dy, wt, k - 1 - p, dres, bn, 2e-5, False, xr, None, tg, tb, wdy, wx,
                                                  wk, wk, ws, wp, dw, defer)
        rdx, rdg, rdb = ext.conv_igemm_fwd(dy, wt, None, 1, k - 1 - p, False, 23, 1, dres, bn, 2e-5, False, True, xr,
                                           None)
    else:
        dx, _, _, slab = ext.conv_dgrad_wgrad(dy, wt, k - 1 - p, dres, None, 0.0, False, None, None, None, None, wdy,
                                              wx, wk, wk, ws, wp, dw, defer)
        rdx = ext.conv_igemm_fwd(dy, wt, None, 1, k - 1 - p, False, 23, 1, dres)[0]
    if defer and slab.numel() > 0:
        # the deferred reduce runs as role 0 of the next grouped launch: a second (throw-away) one
        dw2 = dw0.clone()
        ext.conv_dgrad_wgrad(dy, wt, k - 1 - p, None, None, 0.0, False, None, None, None, None, wdy, wx, wk, wk, ws,
                             wp, dw2, False, slab, dw)
    rdw = dw0.clone()
    ext.conv_wgrad(wdy, wx, wk, wk, ws, wp, 0, rdw)
    torch.cuda.synchronize()
    assert torch.equal(dx, rdx)
    assert torch.allclose(dw.float(), rdw.float(), rtol=1e-2, atol=1e-2 * rdw.float().abs().max().item())
    if with_bn:
        for a, r in ((dgm, rdg), (dbt, rdb)):
            assert torch.allclose(a, r, rtol=1e-4, atol=1e-4 * r.abs().max().item() + 1e-5)


@pytest.mark.gpu
def test_grouped_unit_backward_matches_side_stream(cuda, monkeypatch):
    """A fused stage-3 style unit pair under the FlatParamStore (direct gradient sinks, so the
    grouped launches run) against MXR_GROUPED_BWD=0 (weight gradients on the side stream)."""
    import copy
    from mx_rcnn_amd.core.params import FlatParamStore
    from mx_rcnn_amd.models.resnet import run_stage, _stage
    class _Holder(torch.nn.Module):
        def __init__(self, st):
            super().__init__()
            self.st = st

        def mx_layers(self, mode=None):
            return (m for m in self.modules() if hasattr(m, 'mx_args'))

    torch.manual_seed(0)
    stage = _stage(3, 3, 512, 1024, True, 0.99, True).to(cuda)
    for mod in stage.modules():
        if hasattr(mod, 'moving_var'):
            mod.moving_var.uniform_(0.5, 1.5)
            mod.moving_mean.normal_(0, 0.1)
    x0 = torch.randn(1, 512, 50, 84).bfloat16()
    res = []
    for grouped in ('1', '0'):
        monkeypatch.setenv('MXR_GROUPED_BWD', grouped)
        st = copy.deepcopy(stage)
        store = FlatParamStore(_Holder(st), device=cuda)
        store.zero_grad()
        x = _cl(x0, cuda).requires_grad_()
        out = run_stage(st, x)
        gen = torch.Generator().manual_seed(7)
        out.backward(torch.randn(out.shape, generator=gen).bfloat16().to(cuda).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
        res.append((x.grad.float(), {n: p.grad.float().clone() for n, p in store.params.items()}))
    (xa, ga), (xb, gb) = res
    assert _rel(xa, xb) <= 1e-2
    for n in ga:
        assert _rel(ga[n], gb[n]) <= 2e-2, (n, _rel(ga[n], gb[n]))


@pytest.mark.parametrize('shape', [(16, 512, 4, 4, 512, 3, 1, 1), (16, 1024, 7, 7, 256, 1, 1, 0),
                                   (16, 256, 7, 7, 1024, 1, 2, 0), (1, 256, 50, 84, 1024, 1, 1, 0)])
@pytest.mark.parametrize('tile', [0, 23, 22, 101, 104, 106, 109])
def test_conv_stats_epilogue(cuda, shape, tile):
    """Training-BN statistics partials written by the conv epilogue (ConvEpi::st_part): folded
    they equal the fp32 column sums of the STORED output, shifted by the given shift."""
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    N, Cin, H, W, Cout, k, s, p = shape
    g = torch.Generator().manual_seed(11)
    x = _cl(torch.randn(N, Cin, H, W, generator=g).bfloat16(), cuda)
    w = _cl((torch.randn(Cout, Cin, k, k, generator=g) * 0.05).bfloat16(), cuda)
    shift = (torch.randn(Cout, generator=g) * 0.1).to(cuda)
    res = None
    if s == 1 and k == 1:
        res = _cl(torch.randn(N, Cout, H, W, generator=g).bfloat16(), cuda)
    y, part = ext.conv_igemm_fwd(x, w, None, s, p, False, tile, 0, res, stat_shift=shift)
    assert part.dim() == 2 and part.shape[1] == Cout and part.shape[0] % 2 == 1
    nparts = (part.shape[0] - 1) // 2
    pr = part[:2 * nparts].view(nparts, 2, Cout).sum(0)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, Cout) - shift[None]
    assert torch.allclose(pr[0], yf.sum(0), rtol=1e-4, atol=1e-3)
    assert torch.allclose(pr[1], (yf * yf).sum(0), rtol=1e-4, atol=1e-3)
    assert torch.equal(part[2 * nparts], shift)
    # the output itself is unchanged by the statistics epilogue
    y0 = ext.conv_igemm_fwd(x, w, None, s, p, False, tile, 1, res)[0]
    assert torch.equal(y, y0) if tile else _rel(y, y0) <= 1e-3


def test_bn_train_apply_and_dx_apply(cuda):
    """bn_train_apply (normalisation from conv-epilogue partials) and bn_train_dx_apply (the
    backward finish after a BN-backward dgrad epilogue) vs fp32 torch batch-norm."""
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(12)
    N, Cin, H, W, C = 32, 256, 4, 4, 512
    x = _cl(torch.randn(N, Cin, H, W, generator=g).bfloat16(), cuda)
    w = _cl((torch.randn(C, Cin, 1, 1, generator=g) * 0.1).bfloat16(), cuda)
    gamma = (torch.rand(C, generator=g) + 0.5).to(cuda)
    beta = (torch.randn(C, generator=g) * 0.1).to(cuda)
    rm = (torch.randn(C, generator=g) * 0.1).to(cuda)
    rv = (torch.rand(C, generator=g) + 0.5).to(cuda)
    rm0, rv0 = rm.clone(), rv.clone()
    y, part = ext.conv_igemm_fwd(x, w, None, 1, 0, False, stat_shift=rm)
    a, save = ext.bn_train_apply(y, part, gamma, beta, rm, rv, 0.9, 2e-5, False, True)
    yf = y.float()
    mu = yf.mean(dim=(0, 2, 3))
    var = yf.var(dim=(0, 2, 3), unbiased=False)
    ref = torch.relu((yf - mu[None, :, None, None]) * (gamma * torch.rsqrt(var + 2e-5))[None, :, None, None] +
                     beta[None, :, None, None])
    assert _rel(a.float(), ref) <= 1e-2
    assert torch.allclose(save[0], mu, atol=1e-4, rtol=1e-4)
    assert torch.allclose(save[2], var + 2e-5, atol=1e-4, rtol=1e-4)
    Mr = N * H * W
    assert torch.allclose(rm, 0.9 * rm0 + 0.1 * mu, atol=1e-4)
    assert torch.allclose(rv, 0.9 * rv0 + 0.1 * var * Mr / (Mr - 1), atol=1e-4, rtol=1e-4)
    # backward: d_a (gradient at the BN-ReLU output) comes from a dgrad conv in the real unit; here
    # the BN-backward epilogue is driven by a 1x1 "dgrad" of a random dY through the conv weight
    w2 = _cl((torch.randn(1024, C, 1, 1, generator=g) * 0.05).bfloat16(), cuda)  # the next conv: C -> 1024
    dy = _cl(torch.randn(N, 1024, H, W, generator=g).bfloat16(), cuda)
    from mx_rcnn_amd.ops.conv import _flip_t
    wf = _cl(_flip_t(w2), cuda)
    dres = _cl(torch.randn(N, C, H, W, generator=g).bfloat16(), cuda)
    nparts = (N * H * W + 63) // 64
    part = torch.empty(nparts * 2 * C, device=cuda)
    o = ext.conv_igemm_fwd(dy, wf, None, 1, 0, False, 0, 0, None, [gamma, beta, save[0], save[2]], 0.0, False,
                           True, y, bnb_part=part)[0]
    dgam = torch.zeros(C, device=cuda)
    dbet = torch.zeros(C, device=cuda)
    dx = ext.bn_train_dx_apply(o, y, save, gamma, part, nparts, dres, dgam, dbet)
    # fp32 oracle
    yr = yf.clone().requires_grad_()
    out = torch.relu(F.batch_norm(yr, None, None, gamma, beta, training=True, eps=2e-5))
    d_act = F.conv2d(dy.float(), w2.float().permute(1, 0, 2, 3))
    out.backward(d_act)
    assert _rel(dx.float() - dres.float(), yr.grad) <= 3e-2
    assert _rel(dgam, _ref_dgamma(yf, d_act, gamma, beta)) <= 1e-2
    assert _rel(dbet, (d_act * (out > 0)).sum(dim=(0, 2, 3))) <= 1e-2


def _ref_dgamma(yf, d_act, gamma, beta):
    mu = yf.mean(dim=(0, 2, 3), keepdim=True)
    var = yf.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
    xh = (yf - mu) * torch.rsqrt(var + 2e-5)
    mask = (xh * gamma[None, :, None, None] + beta[None, :, None, None]) > 0
    return (d_act * mask * xh).sum(dim=(0, 2, 3))


def _train_stage(cuda, n_units=3, cin=512, cout=1024):
    from mx_rcnn_amd.models.resnet import _stage
    from mx_rcnn_amd.models.layers import BatchNorm
    torch.manual_seed(3)
    st = _stage(4, n_units, cin, cout, True, 0.9, False)
    tail = BatchNorm('bn1', cout, momentum=0.9, use_global_stats=False)
    with torch.no_grad():
        for m in list(st.modules()) + [tail]:
            if hasattr(m, 'moving_var'):
                m.moving_mean.normal_(0, 0.2)
                m.moving_var.uniform_(0.5, 1.5)
                m.gamma.uniform_(0.5, 1.5)
                m.beta.normal_(0, 0.1)
            elif hasattr(m, 'weight') and m.weight is not None:
                m.weight.normal_(0, 0.03)
    st, tail = st.to(cuda).train(), tail.to(cuda).train()
    for m in st.modules():
        if hasattr(m, 'weight') and m.weight is not None and m.weight.dim() == 4:
            m.weight = torch.nn.Parameter(m.weight.detach().bfloat16().contiguous(memory_format=torch.channels_last))
    return st, tail


def test_train_units_match_module_path(cuda, monkeypatch):
    """The RoI-head stage (batch-statistics BNs) through the fused train-unit op -- statistics
    in the conv epilogues, BN backward in the dgrad epilogues + dx_apply -- vs the per-module
    path (MXR_TRAIN_UNIT=0), including the head bn1 fed by the last unit's partials.  Both bf16
    paths are scored against an fp32 CPU run of the same stage: the fused path's error may not
    exceed the module path's by more than bf16 noise."""
    import copy
    from mx_rcnn_amd.models.resnet import run_stage_parts
    st0, tail0 = _train_stage(cuda)
    g = torch.Generator().manual_seed(9)
    x0 = torch.randn(16, 512, 8, 8, generator=g).bfloat16()
    d0 = torch.randn(16, 1024, 4, 4, generator=torch.Generator().manual_seed(7)).bfloat16()

    def run(st, tail, dev, dtype):
        x = x0.to(dev, dtype).contiguous(memory_format=torch.channels_last).requires_grad_()
        y, parts = run_stage_parts(st, x, tail)
        out = tail(y, parts=parts)
        out.backward(d0.to(dev, out.dtype).contiguous(memory_format=torch.channels_last))
        grads = {n: p.grad.float().cpu().clone() for n, p in list(st.named_parameters()) +
                 [('tail.' + n, p) for n, p in tail.named_parameters()] if p.grad is not None}
        stats = {n: b.float().cpu().clone() for n, b in list(st.named_buffers()) +
                 [('tail.' + n, b) for n, b in tail.named_buffers()]}
        return out.detach().float().cpu(), x.grad.float().cpu(), grads, stats, parts

    ref = run(copy.deepcopy(st0).cpu().float(), copy.deepcopy(tail0).cpu().float(), 'cpu', torch.float32)
    res = []
    for flag in ('0', '1'):
        monkeypatch.setenv('MXR_TRAIN_UNIT', flag)
        r = run(copy.deepcopy(st0), copy.deepcopy(tail0), cuda, torch.bfloat16)
        assert (r[4] is not None) == (flag == '1')
        torch.cuda.synchronize()
        res.append(r)
    (oa, xa, ga, sa, _), (ob, xb, gb, sb, _) = res
    o_r, x_r, g_r, s_r, _ = ref

    def close(b, a, r, what):
        ea, eb = _rel(a, r), _rel(b, r)
        assert eb <= max(1.25 * ea, 0.03), (what, eb, ea)

    close(ob, oa, o_r, 'out')
    close(xb, xa, x_r, 'dx')
    assert set(ga) == set(gb) == set(g_r), set(ga) ^ set(gb)
    for n in ga:
        close(gb[n], ga[n], g_r[n], n)
    for n in sa:
        close(sb[n], sa[n], s_r[n], n)


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('stride', [1, 2])
def test_inference_bn_fold_matches_training_form(cuda, monkeypatch, dtype, stride):
    """Inference folds each bottleneck's frozen bn2 / bn3 into its 1x1 reduce / 3x3 (scale into a
    cached filter copy, shift as the bias, ReLU epilogue; ops/fused.py _folded) on our kernels --
    no vendor GEMM (torch._addmm_activation / F.linear / F.conv2d are made to raise).  The unit
    output matches the training-form epilogues (MXR_INFER_FOLD=0) within the 16-bit rounding, and
    the fold is rebuilt when the BN statistics or (through the training generation) the weights
    change."""
    import torch.nn.functional as Fn
    from mx_rcnn_amd.ops import fused
    u = _unit(1024, 1024, stride, stride == 1, cuda)
    for m in u.modules():
        if hasattr(m, 'weight') and m.weight is not None and m.weight.dim() == 4:
            m.weight = torch.nn.Parameter(m.weight.detach().to(dtype).contiguous(memory_format=torch.channels_last))
    x = torch.randn(4, 1024, 64, 64, device=cuda).to(dtype).contiguous(memory_format=torch.channels_last)

    def boom(*a, **k):
        raise AssertionError('vendor GEMM / conv on the inference path')

    def run(fold):
        monkeypatch.setenv('MXR_INFER_FOLD', '1' if fold else '0')
        with monkeypatch.context() as mp:
            mp.setattr(torch, '_addmm_activation', boom)
            mp.setattr(Fn, 'conv2d', boom)
            mp.setattr(Fn, 'linear', boom)
            with torch.no_grad():
                return fused.fused_unit(u, x)[0].float()

    a = run(True)
    assert '_mxr_bn_fold' in u.conv1.weight.__dict__ and '_mxr_bn_fold' in u.conv2.weight.__dict__
    b = run(False)
    scale = b.abs().max().item()
    assert (a - b).abs().max().item() <= 2e-2 * scale
    with torch.no_grad():
        u.bn2.moving_var.mul_(4.0)
    c, d = run(True), run(False)
    assert (c - d).abs().max().item() <= 2e-2 * d.abs().max().item()
    assert (c - a).abs().max().item() > 1e-3 * scale  # the new statistics were used
    # a training step rewrites trainable weights in place, moving no version counter: the fold
    # follows the training generation (core/trainer.py bumps it every step)
    from mx_rcnn_amd.ops import precision
    with torch.no_grad():
        u.conv1.weight.data.mul_(0.5)
    precision.bump_generation()
    e, f = run(True), run(False)
    assert (e - f).abs().max().item() <= 2e-2 * f.abs().max().item()
    assert (e - c).abs().max().item() > 1e-3 * scale

