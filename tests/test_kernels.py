"""RoIPool / fused losses / frozen BN+ReLU / fused SGD: CPU reference vs plain PyTorch fp32
formulations, and HIP kernels vs the fp32 reference (gpu)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from mx_rcnn_amd import ops
from mx_rcnn_amd.ops.roi_pool import roi_pool_ref


def _naive_roi_pool(feat, rois, PH, PW, scale):
    B, C, H, W = feat.shape
    out = np.zeros((rois.shape[0], C, PH, PW))
    for r, roi in enumerate(rois):
        b = int(roi[0])
        rd = lambda v: math.floor(v + 0.5)  # noqa: E731
        x1, y1, x2, y2 = [rd(v * scale) for v in roi[1:]]
        rw, rh = max(x2 - x1 + 1, 1), max(y2 - y1 + 1, 1)
        for ph in range(PH):
            for pw in range(PW):
                hs = min(max(math.floor(ph * rh / PH) + y1, 0), H)
                he = min(max(math.ceil((ph + 1) * rh / PH) + y1, 0), H)
                ws = min(max(math.floor(pw * rw / PW) + x1, 0), W)
                we = min(max(math.ceil((pw + 1) * rw / PW) + x1, 0), W)
                if he > hs and we > ws:
                    out[r, :, ph, pw] = feat[b, :, hs:he, ws:we].reshape(C, -1).max(1)
    return out


def _rois(g, R, B, H, W, stride=16):
    xy = torch.rand(R, 2, generator=g) * torch.tensor([W * stride * 0.8, H * stride * 0.8])
    wh = torch.rand(R, 2, generator=g) * 200 + 1
    b = torch.randint(0, B, (R, 1), generator=g).float()
    return torch.cat([b, xy, xy + wh], 1)


def test_roi_pool_ref_matches_naive():
    g = torch.Generator().manual_seed(0)
    feat = torch.randn(2, 5, 12, 17, generator=g)
    rois = _rois(g, 9, 2, 12, 17)
    rois[0, 1:] = torch.tensor([-30., -30, -20, -20])  # fully outside -> empty bins
    out, arg = roi_pool_ref(feat, rois, 7, 7, 1 / 16)
    np.testing.assert_allclose(out.numpy(), _naive_roi_pool(feat.numpy(), rois.numpy(), 7, 7, 1 / 16), atol=1e-6)


def test_roi_pool_backward_ref():
    g = torch.Generator().manual_seed(1)
    feat = torch.randn(1, 3, 10, 10, generator=g, dtype=torch.float64).requires_grad_()
    rois = _rois(g, 4, 1, 10, 10)
    out = ops.roi_pool(feat, rois, (7, 7), 1 / 16)
    gout = torch.randn_like(out)
    out.backward(gout)
    # scatter check: gradient mass equals the sum of top grads of non-empty bins
    _, arg = roi_pool_ref(feat.detach(), rois, 7, 7, 1 / 16)
    assert torch.allclose(feat.grad.sum(), (gout * (arg >= 0)).sum())


def test_losses_cpu_vs_torch():
    g = torch.Generator().manual_seed(2)
    B, A, H, W = 2, 3, 4, 5
    logits = torch.randn(B, 2 * A, H, W, generator=g, requires_grad=True)
    label = torch.randint(-1, 2, (B, A * H * W), generator=g)
    loss = ops.rpn_softmax_ce(logits, label)
    loss.backward()
    z = logits.detach().reshape(B, 2, A * H, W).clone().requires_grad_()
    lab = label.reshape(B, A * H, W)
    ref = F.cross_entropy(z, lab.clamp_min(0), reduction='none')
    valid = (lab >= 0).float()
    ref = (ref * valid).sum() / valid.sum()
    ref.backward()
    assert torch.allclose(loss, ref, atol=1e-6)
    assert torch.allclose(logits.grad.reshape(B, 2, A * H, W), z.grad, atol=1e-6)

    x = torch.randn(7, 5, generator=g, requires_grad=True)
    lab = torch.randint(0, 5, (7,), generator=g)
    l2, prob = ops.softmax_ce(x, lab)
    l2.backward()
    x2 = x.detach().clone().requires_grad_()
    r2 = F.cross_entropy(x2, lab)
    r2.backward()
    assert torch.allclose(l2, r2, atol=1e-6) and torch.allclose(x.grad, x2.grad, atol=1e-6)

    pred = torch.randn(3, 8, generator=g, requires_grad=True)
    tgt = torch.randn(3, 8, generator=g)
    iw = (torch.rand(3, 8, generator=g) > 0.5).float()
    ow = torch.rand(3, 8, generator=g)
    l3 = ops.smooth_l1(pred, tgt, iw, ow, sigma=3.0, grad_scale=0.5)
    l3.backward()
    p2 = pred.detach().clone().requires_grad_()
    x3 = iw * (p2 - tgt)
    s2 = 9.0
    f = torch.where(x3.abs() < 1 / s2, 0.5 * s2 * x3 * x3, x3.abs() - 0.5 / s2)
    (ow * f).sum().mul(0.5).backward()
    assert torch.allclose(l3, (ow * f).sum(), atol=1e-6)
    assert torch.allclose(pred.grad, p2.grad, atol=1e-6)


def test_frozen_bn_relu_cpu():
    g = torch.Generator().manual_seed(3)
    C = 8
    x = torch.randn(2, C, 5, 6, generator=g, requires_grad=True)
    gamma = torch.rand(C, generator=g).requires_grad_()
    beta = torch.randn(C, generator=g).requires_grad_()
    mean, var = torch.randn(C, generator=g), torch.rand(C, generator=g) + 0.5
    y = ops.frozen_bn_relu(x, gamma, beta, mean, var, 2e-5)
    y.sum().backward()
    x2, g2, b2 = [t.detach().clone().requires_grad_() for t in (x, gamma, beta)]
    y2 = F.relu(F.batch_norm(x2, mean, var, g2, b2, training=False, eps=2e-5))
    y2.sum().backward()
    assert torch.allclose(y, y2, atol=1e-5)
    for a, b in [(x.grad, x2.grad), (gamma.grad, g2.grad), (beta.grad, b2.grad)]:
        assert torch.allclose(a, b, atol=1e-4)


def test_sgd_cpu_semantics():
    w = torch.tensor([1.0, -2.0, 3.0])
    m = torch.tensor([0.1, 0.0, -0.1])
    g = torch.tensor([5.0, -0.5, 0.2])
    lr = torch.tensor([0.1])
    w0, m0 = w.clone(), m.clone()
    ops.sgd_momentum_(w, m, g, lr, momentum=0.9, wd=0.01, rescale=1.0, clip=1.0)
    gc = g.clamp(-1, 1)
    m_ref = 0.9 * m0 - 0.1 * (gc + 0.01 * w0)
    assert torch.allclose(m, m_ref) and torch.allclose(w, w0 + m_ref)


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize('dtype,C', [(torch.float32, 64), (torch.bfloat16, 1024), (torch.float32, 6)])
def test_roi_pool_gpu(cuda, dtype, C):
    g = torch.Generator().manual_seed(4)
    B, H, W = 2, 38, 50
    feat = torch.randn(B, C, H, W, generator=g)
    rois = _rois(g, 64, B, H, W)
    rois[3, 0] = -1  # invalid batch index
    ref, arg_ref = roi_pool_ref(feat.to(dtype).float(), rois, 7, 7, 1 / 16)
    fg = feat.to(cuda, dtype).contiguous(memory_format=torch.channels_last).requires_grad_()
    from mx_rcnn_amd.ops import need_ext
    _, arg_gpu = need_ext().roi_pool_fwd(fg.detach(), rois.to(cuda), 7, 7, 1 / 16)
    assert torch.equal(arg_gpu.cpu(), arg_ref), int((arg_gpu.cpu() != arg_ref).sum())
    out = ops.roi_pool(fg, rois.to(cuda), (7, 7), 1 / 16)
    assert torch.allclose(out.float().cpu(), ref, atol=0, rtol=0)
    gout = torch.randn(out.shape, generator=g).to(cuda, dtype)
    out.backward(gout)
    # reference backward in fp32 from the reference argmax
    gin = torch.zeros(B, C * H * W, dtype=torch.float64)
    go = gout.double().cpu().reshape(64, C, -1)
    a = arg_ref.reshape(64, C, -1).long()
    for r in range(64):
        b = int(rois[r, 0])
        if b < 0:
            continue
        m = a[r] >= 0
        gin[b].index_add_(0, (torch.arange(C)[:, None] * H * W + a[r].clamp_min(0))[m], go[r][m])
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    got = fg.grad.double().cpu().reshape(B, -1)
    bad = ~torch.isclose(got, gin, atol=tol, rtol=tol)
    assert not bad.any(), 'mismatch %d/%d max %.4g; argmax equal: %s' % (
        int(bad.sum()), bad.numel(), float((got - gin).abs().max()),
        bool(torch.equal(torch.empty(0), torch.empty(0))))


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_roi_pool_backward_propagates_nonfinite(cuda, dtype):
    """the fixed-point backward must not turn a NaN / inf head gradient into a large
    finite trunk gradient -- the affected (image, channel) comes out NaN, every other channel exact."""
    g = torch.Generator().manual_seed(6)
    B, C, H, W = 2, 64, 30, 40
    feat = torch.randn(B, C, H, W, generator=g)
    rois = _rois(g, 32, B, H, W)
    fg = feat.to(cuda, dtype).contiguous(memory_format=torch.channels_last).requires_grad_()
    out = ops.roi_pool(fg, rois.to(cuda), (7, 7), 1 / 16)
    gout = torch.randn(out.shape, generator=g)
    r_nan = int((rois[:, 0] == 0).nonzero()[0])
    r_inf = int((rois[:, 0] == 1).nonzero()[0])
    gout[r_nan, 5, 3, 3] = float('nan')
    gout[r_inf, 9, 0, 0] = float('inf')
    out.backward(gout.to(cuda, dtype))
    got = fg.grad.float().cpu()
    assert torch.isnan(got[0, 5]).all() and torch.isnan(got[1, 9]).all()
    clean = torch.ones(B, C, dtype=torch.bool)
    clean[0, 5] = False
    clean[1, 9] = False
    assert torch.isfinite(got[clean]).all()
    gc = gout.clone()
    gc[r_nan, 5, 3, 3] = 0
    gc[r_inf, 9, 0, 0] = 0
    fg2 = fg.detach().clone().requires_grad_()
    ops.roi_pool(fg2, rois.to(cuda), (7, 7), 1 / 16).backward(gc.to(cuda, dtype))
    assert torch.equal(got[clean], fg2.grad.float().cpu()[clean])


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_losses_gpu(cuda, dtype):
    g = torch.Generator().manual_seed(5)
    B, A, H, W = 2, 12, 20, 31
    logits = torch.randn(B, 2 * A, H, W, generator=g)
    label = torch.randint(-1, 2, (B, A * H * W), generator=g)
    lc = logits.to(dtype).float().clone().requires_grad_()
    l_cpu = ops.rpn_softmax_ce(lc, label)
    l_cpu.backward()
    lg = logits.to(cuda, dtype).contiguous(memory_format=torch.channels_last).requires_grad_()
    l_gpu = ops.rpn_softmax_ce(lg, label.to(cuda))
    l_gpu.backward()
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    assert abs(float(l_gpu) - float(l_cpu)) < 1e-4
    assert torch.allclose(lg.grad.float().cpu(), lc.grad, atol=tol)

    x = torch.randn(128, 81, generator=g)
    lab = torch.randint(0, 81, (128,), generator=g)
    xc = x.to(dtype).float().clone().requires_grad_()
    lcpu, pc = ops.softmax_ce(xc, lab)
    lcpu.backward()
    xg = x.to(cuda, dtype).requires_grad_()
    lgpu, pg = ops.softmax_ce(xg, lab.to(cuda))
    lgpu.backward()
    assert abs(float(lgpu) - float(lcpu)) < 1e-4
    assert torch.allclose(pg.cpu(), pc, atol=1e-5)
    assert torch.allclose(xg.grad.float().cpu(), xc.grad, atol=tol)

    pred = torch.randn(B, 4 * A, H, W, generator=g)
    tgt = torch.randn(B, 4 * A, H, W, generator=g)
    iw = (torch.rand(B, 4 * A, H, W, generator=g) > 0.7).float()
    ow = iw / 256
    pc_ = pred.to(dtype).float().clone().requires_grad_()
    s_cpu = ops.smooth_l1(pc_, tgt, iw, ow, 3.0, 1.0)
    s_cpu.backward()
    pg_ = pred.to(cuda, dtype).contiguous(memory_format=torch.channels_last).requires_grad_()
    s_gpu = ops.smooth_l1(pg_, tgt.to(cuda), iw.to(cuda), ow.to(cuda), 3.0, 1.0)
    s_gpu.backward()
    assert abs(float(s_gpu) - float(s_cpu)) < 1e-3 * max(1.0, abs(float(s_cpu)))
    assert torch.allclose(pg_.grad.float().cpu(), pc_.grad, atol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize('dtype,C', [(torch.float32, 64), (torch.bfloat16, 256), (torch.bfloat16, 2048),
                                     (torch.bfloat16, 3)])
def test_frozen_bn_relu_gpu(cuda, dtype, C):
    g = torch.Generator().manual_seed(6)
    x = torch.randn(2, C, 9, 13, generator=g)
    gamma, beta = torch.rand(C, generator=g), torch.randn(C, generator=g)
    mean, var = torch.randn(C, generator=g), torch.rand(C, generator=g) + 0.5
    xc = x.to(dtype).float().clone().requires_grad_()
    gc, bc = gamma.clone().requires_grad_(), beta.clone().requires_grad_()
    y = ops.frozen_bn_relu(xc, gc, bc, mean, var)
    dy = torch.randn(y.shape, generator=g).to(dtype).float()
    y.backward(dy)
    xg = x.to(cuda, dtype).contiguous(memory_format=torch.channels_last).requires_grad_()
    gg, bg = gamma.to(cuda).requires_grad_(), beta.to(cuda).requires_grad_()
    yg = ops.frozen_bn_relu(xg, gg, bg, mean.to(cuda), var.to(cuda))
    yg.backward(dy.to(cuda, dtype))
    tol = 1e-5 if dtype == torch.float32 else 3e-2
    assert torch.allclose(yg.float().cpu(), y.detach(), atol=tol, rtol=tol)
    assert torch.allclose(xg.grad.float().cpu(), xc.grad, atol=tol, rtol=tol)
    assert torch.allclose(gg.grad.cpu(), gc.grad, atol=1e-2, rtol=1e-2)
    assert torch.allclose(bg.grad.cpu(), bc.grad, atol=1e-2, rtol=1e-2)


@pytest.mark.gpu
def test_sgd_gpu(cuda):
    g = torch.Generator().manual_seed(7)
    n = 100003
    w = torch.randn(n, generator=g)
    m = torch.randn(n, generator=g) * 0.01
    gr = torch.randn(n, generator=g) * 2
    lr = torch.tensor([0.01])
    wc, mc = w.clone(), m.clone()
    ops.sgd_momentum_(wc, mc, gr, lr, 0.9, 5e-4, 1.0, 1.0)
    wg, mg = w.to(cuda), m.to(cuda)
    wb = torch.empty(n, dtype=torch.bfloat16, device=cuda)
    ops.sgd_momentum_(wg, mg, gr.to(cuda).bfloat16(), lr.to(cuda), 0.9, 5e-4, 1.0, 1.0, wb)
    # bf16 grads -> loose; fp32 path exact
    assert torch.allclose(wg.cpu(), wc, atol=1e-4)
    assert torch.allclose(wb.float().cpu(), wg.cpu(), atol=1e-2, rtol=1e-2)
    wg2, mg2 = w.to(cuda), m.to(cuda)
    ops.sgd_momentum_(wg2, mg2, gr.to(cuda), lr.to(cuda), 0.9, 5e-4, 1.0, 1.0)
    assert torch.allclose(wg2.cpu(), wc, atol=1e-6) and torch.allclose(mg2.cpu(), mc, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize('variant', ['0', '2'])
def test_sgd_gpu_fused_gradient_clear(cuda, variant):
    """The update kernel zeroes the gradient buffer it consumed: in place (zero is grad itself, the
    1-GPU / fp32-wire case: every element read before its zero lands) and a separate bf16 buffer
    (the DP bf16 case: the kernel reads the fp32 wire buffer); the update itself is unchanged.
    Both kernel variants (MXR_SGD=0 4-wide, 2 = 8-wide nontemporal; n not a multiple of 8)."""
    import subprocess
    import sys
    code = """
import torch
from mx_rcnn_amd import ops
g = torch.Generator().manual_seed(3)
n = 100003
w = torch.randn(n, generator=g).cuda(); m = (torch.randn(n, generator=g) * 0.01).cuda()
gr = (torch.randn(n, generator=g) * 2).cuda(); lr = torch.tensor([0.01]).cuda()
w0, m0 = w.clone(), m.clone()
ops.sgd_momentum_(w0, m0, gr.clone(), lr, 0.9, 5e-4, 1.0, 1.0)
g1 = gr.clone()
ops.sgd_momentum_(w, m, g1, lr, 0.9, 5e-4, 1.0, 1.0, zero=g1)
assert torch.equal(w, w0) and torch.equal(m, m0), 'update changed'
assert not g1.any(), 'fp32 in-place clear'
w2, m2 = w0.clone(), m0.clone(); w3, m3 = w0.clone(), m0.clone()
gb = torch.randn(n, generator=g).cuda().bfloat16()
ops.sgd_momentum_(w3, m3, gr, lr, 0.9, 5e-4, 1.0, 1.0)
ops.sgd_momentum_(w2, m2, gr, lr, 0.9, 5e-4, 1.0, 1.0, zero=gb)
assert torch.equal(w2, w3) and not gb.any(), 'bf16 side clear'
print('ok')
"""
    env = dict(__import__('os').environ, MXR_SGD=variant)
    r = subprocess.run([sys.executable, '-c', code], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=200, cwd=__import__('os').path.dirname(__import__('os').path.dirname(
                           __import__('os').path.abspath(__file__))))
    assert r.returncode == 0 and 'ok' in r.stdout, r.stdout[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [
    # N, Cin, H, W, Cout, k, s, p, bias, relu
    (1, 64, 23, 37, 64, 3, 1, 1, False, False),
    (2, 128, 13, 9, 192, 3, 1, 1, True, True),
    (1, 256, 50, 84, 256, 3, 1, 1, False, False),
    (1, 128, 31, 40, 128, 3, 2, 1, False, False),
    (3, 512, 7, 7, 512, 3, 2, 1, False, False),
    (1, 64, 20, 30, 96, 5, 1, 2, True, False),
])
def test_conv_igemm_fwd_vs_fp32(cuda, shape):
    from mx_rcnn_amd.ops import need_ext
    N, Cin, H, W, Cout, k, s, p, bias, relu = shape
    g = torch.Generator().manual_seed(8)
    x = torch.randn(N, Cin, H, W, generator=g).bfloat16()
    w = (torch.randn(Cout, Cin, k, k, generator=g) * 0.05).bfloat16()
    b = torch.randn(Cout, generator=g) if bias else None
    ref = F.conv2d(x.float(), w.float(), b, stride=s, padding=p)
    if relu:
        ref = torch.relu(ref)
    for tile, splits in ((1, 1), (2, 1), (3, 1), (3, 2), (3, 4), (0, 0), (21, 1), (22, 1), (23, 1), (23, 2), (31, 2),
                         (33, 1), (12, 1), (16, 2), (24, 1), (25, 1), (24, 2)) + \
            tuple((100 + i, 1) for i in range(12)) + ((105, 2), (106, 4), (200, 1), (201, 1)):
        y = need_ext().conv_igemm_fwd(x.to(cuda).contiguous(memory_format=torch.channels_last),
                                      w.to(cuda).contiguous(memory_format=torch.channels_last),
                                      None if b is None else b.to(cuda), s, p, relu, tile, splits)[0]
        err = (y.float().cpu() - ref).abs().max().item()
        scale = ref.abs().max().item()
        assert err <= 1e-2 * scale + 1e-2, (tile, splits, err, scale)


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('tile', [200, 201, 202, 203, 204, 205, 206, 207])
def test_conv_big_epilogue_vs_fp32(cuda, dtype, tile):
    """The large-tile kernel (conv_big.hip: every tile shape and ring depth) with its full epilogue --
    bias, residual, ReLU and the frozen BN + ReLU second output -- against the fp32 reference of the
    same 16-bit operands; M = 2 * 37 * 53 (not a multiple of 256) and Cout = 320 (a partial column tile)."""
    from mx_rcnn_amd.ops import need_ext
    g = torch.Generator().manual_seed(21)
    N, Cin, H, W, Cout = 2, 128, 37, 53, 320
    x = torch.randn(N, Cin, H, W, generator=g).to(dtype)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.05).to(dtype)
    b = torch.randn(Cout, generator=g)
    res = torch.randn(N, Cout, H, W, generator=g).to(dtype)
    gamma, beta = torch.rand(Cout, generator=g) + 0.5, torch.randn(Cout, generator=g)
    mean, var = torch.randn(Cout, generator=g), torch.rand(Cout, generator=g) + 0.5
    ref = torch.relu(F.conv2d(x.float(), w.float(), b, padding=1) + res.float())
    cl = dict(memory_format=torch.channels_last)
    y1, y2 = need_ext().conv_igemm_fwd(x.to(cuda).contiguous(**cl), w.to(cuda).contiguous(**cl), b.to(cuda), 1, 1,
                                       True, tile, 1, res.to(cuda).contiguous(**cl),
                                       [t.to(cuda) for t in (gamma, beta, mean, var)], 2e-5, False, True)
    scale = ref.abs().max().item()
    assert (y1.float().cpu() - ref).abs().max().item() <= 1e-2 * scale
    # the BN reads the STORED 16-bit output
    ys = y1.float().cpu()
    ref2 = torch.relu((ys - mean[:, None, None]) / torch.sqrt(var[:, None, None] + 2e-5) * gamma[:, None, None] +
                      beta[:, None, None])
    assert (y2.float().cpu() - ref2).abs().max().item() <= 1e-2 * ref2.abs().max().item()


@pytest.mark.gpu
def test_conv_igemm_autograd(cuda):
    from mx_rcnn_amd.ops.conv import conv2d
    g = torch.Generator().manual_seed(9)
    x = torch.randn(1, 128, 21, 33, generator=g).bfloat16()
    w = (torch.randn(192, 128, 3, 3, generator=g) * 0.05).bfloat16()
    b = torch.randn(192, generator=g)
    xr, wr, br = [t.float().clone().requires_grad_() for t in (x, w, b)]
    yr = torch.relu(F.conv2d(xr, wr, br, padding=1))
    dy = torch.randn(yr.shape, generator=g).bfloat16()
    yr.backward(dy.float())
    xg = x.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    wg = w.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    bg = b.to(cuda).requires_grad_()
    yg = conv2d(xg, wg, bg, 1, 1, relu=True)
    yg.backward(dy.to(cuda).contiguous(memory_format=torch.channels_last))
    for a, r in [(yg, yr), (xg.grad, xr.grad), (wg.grad, wr.grad), (bg.grad, br.grad)]:
        err = (a.float().cpu() - r.detach()).abs().max().item()
        assert err <= 2e-2 * r.abs().max().item() + 2e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [
    # N, Cin, H, W, Cout, k, s, p
    (1, 64, 23, 37, 64, 3, 1, 1),
    (1, 256, 50, 84, 256, 3, 1, 1),
    (2, 128, 13, 9, 192, 3, 2, 1),
    (1, 1024, 50, 84, 512, 3, 1, 1),
    (1, 128, 20, 30, 64, 1, 1, 0),
    (8, 512, 7, 7, 512, 3, 1, 1),
])
def test_conv_wgrad_vs_fp32(cuda, shape):
    from mx_rcnn_amd.ops import need_ext
    N, Cin, H, W, Cout, k, s, p = shape
    g = torch.Generator().manual_seed(10)
    x = torch.randn(N, Cin, H, W, generator=g).bfloat16()
    w = torch.zeros(Cout, Cin, k, k)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(N, Cout, Ho, Wo, generator=g).bfloat16()
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                              [False, True, False])[1]
    dyc = dy.to(cuda).contiguous(memory_format=torch.channels_last)
    xc = x.to(cuda).contiguous(memory_format=torch.channels_last)
    tol = 1e-2 * ref.abs().max().item() + 1e-2
    for variant in (0, 1):  # 0: LDS-DMA kernel (default), 1: register-staged kernel
        for splits in (1, 0, 3):
            dw = need_ext().conv_wgrad(dyc, xc, k, k, s, p, splits, variant=variant)
            err = (dw.float().cpu() - ref).abs().max().item()
            assert err <= tol, (variant, splits, err)
        # accumulate into an existing gradient (flat-buffer delivery), direct and split paths
        for splits in (1, 2):
            base = (torch.randn(ref.shape, generator=g) * ref.abs().max()).bfloat16()
            out = base.to(cuda).contiguous(memory_format=torch.channels_last)
            need_ext().conv_wgrad(dyc, xc, k, k, s, p, splits, out, variant=variant)
            err = (out.float().cpu() - (ref + base.float())).abs().max().item()
            assert err <= 2 * tol, ('acc', variant, splits, err)


@pytest.mark.gpu
def test_direct_grad_delivery(cuda):
    """Kernels that accumulate straight into a FlatParamStore-style preset .grad view must
    produce the same gradient as the autograd path, and fire the readiness hook once."""
    from mx_rcnn_amd.ops import grad_sink
    from mx_rcnn_amd.ops.conv import conv2d
    g = torch.Generator().manual_seed(11)
    x = torch.randn(1, 128, 21, 33, generator=g).bfloat16().to(cuda).contiguous(memory_format=torch.channels_last)
    w0 = (torch.randn(128, 128, 3, 3, generator=g) * 0.05).bfloat16().to(cuda).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(1, 128, 21, 33, generator=g).bfloat16().to(cuda).contiguous(memory_format=torch.channels_last)
    # reference: plain autograd result
    wr = w0.clone().requires_grad_()
    conv2d(x, wr, None, 1, 1).backward(dy)
    # managed param: grad preset to a view of a flat buffer, direct delivery enabled
    flat = torch.zeros(w0.numel(), dtype=torch.bfloat16, device=cuda)
    wm = torch.nn.Parameter(w0.clone())
    wm.grad = flat.view(128, 3, 3, 128).permute(0, 3, 1, 2)
    grad_sink.enable_direct(wm)
    fired = []
    grad_sink.add_hook(wm, lambda p: fired.append(1))
    conv2d(x, wm, None, 1, 1).backward(dy)
    torch.cuda.synchronize()
    assert len(fired) == 1
    assert torch.allclose(wm.grad.float(), wr.grad.float(), atol=1e-2, rtol=1e-2)
    # BN gamma/beta
    C = 256
    xb = torch.randn(1, C, 9, 13, generator=g).bfloat16().to(cuda).contiguous(memory_format=torch.channels_last)
    mean, var = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    gr, br = torch.ones(C, device=cuda, requires_grad=True), torch.zeros(C, device=cuda, requires_grad=True)
    ops.frozen_bn_relu(xb, gr, br, mean, var).float().sum().backward()
    fb = torch.zeros(2 * C, device=cuda)
    gm, bm = torch.nn.Parameter(torch.ones(C, device=cuda)), torch.nn.Parameter(torch.zeros(C, device=cuda))
    gm.grad, bm.grad = fb[:C], fb[C:]
    grad_sink.enable_direct(gm)
    grad_sink.enable_direct(bm)
    ops.frozen_bn_relu(xb, gm, bm, mean, var).float().sum().backward()
    assert torch.allclose(gm.grad, gr.grad, atol=1e-2, rtol=1e-3)
    assert torch.allclose(bm.grad, br.grad, atol=1e-2, rtol=1e-3)


@pytest.mark.gpu
def test_loss_grid_reduction_meta_and_combine(cuda):
    """Losses finalise in-kernel (last-block reduction, ticket re-armed per launch): repeated
    many-block launches, the anchor-sampler count as normaliser, the backward scale, and the
    one-launch loss/objective/non-finite combine."""
    from mx_rcnn_amd.ops.losses import combine_losses
    g = torch.Generator().manual_seed(5)
    B, A, H, W = 2, 12, 50, 84
    lc = torch.randn(B, 2 * A, H, W, generator=g)
    label = torch.randint(-1, 2, (B, A * H * W), generator=g, dtype=torch.int32)
    meta = torch.zeros(B, 4, dtype=torch.int32)
    meta[:, 2] = (label == 1).sum(1)
    meta[:, 3] = (label == 0).sum(1)
    lcr = lc.clone().requires_grad_()
    ref = ops.rpn_softmax_ce(lcr, label)
    ref.backward(torch.tensor(2.0))
    for _ in range(3):
        for m in (None, meta.to(cuda)):
            lg = lc.to(cuda).requires_grad_()
            out = ops.rpn_softmax_ce(lg, label.to(cuda), sample_meta=m)
            out.backward(torch.tensor(2.0, device=cuda))
            assert abs(out.item() - ref.item()) <= 1e-4 * abs(ref.item()) + 1e-5
            assert torch.allclose(lg.grad.cpu(), lcr.grad, atol=1e-6, rtol=1e-3)
    pred = torch.randn(B, 4 * A, H, W, generator=g)
    tgt, iw, ow = torch.randn_like(pred), (torch.rand_like(pred) > 0.5).float(), torch.rand_like(pred)
    s_ref = ops.smooth_l1(pred, tgt, iw, ow, 3.0, 1.0)
    for _ in range(3):
        s = ops.smooth_l1(pred.to(cuda), tgt.to(cuda), iw.to(cuda), ow.to(cuda), 3.0, 1.0, slot=5)
        assert abs(s.item() - s_ref.item()) <= 1e-4 * abs(s_ref.item()) + 1e-4
    nf = torch.zeros((), dtype=torch.int32, device=cuda)
    a = torch.tensor(1.5, device=cuda, requires_grad=True)
    b = torch.tensor(4.0, device=cuda, requires_grad=True)
    tot, obj = combine_losses([a, b], [1.0, 0.25], nf)
    tot.backward()
    assert tot.item() == 5.5 and obj.item() == 2.5 and int(nf) == 0
    assert a.grad.item() == 1.0 and b.grad.item() == 1.0
    combine_losses([a, torch.tensor(float('nan'), device=cuda)], [1.0, 1.0], nf)
    assert int(nf) == 1


def test_roi_pool_cpu_twin_matches_reference():
    """C++ CPU RoI max-pool == the loop reference (ties -> first max in row-major order, empty
    bins, RoIs outside the map and an out-of-range batch index)."""
    from mx_rcnn_amd.ops import ext_available, need_ext
    if not ext_available():
        pytest.skip('extension not built')
    g = torch.Generator().manual_seed(3)
    feat = torch.randn(2, 5, 23, 31, generator=g)
    feat[0, :, 3:8, 4:9] = 1.5  # plateau: tie-breaking
    rois = torch.tensor([[0, 10, 20, 200, 150], [1, 0, 0, 15, 15], [0, 300, 300, 900, 900],
                         [1, -40, -40, 40, 40], [5, 0, 0, 100, 100], [0, 64, 48, 64.4, 48.6]])
    for ph, pw, sc in [(7, 7, 1.0 / 16), (3, 5, 0.125), (14, 14, 0.0625)]:
        ref_o, ref_a = roi_pool_ref(feat, rois, ph, pw, sc)
        o, a = need_ext().roi_pool_fwd_cpu(feat, rois, ph, pw, sc)
        assert torch.equal(a, ref_a), (ph, pw, sc)
        assert torch.equal(o, ref_o), (ph, pw, sc)


def test_roi_pool_bwd_cpu_twin_matches_scatter():
    from mx_rcnn_amd.ops import ext_available, need_ext
    if not ext_available():
        pytest.skip('extension not built')
    g = torch.Generator().manual_seed(9)
    feat = torch.randn(2, 16, 30, 40, generator=g)
    rois = _rois(g, 64, 2, 30, 40)
    rois[3, 0] = -1
    _, arg = roi_pool_ref(feat, rois, 7, 7, 1 / 16)
    gout = torch.randn(64, 16, 7, 7, generator=g)
    ref = torch.zeros(2, 16 * 30 * 40, dtype=torch.float64)
    for r in range(64):
        b = int(rois[r, 0])
        if b < 0:
            continue
        a = arg[r].reshape(16, -1).long()
        m = a >= 0
        ref[b].index_add_(0, (torch.arange(16)[:, None] * 1200 + a.clamp_min(0))[m], gout[r].reshape(16, -1)[m].double())
    gin = need_ext().roi_pool_bwd_cpu(gout, arg, rois, 2, 30, 40)
    assert torch.allclose(gin.double(), ref.reshape(2, 16, 30, 40), atol=1e-5)
    assert torch.equal(gin, need_ext().roi_pool_bwd_cpu(gout, arg, rois, 2, 30, 40))


@pytest.mark.parametrize('which', ['rpn_ce', 'smooth_l1', 'row_ce'])
def test_loss_cpu_twins_match_tensor_path(which, monkeypatch):
    """C++ loss twins (host_ops.h) vs the tensor path (ext disabled): value and autograd grad."""
    from mx_rcnn_amd.ops import ext_available
    from mx_rcnn_amd.ops import losses as L
    if not ext_available():
        pytest.skip('extension not built')
    g = torch.Generator().manual_seed(12)
    if which == 'rpn_ce':
        x = torch.randn(2, 18, 7, 9, generator=g) * 3
        lab = torch.randint(-1, 2, (2, 9 * 7 * 9), generator=g).to(torch.int32)
        fn = lambda t: L.rpn_softmax_ce(t, lab, grad_scale=1.0)  # noqa: E731
    elif which == 'row_ce':
        x = torch.randn(300, 21, generator=g) * 4
        lab = torch.randint(-1, 21, (300,), generator=g).to(torch.int32)
        fn = lambda t: L.softmax_ce(t, lab, 'batch', grad_scale=1.0)[0]  # noqa: E731
    else:
        x = torch.randn(64, 84, generator=g)
        tgt = torch.randn(64, 84, generator=g)
        iw = (torch.rand(64, 84, generator=g) > 0.5).float()
        ow = iw / 64
        fn = lambda t: L.smooth_l1(t, tgt, iw, ow, sigma=3.0, grad_scale=0.5)  # noqa: E731
    outs = []
    for use_ext in (True, False):
        if not use_ext:
            monkeypatch.setattr(L, 'ext_available', lambda: False)
        xi = x.clone().requires_grad_()
        v = fn(xi)
        (v * 1.5).backward()
        outs.append((v.detach(), xi.grad))
    (v1, g1), (v2, g2) = outs
    assert torch.allclose(v1, v2, rtol=1e-5, atol=1e-6), (v1, v2)
    assert torch.allclose(g1, g2, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize('clip', [-1.0, 0.05])
def test_sgd_cpu_twin_matches_tensor_path(clip, monkeypatch):
    from mx_rcnn_amd.ops import ext_available
    from mx_rcnn_amd.ops import sgd as S
    if not ext_available():
        pytest.skip('extension not built')
    g = torch.Generator().manual_seed(31)
    n = 300001  # not a multiple of the parallel grain
    w0, m0, gr = (torch.randn(n, generator=g) for _ in range(3))
    lr = torch.tensor([0.01])
    res = []
    for use_ext in (True, False):
        if not use_ext:
            monkeypatch.setattr(S, 'ext_available', lambda: False)
        w, m = w0.clone(), m0.clone()
        wb = torch.empty(n, dtype=torch.bfloat16)
        S.sgd_momentum_(w, m, gr, lr, momentum=0.9, wd=5e-4, rescale=0.5, clip=clip, w_bf16=wb)
        res.append((w, m, wb))
    for a, b in zip(*res):
        assert torch.allclose(a.float(), b.float(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('channels_last,fix_gamma,relu', [(False, False, True), (True, True, False)])
def test_bn_relu_cpu_twin_matches_tensor_path(channels_last, fix_gamma, relu, monkeypatch):
    from mx_rcnn_amd.ops import ext_available
    from mx_rcnn_amd.ops import bn as BN
    if not ext_available():
        pytest.skip('extension not built')
    g = torch.Generator().manual_seed(43)
    x = torch.randn(2, 24, 9, 11, generator=g)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    gamma, beta, mean = (torch.randn(24, generator=g) for _ in range(3))
    var = torch.rand(24, generator=g) + 0.1
    outs = []
    for use_ext in (True, False):
        if not use_ext:
            monkeypatch.setattr(BN, 'ext_available', lambda: False)
        xi, gi, bi = x.clone().requires_grad_(), gamma.clone().requires_grad_(), beta.clone().requires_grad_()
        y = BN._FrozenBnRelu.apply(xi, gi, bi, mean, var, 2e-5, fix_gamma, relu)
        (y * torch.linspace(-1, 1, y.numel()).reshape(y.shape)).sum().backward()
        outs.append((y.detach(), xi.grad, bi.grad))
        assert y.is_contiguous(memory_format=torch.channels_last) == channels_last
    for a, b in zip(*outs):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_conv_autotune_picks_a_candidate_and_matches(cuda, monkeypatch):
    """The per-shape autotune (first eager call) caches a tile choice; its output is the
    chosen tile's own output, and equals the static plan's bitwise unless the choice sums K in a
    different order (the K-group tiles 27-29, split-K), then to bf16 rounding."""
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(1, 256, 38, 61, generator=g).bfloat16().to(cuda).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(256, 256, 3, 3, generator=g) * 0.05).bfloat16().to(cuda).contiguous(
        memory_format=torch.channels_last)
    y_tuned = ext.conv_igemm_fwd(x, w, None, 1, 1, False)[0]
    hits = [(k, t, s) for k, t, s in ext.conv_tune_table() if k.startswith('1,38,61,256,256,3,3,1,1|')]
    assert len(hits) == 1
    _, tile, splits = hits[0]
    assert torch.equal(y_tuned, ext.conv_igemm_fwd(x, w, None, 1, 1, False, tile, splits)[0])
    y_plan = ext.conv_igemm_fwd(x, w, None, 1, 1, False, 23, 1)[0]
    if tile in (27, 28, 29) or splits > 1:
        assert torch.allclose(y_tuned.float(), y_plan.float(), rtol=1e-2, atol=1e-2)
    else:
        assert torch.equal(y_tuned, y_plan)


def test_philox_host_twin_statistics():
    """The counter-based dropout generator: deterministic, uniform, distinct per step and seed."""
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    u = ext.philox_uniform(7, 3, 1 << 16)
    assert torch.equal(u, ext.philox_uniform(7, 3, 1 << 16))
    assert 0.0 <= u.min().item() and u.max().item() < 1.0
    assert abs(u.mean().item() - 0.5) < 0.01 and abs((u < 0.5).float().mean().item() - 0.5) < 0.01
    assert (u != ext.philox_uniform(7, 4, 1 << 16)).float().mean() > 0.99
    assert (u != ext.philox_uniform(8, 3, 1 << 16)).float().mean() > 0.99


@pytest.mark.gpu
@pytest.mark.parametrize('M,K,N,relu,drop', [(128, 25088, 4096, True, 0.5), (128, 4096, 4096, True, 0.5),
                                             (128, 4096, 21, False, 0.0), (300, 2048, 324, False, 0.0),
                                             (96, 512, 256, True, 0.0)])
def test_fc_fused_vs_fp32(cuda, M, K, N, relu, drop):
    """FullyConnected on the MFMA kernel (+bias, ReLU, Philox dropout) and its backward vs fp32 torch
    with the same mask (host twin of the generator)."""
    from mx_rcnn_amd.ops import need_ext
    from mx_rcnn_amd.ops.fc import _FC
    g = torch.Generator().manual_seed(5)
    x = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, generator=g).bfloat16()
    step = torch.tensor([11], dtype=torch.int64, device=cuda)
    xg = x.to(cuda).requires_grad_(True)
    wg = w.to(cuda).requires_grad_(True)
    bg = b.to(cuda).requires_grad_(True)
    y = _FC.apply(xg, wg, bg, relu, drop, 1234, step)
    ref = x.float() @ w.float().t() + b.float()
    if relu:
        ref = torch.relu(ref)
    mask = torch.ones(M, N)
    if drop > 0:
        mask = (need_ext().philox_uniform(1234, 11, M * N).view(M, N) >= drop).float() / (1 - drop)
    ref = ref * mask
    err = (y.float().cpu() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 2e-2, err
    dy = torch.randn(M, N, generator=g).bfloat16()
    y.backward(dy.to(cuda))
    xr, wr, br = x.float().requires_grad_(True), w.float().requires_grad_(True), b.float().requires_grad_(True)
    r = xr @ wr.t() + br
    if relu:
        r = torch.relu(r)
    (r * mask).backward(dy.float())
    for got, want in ((xg.grad, xr.grad), (wg.grad, wr.grad), (bg.grad, br.grad)):
        e = (got.float().cpu() - want).abs().max().item()
        assert e <= 3e-2 * want.abs().max().item() + 3e-2, (e, want.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize('N,C,H,W,k,s,p', [(1, 64, 61, 97, 2, 2, 0), (1, 512, 75, 125, 2, 2, 0),
                                           (1, 64, 400, 667, 3, 2, 1), (2, 16, 9, 14, 3, 2, 1)])
def test_maxpool_vs_torch(cuda, N, C, H, W, k, s, p):
    from mx_rcnn_amd.ops.pool import max_pool2d
    g = torch.Generator().manual_seed(6)
    x = torch.randn(N, C, H, W, generator=g).bfloat16()
    xg = x.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = max_pool2d(xg, k, s, p)
    xr = x.float().requires_grad_(True)
    ref = F.max_pool2d(xr, k, s, p)
    assert torch.equal(y.float().cpu(), ref.detach())
    dy = torch.randn(ref.shape, generator=g).bfloat16()
    y.backward(dy.to(cuda).contiguous(memory_format=torch.channels_last))
    ref.backward(dy.float())
    assert (xg.grad.float().cpu() - xr.grad).abs().max().item() <= 2e-2 * xr.grad.abs().max().item()


def _post_bn(g, C, cuda, fix_gamma):
    """Frozen-BN params with both signs of gamma (a negative scale flips which input is largest)."""
    gamma = torch.randn(C, generator=g)
    beta = torch.randn(C, generator=g) * 0.5
    mean = torch.randn(C, generator=g) * 0.3
    var = torch.rand(C, generator=g) + 0.2
    return [t.to(cuda).contiguous() for t in (gamma, beta, mean, var)], 2e-5, fix_gamma


def _bn_relu_ref(y, prm, eps, fix):
    gamma, beta, mean, var = [t.cpu().double() for t in prm]
    s = (torch.ones_like(gamma) if fix else gamma) / torch.sqrt(var + eps)
    return torch.relu(y.double() * s[None, :, None, None] + (beta - mean * s)[None, :, None, None])


@pytest.mark.gpu
@pytest.mark.parametrize('dtype,C,fix', [(torch.bfloat16, 1024, False), (torch.float16, 256, True),
                                         (torch.float32, 64, False), (torch.float32, 6, False)])
def test_roi_pool_post_bn_matches_pool_then_bn(cuda, dtype, C, fix):
    """roi_pool_fwd(post_bn=...) == bn_relu_fwd(roi_pool_fwd(...)) bit for bit on 16-bit maps (the
    inference fusion of stage4_unit1_bn1 into the pooling store); fp32 / odd C vs a float64 reference."""
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(11)
    B, H, W = 2, 38, 50
    feat = torch.randn(B, C, H, W, generator=g).to(cuda, dtype).contiguous(memory_format=torch.channels_last)
    rois = _rois(g, 64, B, H, W).to(cuda)
    rois[3, 0] = -1  # empty output rows: relu(bn(0))
    prm, eps, fix = _post_bn(g, C, cuda, fix)
    aff = ext.bn_affine(*prm, eps, fix)
    gm = torch.ones(C) if fix else prm[0].cpu()
    s_ref = gm / torch.sqrt(prm[3].cpu() + eps)
    assert torch.allclose(aff[0].cpu(), s_ref, rtol=1e-6) and torch.allclose(
        aff[1].cpu(), prm[1].cpu() - prm[2].cpu() * s_ref, rtol=1e-5, atol=1e-6)
    got, arg = ext.roi_pool_fwd(feat, rois, 7, 7, 1 / 16, 0, False, aff)
    assert arg.numel() == 0 and got.is_contiguous(memory_format=torch.channels_last)
    pooled = ext.roi_pool_fwd(feat, rois, 7, 7, 1 / 16, 0, False)[0]
    if dtype != torch.float32:
        want = ext.bn_relu_fwd(pooled, *prm, eps, fix, True, 0)
        assert torch.equal(got, want), (got.float() - want.float()).abs().max().item()
    want = _bn_relu_ref(pooled.float().cpu(), prm, eps, fix)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert torch.allclose(got.double().cpu(), want, atol=tol, rtol=tol)
    with pytest.raises(RuntimeError, match='inference-only'):
        ext.roi_pool_fwd(feat, rois, 7, 7, 1 / 16, 0, True, aff)


@pytest.mark.gpu
@pytest.mark.parametrize('dtype,fix', [(torch.bfloat16, False), (torch.float16, True)])
def test_maxpool_post_bn_matches_pool_then_bn(cuda, dtype, fix):
    """maxpool_fwd(need_arg=False, post_bn=...) == bn_relu_fwd(maxpool_fwd(...)) bit for bit (ResNet
    pool0 -> stage1_unit1_bn1 at inference), and no tap map is written."""
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(12)
    x = torch.randn(2, 64, 41, 53, generator=g).to(cuda, dtype).contiguous(memory_format=torch.channels_last)
    prm, eps, fix = _post_bn(g, 64, cuda, fix)
    aff = ext.bn_affine(*prm, eps, fix)
    got, arg = ext.maxpool_fwd(x, 3, 2, 1, 0, False, aff)
    assert arg.numel() == 0
    want = ext.bn_relu_fwd(ext.maxpool_fwd(x, 3, 2, 1, 0)[0], *prm, eps, fix, True, 0)
    assert torch.equal(got, want), (got.float() - want.float()).abs().max().item()
    ref = _bn_relu_ref(F.max_pool2d(x.float().cpu(), 3, 2, 1), prm, eps, fix)
    assert torch.allclose(got.double().cpu(), ref, atol=1e-2, rtol=1e-2)
    with pytest.raises(RuntimeError, match='inference-only'):
        ext.maxpool_fwd(x, 3, 2, 1, 0, True, aff)


@pytest.mark.gpu
def test_global_avgpool_vs_torch(cuda):
    from mx_rcnn_amd.ops.pool import global_avg_pool
    g = torch.Generator().manual_seed(7)
    x = torch.randn(128, 2048, 4, 4, generator=g).bfloat16()
    xg = x.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = global_avg_pool(xg)
    xr = x.float().requires_grad_(True)
    ref = xr.mean(dim=(2, 3))
    assert (y.float().cpu() - ref.detach()).abs().max().item() <= 1e-2
    dy = torch.randn(128, 2048, generator=g).bfloat16()
    y.backward(dy.to(cuda))
    ref.backward(dy.float())
    assert (xg.grad.float().cpu() - xr.grad).abs().max().item() <= 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize('M,K,N1,N2,relu_mask', [(128, 2048, 81, 324, False), (128, 4096, 21, 84, False),
                                                (4200, 512, 24, 48, True), (333, 256, 18, 36, True)])
def test_head_pair_bwd_vs_fp32(cuda, M, K, N1, N2, relu_mask):
    """csrc/hip/head_bwd.hip: dX (ReLU-masked), both dW (accumulated) and db (fp32 / bf16 targets,
    accumulated) of a head pair vs fp32 torch; row-split (rs > 1) and single-pass shapes."""
    from mx_rcnn_amd.ops import need_ext
    g = torch.Generator(device='cpu').manual_seed(3)
    x = torch.randn(M, K, generator=g)
    if relu_mask:
        x = x.clamp(min=0)  # a ReLU output: the mask is x > 0
    dys = [torch.randn(M, n, generator=g) for n in (N1, N2)]
    ws = [torch.randn(n, K, generator=g) * 0.05 for n in (N1, N2)]
    xb, dyb, wb = x.bfloat16(), [d.bfloat16() for d in dys], [w.bfloat16() for w in ws]
    xf, dyf, wf = xb.float(), [d.float() for d in dyb], [w.float() for w in wb]
    dw0 = [torch.randn(n, K, generator=g).bfloat16() for n in (N1, N2)]
    db0 = [torch.randn(N1, generator=g), torch.randn(N2, generator=g).bfloat16()]
    dws = [d.clone().to(cuda) for d in dw0]
    dbs = [d.clone().to(cuda) for d in db0]
    dx = need_ext().head_bwd(xb.to(cuda), [d.to(cuda) for d in dyb], [w.to(cuda) for w in wb], dws, [True, True],
                             dbs, [True, True], True, relu_mask)
    ref_dx = dyf[0] @ wf[0] + dyf[1] @ wf[1]
    if relu_mask:
        ref_dx = ref_dx * (xf > 0)
    assert torch.allclose(dx.float().cpu(), ref_dx, rtol=2e-2, atol=2e-2 * ref_dx.abs().max().item())
    for h in range(2):
        ref_dw = dw0[h].float() + dyf[h].t() @ xf
        got = dws[h].float().cpu()
        assert torch.allclose(got, ref_dw, rtol=2e-2, atol=1e-2 * ref_dw.abs().max().item()), h
        ref_db = db0[h].float() + dyf[h].sum(0)
        assert torch.allclose(dbs[h].float().cpu(), ref_db, rtol=1e-2, atol=1e-2 * ref_db.abs().max().item()), h


@pytest.mark.gpu
@pytest.mark.parametrize('N,C,H,W', [(1, 512, 50, 84), (2, 24, 7, 9), (128, 1024, 1, 1)])
def test_chan_sum_vs_torch(cuda, N, C, H, W):
    from mx_rcnn_amd.ops import need_ext
    x = torch.randn(N, C, H, W).bfloat16().contiguous(memory_format=torch.channels_last)
    ref = x.float().sum((0, 2, 3))
    out = torch.zeros(C, device=cuda)
    need_ext().chan_sum(x.to(cuda), out, False)
    assert torch.allclose(out.cpu(), ref, rtol=1e-4, atol=1e-3)
    acc = torch.ones(C, device=cuda).bfloat16()
    need_ext().chan_sum(x.to(cuda), acc, True)
    assert torch.allclose(acc.float().cpu(), ref + 1, rtol=1e-2, atol=1e-2 * (ref.abs().max().item() + 1))


@pytest.mark.gpu
@pytest.mark.parametrize('network', ['resnet', 'vgg'])
def test_head_pair_ops_match_modules(cuda, network):
    """ops/head.py: the fused RPN head / FC pair (forward + one-kernel backward) against the same
    modules run separately (MXR_HEAD_KERNEL path off), gradients of every input and parameter."""
    import copy
    import os
    from mx_rcnn_amd.models.faster_rcnn import RPNHead
    from mx_rcnn_amd.models.layers import Linear
    from mx_rcnn_amd.ops.head import fc_pair
    torch.manual_seed(0)
    if network == 'resnet':
        mod = RPNHead(1024, 12).to(cuda).bfloat16()
        for p in mod.parameters():
            p.data = p.data.contiguous(memory_format=torch.channels_last) if p.dim() == 4 else p.data
            p.data.normal_(0, 0.02)
        inp = torch.randn(1, 1024, 20, 31, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
        run = lambda m, x: m(x)  # noqa: E731
    else:
        mod = torch.nn.ModuleList([Linear('cls_score', 2048, 81), Linear('bbox_pred', 2048, 324)]).to(cuda).bfloat16()
        for p in mod.parameters():
            p.data.normal_(0, 0.02)
        inp = torch.randn(128, 2048, device=cuda).bfloat16()
        run = lambda m, x: fc_pair(x, m[0], m[1])  # noqa: E731
    ref_mod = copy.deepcopy(mod)
    outs = []
    for m, env in ((mod, '1'), (ref_mod, '0')):
        os.environ['MXR_HEAD_KERNEL'] = env
        try:
            x = inp.clone().requires_grad_(True)
            y1, y2 = run(m, x)
            g = torch.Generator(device='cpu').manual_seed(1)
            loss = (y1.float() * torch.randn(y1.shape, generator=g).to(cuda)).sum() + \
                (y2.float() * torch.randn(y2.shape, generator=g).to(cuda)).sum()
            loss.backward()
            outs.append([y1.float(), y2.float(), x.grad.float()] + [p.grad.float() for p in m.parameters()])
        finally:
            os.environ.pop('MXR_HEAD_KERNEL', None)
    for a, b in zip(*outs):
        scale = b.abs().max().item() + 1e-6
        assert (a - b).abs().max().item() <= 3e-2 * scale, (a.shape, (a - b).abs().max().item(), scale)
