"""Multi-plane fp32 kernels (ops/precision.py): every MFMA operand as bf16 planes with fp32
accumulation -- P = 3 (the fp32 mode: exact (mid, hi, lo) triples, six products) and P = 2 (bf16x3:
hi / lo pairs, 16 significant bits, three products).  Each kernel is checked against an fp64
PyTorch computation of the same op on the SAME fp32 inputs:
  * P = 3 to 2e-6 relative (to the output's max magnitude) -- or, for deep reductions, within 2x
    of what IEEE fp32 arithmetic itself achieves on the same op (torch's fp32 CPU result vs fp64);
  * P = 2 to 2e-5 relative (16-bit storage).

The CPU tests cover the plane helpers; the kernel tests run on the GPU.
"""
import pytest
import torch
import torch.nn.functional as F

from mx_rcnn_amd.ops import precision

TOL = 2e-5  # P = 2, relative (to the output's max magnitude)
TOLS = {2: 2e-5, 3: 2e-6}
PLANES = [2, 3]


def _err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-20))


def _tol(P, ref=None, f32=None):
    """P's tolerance; for P = 3 also at least 2x the error of the same op in IEEE fp32 (f32: the
    fp32 result computed by torch on the CPU, ref: the fp64 reference)."""
    t = TOLS[P]
    if P == 3 and f32 is not None:
        t = max(t, 2 * _err(f32, ref))
    return t


def test_split_join_roundtrip_cpu():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 8, 5, 7, generator=g) * 100
    p = precision.split(x, 2)
    assert p.dtype == torch.bfloat16 and p.shape == (6, 8, 5, 7)
    j = precision.join(p, 2)
    rel = ((j - x).abs() / x.abs().clamp_min(1e-30)).max()
    assert float(rel) <= 2.0 ** -16, float(rel)
    xc = x.contiguous(memory_format=torch.channels_last)
    pc = precision.split(xc, 2)
    assert pc.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(precision.join(pc, 2), j)


def test_split3_is_exact_cpu():
    """The fp32 mode's (mid, hi, lo) triple holds the fp32 value exactly, hi carries its sign --
    for |v| in [2^-100, bf16 max = 3.39e38]: above, hi = RNE(v) overflows to inf; below ~2^-110 the
    lo plane is subnormal (a training tensor never lives at either end)."""
    g = torch.Generator().manual_seed(1)
    x = torch.cat([torch.randn(4096, generator=g) * 10 ** torch.randint(-28, 28, (4096,), generator=g).float(),
                   torch.tensor([0.0, -0.0, 1.0, -1.0, 3.3e38, -1e-30, 1e-30, 65504.0, 1.1754944e-38 * 2 ** 26])])
    p = precision.split(x, 3)
    assert p.shape == (3 * x.numel(),)
    assert torch.equal(precision.join(p, 3), x)
    hi = precision.hi_plane(p, 3).float()
    assert torch.equal(torch.sign(hi), torch.sign(x))


def test_x2_mode_switch_cpu():
    assert not precision.x2_enabled()
    with precision.x2_mode(True):
        assert precision.x2_enabled() == 2
        assert precision.is_pair(torch.zeros(2, dtype=torch.bfloat16)) == 2
        assert not precision.is_pair(torch.zeros(2))
        with precision.x2_mode(3):
            assert precision.x2_enabled() == 3 and precision.x3_enabled()
        assert precision.x2_enabled() == 2
    assert not precision.x2_enabled()


def test_weight_pair_cache_cpu():
    w = torch.nn.Parameter(torch.randn(64, 32, 3, 3).contiguous(memory_format=torch.channels_last))
    hi, pl = precision.weight_pair(w)
    assert hi.shape == (64, 32, 3, 3) and pl == w.numel()
    assert hi.is_contiguous(memory_format=torch.channels_last)
    full = hi.reshape(-1)  # noqa: F841  (the hi view is a real tensor)
    with torch.no_grad():
        w.mul_(2)
    hi2, _ = precision.weight_pair(w)
    assert not torch.equal(hi.float(), hi2.float())  # rebuilt after the version bump


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last) if t.dim() == 4 else t.contiguous()


def _pair(t, dev, P=2):
    return _cl(precision.split(_cl(t.to(dev)), P))


def _unpair(p, P=2):
    return precision.join(p, P)


@pytest.mark.gpu
@pytest.mark.parametrize('P', PLANES)
@pytest.mark.parametrize('k,stride,pad,N,C,H,W,O', [
    (1, 1, 0, 1, 64, 20, 30, 128),     # 1x1
    (3, 1, 1, 1, 128, 17, 23, 64),     # 3x3 s1
    (3, 2, 1, 2, 64, 21, 19, 64),      # 3x3 s2
    (1, 1, 0, 1, 256, 6, 7, 64),       # small grid: split-K
])
def test_conv_fwd_x2_matches_fp32(cuda, P, k, stride, pad, N, C, H, W, O):
    from mx_rcnn_amd.ops import need_ext
    g = torch.Generator().manual_seed(k * 100 + C)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(O, C, k, k, generator=g) * (2.0 / (C * k * k)) ** 0.5
    b = torch.randn(O, generator=g)
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=stride, padding=pad)
    tol = _tol(P, ref, F.conv2d(x, w, b, stride=stride, padding=pad))
    wp = _pair(w, cuda, P)
    y = need_ext().conv_igemm_fwd(_pair(x, cuda, P), wp[:O], b.to(cuda), stride, pad, False, x2=P,
                                  w_plane=wp.numel() // P)[0]
    assert y.shape == (P * N, O, ref.shape[2], ref.shape[3])
    assert _err(_unpair(y, P), ref) <= tol
    # fp32 output (the prediction heads) and the frozen-BN + ReLU second output
    yf = need_ext().conv_igemm_fwd(_pair(x, cuda, P), wp[:O], b.to(cuda), stride, pad, False, x2=P,
                                   w_plane=wp.numel() // P, out_f32=True)[0]
    assert yf.dtype == torch.float32 and _err(yf, ref) <= tol
    gam, bet = torch.rand(O) + 0.5, torch.randn(O)
    mu, var = torch.randn(O), torch.rand(O) + 0.5
    bn = [t.to(cuda) for t in (gam, bet, mu, var)]
    res = torch.randn(ref.shape, generator=g)
    y1, y2 = need_ext().conv_igemm_fwd(_pair(x, cuda, P), wp[:O], None, stride, pad, False, 0, 0, _pair(res, cuda, P),
                                       bn, 2e-5, False, True, x2=P, w_plane=wp.numel() // P)
    r1 = ref - b.double().view(1, -1, 1, 1) + res.double()
    r2 = torch.relu((r1 - mu.double().view(1, -1, 1, 1)) / torch.sqrt(var.double().view(1, -1, 1, 1) + 2e-5)
                    * gam.double().view(1, -1, 1, 1) + bet.double().view(1, -1, 1, 1))
    assert _err(_unpair(y1, P), r1) <= tol
    assert _err(_unpair(y2, P), r2) <= 4 * tol


@pytest.mark.gpu
@pytest.mark.parametrize('P', PLANES)
def test_conv_dgrad_bt_x3_matches_fp32(cuda, P):
    """Stride-1 data gradient reading the forward filter transposed in-kernel (ConvEpi::bt)."""
    from mx_rcnn_amd.ops import need_ext
    g = torch.Generator().manual_seed(21)
    N, C, H, W, O = 1, 128, 19, 26, 256
    w = torch.randn(O, C, 3, 3, generator=g) * 0.03
    dy = torch.randn(N, O, H, W, generator=g)
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.double(), dy.double(), padding=1)
    f32 = torch.nn.grad.conv2d_input((N, C, H, W), w, dy, padding=1)
    wp = _pair(w, cuda, P)
    dx = need_ext().conv_igemm_fwd(_pair(dy, cuda, P), wp[:O], None, 1, 1, False, bt=True, x2=P,
                                   w_plane=wp.numel() // P)[0]
    assert _err(_unpair(dx, P), ref) <= _tol(P, ref, f32)


@pytest.mark.gpu
@pytest.mark.parametrize('P', PLANES)
@pytest.mark.parametrize('k,stride,pad', [(1, 1, 0), (3, 1, 1), (3, 2, 1)])
def test_conv_wgrad_x2_matches_fp32(cuda, P, k, stride, pad):
    from mx_rcnn_amd.ops import need_ext
    g = torch.Generator().manual_seed(7 + k + stride)
    N, C, H, W, O = 1, 64, 19, 26, 128
    x = torch.randn(N, C, H, W, generator=g)
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    dy = torch.randn(N, O, Ho, Wo, generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (O, C, k, k), dy.double(), stride=stride, padding=pad)
    tol = _tol(P, ref, torch.nn.grad.conv2d_weight(x, (O, C, k, k), dy, stride=stride, padding=pad))
    dw = need_ext().conv_wgrad(_pair(dy, cuda, P), _pair(x, cuda, P), k, k, stride, pad, x2=P)
    assert dw.dtype == torch.float32
    assert _err(dw, ref) <= tol
    acc = _cl(torch.ones(O, C, k, k, device=cuda))
    need_ext().conv_wgrad(_pair(dy, cuda, P), _pair(x, cuda, P), k, k, stride, pad, 0, acc, x2=P)
    assert _err(acc - 1, ref) <= tol


@pytest.mark.gpu
@pytest.mark.parametrize('P', PLANES)
def test_grouped_dgrad_wgrad_x2_matches_fp32(cuda, P):
    """The fused unit backward's grouped launch: dgrad with the frozen BN-ReLU backward epilogue
    plus the weight gradient of another conv reading the same dY."""
    from mx_rcnn_amd.ops import need_ext
    from mx_rcnn_amd.ops.conv import _flip_t
    g = torch.Generator().manual_seed(3)
    N, C, H, W, O = 1, 64, 14, 18, 128
    dy = torch.randn(N, O, H, W, generator=g)
    w = torch.randn(O, C, 3, 3, generator=g) * 0.05
    xbn = torch.randn(N, C, H, W, generator=g)  # the BN input (bnb_x)
    gam, bet, mu, var = torch.rand(C) + 0.5, torch.randn(C) * 0.1, torch.randn(C) * 0.1, torch.rand(C) + 0.5
    # reference: d(act) = conv_transpose(dy, w); g = d(act) * [bn(x) > 0]; d(x) = g * s
    dact = torch.nn.grad.conv2d_input((N, C, H, W), w.double(), dy.double(), padding=1)
    s = gam.double() / torch.sqrt(var.double() + 2e-5)
    pre = (xbn.double() - mu.double().view(1, -1, 1, 1)) * s.view(1, -1, 1, 1) + bet.double().view(1, -1, 1, 1)
    gm = dact * (pre > 0)
    ref_dx = gm * s.view(1, -1, 1, 1)
    ref_db = gm.sum((0, 2, 3))
    # the wgrad role: the same dy against an input of its conv (a 1x1 here)
    xin = torch.randn(N, 256, H, W, generator=g)
    ref_dw = torch.nn.grad.conv2d_weight(xin.double(), (O, 256, 1, 1), dy.double())
    tol = TOLS[P]
    wf = _pair(_flip_t(w), cuda, P)
    dgm = torch.zeros(C, device=cuda)
    dbt = torch.zeros(C, device=cuda)
    wg = _cl(torch.zeros(O, 256, 1, 1, device=cuda))
    bn = [t.to(cuda) for t in (gam, bet, mu, var)]
    out = need_ext().conv_dgrad_wgrad(_pair(dy, cuda, P), wf[:C], 1, None, bn, 2e-5, False, _pair(xbn, cuda, P), None,
                                      dgm, dbt, _pair(dy, cuda, P), _pair(xin, cuda, P), 1, 1, 1, 0, wg, x2=P,
                                      w_plane=wf.numel() // P)
    assert _err(_unpair(out[0], P), ref_dx) <= 4 * tol
    assert _err(dbt, ref_db) <= 4 * tol
    assert _err(wg, ref_dw) <= tol


@pytest.mark.gpu
@pytest.mark.parametrize('P', PLANES)
def test_elementwise_x2_kernels_match_fp32(cuda, P):
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 64, 17, 23, generator=g) * 3
    C = 64
    tol = TOLS[P]
    gam, bet, mu, var = torch.rand(C) + 0.5, torch.randn(C), torch.randn(C), torch.rand(C) + 0.5
    bn = [t.to(cuda) for t in (gam, bet, mu, var)]
    # frozen BN + ReLU
    y = ext.bn_relu_fwd(_pair(x, cuda, P), *bn, 2e-5, False, True, P)
    ref = torch.relu((x.double() - mu.double().view(1, -1, 1, 1)) / torch.sqrt(var.double().view(1, -1, 1, 1) + 2e-5)
                     * gam.double().view(1, -1, 1, 1) + bet.double().view(1, -1, 1, 1))
    assert _err(_unpair(y, P), ref) <= tol
    # max pool 3x3/2 pad 1 (values, winners) and its backward: exact (no arithmetic)
    ym, arg = ext.maxpool_fwd(_pair(x, cuda, P), 3, 2, 1, P)
    refm = F.max_pool2d(x.double(), 3, 2, 1)
    assert _err(_unpair(ym, P), refm) <= (0.0 if P == 3 else tol)
    dym = torch.randn(refm.shape, generator=g)
    xr = x.double().requires_grad_()
    F.max_pool2d(xr, 3, 2, 1).backward(dym.double())
    dxm = ext.maxpool_bwd(_pair(dym, cuda, P), arg, 17, 23, 3, 2, 1, P)
    assert _err(_unpair(dxm, P), xr.grad) <= tol
    # global average pool and its backward
    ya = ext.avgpool_fwd(_pair(x, cuda, P), P)
    assert _err(_unpair(ya, P), x.double().mean((2, 3))) <= tol
    dya = torch.randn(2, C, generator=g)
    dxa = ext.avgpool_bwd(_pair(dya, cuda, P).contiguous(), 17, 23, P)
    assert _err(_unpair(dxa, P), (dya.double() / (17 * 23)).view(2, C, 1, 1).expand(2, C, 17, 23)) <= tol
    # channel sum (conv bias gradient)
    out = torch.zeros(C, device=cuda)
    ext.chan_sum(_pair(x, cuda, P), out, False, P)
    assert _err(out, x.double().sum((0, 2, 3))) <= tol
    # ReLU (+ dropout scale) backward masked by the ReLU output's sign (its hi plane)
    yr = torch.relu(x)
    dyr = torch.randn(x.shape, generator=g)
    mr = ext.relu_mask_bwd(_pair(dyr, cuda, P), _pair(yr, cuda, P), 2.0, P)
    assert _err(_unpair(mr, P), dyr.double() * (yr > 0) * 2.0) <= tol


@pytest.mark.gpu
@pytest.mark.parametrize('P', PLANES)
def test_bn_train_x2_matches_fp32(cuda, P):
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(12)
    N, C, H, W = 16, 128, 7, 7
    tol = TOLS[P]
    x = torch.randn(N, C, H, W, generator=g) * 2 + 0.5
    gam, bet = torch.rand(C) + 0.5, torch.randn(C)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y, save = ext.bn_train_fwd(_pair(x, cuda, P), gam.to(cuda), bet.to(cuda), rm, rv, 0.9, 2e-5, False, True, P)
    xd = x.double().requires_grad_()
    mean = xd.mean((0, 2, 3), keepdim=True)
    var = ((xd - mean) ** 2).mean((0, 2, 3), keepdim=True)
    ref = torch.relu((xd - mean) / torch.sqrt(var + 2e-5) * gam.double().view(1, -1, 1, 1) + bet.double().view(1, -1, 1, 1))
    assert _err(_unpair(y, P), ref.detach()) <= 4 * tol
    dy = torch.randn(N, C, H, W, generator=g)
    ref.backward(dy.double())
    dx, dg, db = ext.bn_train_bwd(_pair(x, cuda, P), _pair(dy, cuda, P), gam.to(cuda), bet.to(cuda), save[0], save[1],
                                  False, True, True, None, None, P)
    assert _err(_unpair(dx, P), xd.grad) <= 8 * tol


@pytest.mark.gpu
@pytest.mark.parametrize('P', PLANES)
def test_roi_pool_x2_matches_fp32(cuda, P):
    from mx_rcnn_amd.ops import need_ext
    from mx_rcnn_amd.ops.roi_pool import roi_pool_ref
    ext = need_ext()
    g = torch.Generator().manual_seed(13)
    feat = torch.randn(1, 64, 30, 40, generator=g)
    R = 32
    xy = torch.rand(R, 2, generator=g) * 300
    wh = torch.rand(R, 2, generator=g) * 200 + 16
    rois = torch.cat([torch.zeros(R, 1), xy, xy + wh], 1)
    out, arg = ext.roi_pool_fwd(_pair(feat, cuda, P), rois.to(cuda), 7, 7, 1 / 16, P)
    ref, ref_arg = roi_pool_ref(feat, rois, 7, 7, 1 / 16)
    assert _err(_unpair(out, P), ref) <= (0.0 if P == 3 else TOL)
    gout = torch.randn(R, 64, 7, 7, generator=g)
    gadd = torch.randn(1, 64, 30, 40, generator=g)
    gin = ext.roi_pool_bwd(_pair(gout, cuda, P), arg, rois.to(cuda), 1, 30, 40, _pair(gadd, cuda, P), P)
    refg = gadd.double().clone().reshape(64, -1)
    a = ref_arg.reshape(R, 64, -1).long()
    gg = gout.double().reshape(R, 64, -1)
    for r in range(R):
        m = a[r] >= 0
        refg.view(-1).index_add_(0, (torch.arange(64)[:, None] * 1200 + a[r].clamp_min(0))[m], gg[r][m])
    assert _err(_unpair(gin, P), refg.view(1, 64, 30, 40)) <= TOLS[P]


@pytest.mark.gpu
@pytest.mark.parametrize('P', PLANES)
def test_head_bwd_x2_matches_fp32(cuda, P):
    from mx_rcnn_amd.ops import need_ext
    g = torch.Generator().manual_seed(14)
    M, K = 300, 512
    x = torch.relu(torch.randn(M, K, generator=g))
    ws = [torch.randn(24, K, generator=g) * 0.02, torch.randn(48, K, generator=g) * 0.02]
    dys = [torch.randn(M, 24, generator=g), torch.randn(M, 48, generator=g)]
    wps = [precision.split(w.to(cuda), P) for w in ws]
    dws = [torch.zeros(w.shape, device=cuda) for w in ws]
    dbs = [torch.zeros(w.shape[0], device=cuda) for w in ws]
    dx = need_ext().head_bwd(precision.split(x.to(cuda), P), [d.to(cuda) for d in dys],
                             [p[:p.shape[0] // P] for p in wps], dws, [False, False], dbs, [False, False], True, True, P,
                             [p.numel() // P for p in wps])
    ref_dx = (dys[0].double() @ ws[0].double() + dys[1].double() @ ws[1].double()) * (x > 0)
    f32_dx = (dys[0] @ ws[0] + dys[1] @ ws[1]) * (x > 0)
    assert _err(_unpair(dx, P), ref_dx) <= _tol(P, ref_dx, f32_dx)
    for h in range(2):
        rw = dys[h].double().t() @ x.double()
        assert _err(dws[h], rw) <= _tol(P, rw, dys[h].t() @ x)
        assert _err(dbs[h], dys[h].double().sum(0)) <= TOLS[P]


@pytest.mark.gpu
@pytest.mark.parametrize('P', PLANES)
def test_stem_x2_matches_fp32(cuda, P):
    from mx_rcnn_amd.ops.stem import stem_conv
    from mx_rcnn_amd.models.layers import BatchNorm
    g = torch.Generator().manual_seed(15)
    x = torch.randn(1, 3, 64, 96, generator=g) * 50
    w = torch.randn(64, 3, 7, 7, generator=g) * 0.05
    bn_in = BatchNorm('bn_data', 3, fix_gamma=True, relu=False)
    bn_out = BatchNorm('bn0', 64)
    with torch.no_grad():
        bn_in.moving_mean.copy_(torch.randn(3)); bn_in.moving_var.copy_(torch.rand(3) * 100 + 50)
        bn_out.moving_mean.copy_(torch.randn(64)); bn_out.moving_var.copy_(torch.rand(64) + 0.5)
        bn_out.gamma.copy_(torch.rand(64) + 0.5); bn_out.beta.copy_(torch.randn(64))
    bn_in, bn_out = bn_in.to(cuda), bn_out.to(cuda)
    with precision.x2_mode(P):
        y = stem_conv(_cl(x.to(cuda)), w.to(cuda), 2, 3, in_bn=bn_in, out_bn=bn_out, relu=True)
    xs = (x.double() - bn_in.moving_mean.cpu().double().view(1, -1, 1, 1)) / torch.sqrt(
        bn_in.moving_var.cpu().double().view(1, -1, 1, 1) + bn_in.eps)
    ref = F.conv2d(xs, w.double(), stride=2, padding=3)
    s = bn_out.gamma.detach().cpu().double() / torch.sqrt(bn_out.moving_var.cpu().double() + bn_out.eps)
    ref = torch.relu((ref - bn_out.moving_mean.cpu().double().view(1, -1, 1, 1)) * s.view(1, -1, 1, 1)
                     + bn_out.beta.detach().cpu().double().view(1, -1, 1, 1))
    assert y.shape == (P * 1, 64, 32, 48)
    assert _err(_unpair(y, P), ref) <= 4 * TOLS[P]


@pytest.mark.gpu
@pytest.mark.parametrize('P', PLANES)
@pytest.mark.parametrize('n', [1000, 1003, 65536 + 8])
def test_sgd_x2_shadow(cuda, P, n):
    """The SGD kernel's shadow planes, one padded plane (a multiple of 8 elements) apart."""
    from mx_rcnn_amd.ops import need_ext
    g = torch.Generator().manual_seed(16)
    w = torch.randn(n, generator=g).to(cuda)
    mom = torch.zeros(n, device=cuda)
    grad = torch.randn(n, generator=g).to(cuda)
    pl = (n + 7) // 8 * 8
    sh = torch.zeros(P * pl, dtype=torch.bfloat16, device=cuda)
    lr = torch.full((1,), 0.1, device=cuda)
    w0 = w.clone()
    need_ext().sgd_momentum(w, mom, grad, lr, 0.9, 0.0, 1.0, -1.0, sh, P)
    assert torch.allclose(w, w0 - 0.1 * grad)
    j = sum(sh[k * pl:k * pl + n].float() for k in range(P))
    if P == 3:
        assert torch.equal(j, w)
    else:
        assert float(((j - w).abs() / w.abs().clamp_min(1e-30)).max()) <= 2.0 ** -16


@pytest.mark.gpu
@pytest.mark.parametrize('k,stride,pad,N,C,H,W,O', [(1, 1, 0, 1, 1024, 50, 84, 256), (3, 1, 1, 1, 256, 25, 42, 256),
                                                    (3, 2, 1, 2, 128, 17, 23, 96), (1, 2, 0, 1, 512, 13, 21, 1024)])
def test_conv_x2_wide_stage_equals_narrow(cuda, k, stride, pad, N, C, H, W, O):
    """The wide-stage bf16x3 kernel (tile 26: 64 channels of both planes per LDS stage) sums in
    the same K order as the 32-channel buffer kernel (tile 23): bitwise equal outputs, plain and
    with the residual + frozen-BN second-output epilogue, and within TOL of fp64."""
    from mx_rcnn_amd.ops import need_ext
    g = torch.Generator().manual_seed(k * 1000 + C + O)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(O, C, k, k, generator=g) * (2.0 / (C * k * k)) ** 0.5
    b = torch.randn(O, generator=g)
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=stride, padding=pad)
    xp, wp = _pair(x, cuda), _pair(w, cuda)
    ext = need_ext()
    ya = ext.conv_igemm_fwd(xp, wp[:O], b.to(cuda), stride, pad, False, 23, 1, x2=True, w_plane=wp.numel() // 2)[0]
    yb = ext.conv_igemm_fwd(xp, wp[:O], b.to(cuda), stride, pad, False, 26, 1, x2=True, w_plane=wp.numel() // 2)[0]
    assert torch.equal(ya, yb)
    assert _err(_unpair(yb), ref) <= TOL
    bn = [t.to(cuda) for t in (torch.rand(O) + 0.5, torch.randn(O), torch.randn(O), torch.rand(O) + 0.5)]
    res = _pair(torch.randn(ref.shape, generator=g), cuda)
    a1, a2 = ext.conv_igemm_fwd(xp, wp[:O], None, stride, pad, False, 23, 1, res, bn, 2e-5, False, True, x2=True,
                                w_plane=wp.numel() // 2)
    b1, b2 = ext.conv_igemm_fwd(xp, wp[:O], None, stride, pad, False, 26, 1, res, bn, 2e-5, False, True, x2=True,
                                w_plane=wp.numel() // 2)
    assert torch.equal(a1, b1) and torch.equal(a2, b2)
