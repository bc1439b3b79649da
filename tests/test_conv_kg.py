"""K-group implicit-GEMM conv kernels (csrc/hip/conv_kg.hip, tile codes 27-29): 2 or 4 groups of
four waves per 64x64 tile, each over a contiguous slice of K, partial tiles summed in the LDS
epilogue.  Checked against fp64 PyTorch on the same inputs and against the one-group buffer kernel
(tile 23), in the three storage modes (bf16, bf16x3 pairs, fp32 triples), forward and the stride-1
data gradient read from the forward filter (bt), with the fused epilogues (bias / ReLU, residual +
frozen-BN second output, BN-backward column sums) and split-K."""
import pytest
import torch
import torch.nn.functional as F

from mx_rcnn_amd.ops import precision

pytestmark = pytest.mark.gpu

TILES = [27, 28, 29]
MODES = [0, 2, 3]  # plane count: 0 = bf16 operands
KG_MODES = [0, 2, 3]  # bf16, bf16x3 pairs and fp32 triples (tile 29 falls back to 23 for triples)


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last) if t.dim() == 4 else t.contiguous()


def _err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-20))


def _enc(t, dev, P):
    t = _cl(t.to(dev))
    return _cl(precision.split(t, P)) if P else _cl(t.to(torch.bfloat16))


def _dec(t, P):
    return precision.join(t, P) if P else t.float()


def _wargs(w, dev, P):
    wp = _enc(w, dev, P)
    if not P:
        return wp, {}
    return wp[:w.shape[0]], {'x2': P, 'w_plane': wp.numel() // P}


def _tol(P, base):
    """K groups change the summation order only: within 2x of the one-group kernel's own error
    against fp64 (plus a floor at the storage precision)."""
    return 2 * base + {0: 1e-3, 2: 2e-6, 3: 2e-7}[P]


@pytest.mark.parametrize('P', KG_MODES)
@pytest.mark.parametrize('tile', TILES)
@pytest.mark.parametrize('k,stride,pad,C,H,W,O', [
    (1, 1, 0, 1024, 25, 42, 256),   # stage-3 1x1 reduce (batch-1 800x1333 / 2 in each dim)
    (3, 1, 1, 256, 25, 42, 256),    # stage-3 3x3
    (1, 1, 0, 256, 25, 42, 1024),   # stage-3 1x1 expand
    (3, 2, 1, 128, 23, 31, 128),    # strided 3x3
])
def test_kg_forward_matches(cuda, P, tile, k, stride, pad, C, H, W, O):
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(1000 * k + C + O)
    x = torch.randn(1, C, H, W, generator=g)
    w = torch.randn(O, C, k, k, generator=g) * (2.0 / (C * k * k)) ** 0.5
    b = torch.randn(O, generator=g)
    if not P:  # bf16 mode: the operands themselves are bf16
        x, w = x.bfloat16().float(), w.bfloat16().float()
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=stride, padding=pad)
    xe = _enc(x, cuda, P)
    we, kw = _wargs(w, cuda, P)
    bb = b.to(cuda) if P else b.to(cuda, torch.bfloat16)
    y23 = ext.conv_igemm_fwd(xe, we, bb, stride, pad, True, 23, 1, **kw)[0]
    ykg = ext.conv_igemm_fwd(xe, we, bb, stride, pad, True, tile, 1, **kw)[0]
    rref = torch.relu(ref)
    base = _err(_dec(y23, P), rref)
    assert _err(_dec(ykg, P), rref) <= _tol(P, base), (base, _err(_dec(ykg, P), rref))
    # residual + frozen BN + ReLU second output
    O_ = ref.shape
    res = torch.randn(O_, generator=g)
    bn = [t.to(cuda) for t in (torch.rand(O) + 0.5, torch.randn(O), torch.randn(O), torch.rand(O) + 0.5)]
    re = _enc(res, cuda, P)
    a1, a2 = ext.conv_igemm_fwd(xe, we, None, stride, pad, False, 23, 1, re, bn, 2e-5, False, True, **kw)
    k1, k2 = ext.conv_igemm_fwd(xe, we, None, stride, pad, False, tile, 1, re, bn, 2e-5, False, True, **kw)
    r1 = ref - b.double().view(1, -1, 1, 1) + _dec(re, P).double().cpu()
    assert _err(_dec(k1, P), r1) <= _tol(P, _err(_dec(a1, P), r1))
    assert _err(_dec(k2, P), _dec(a2, P)) <= 4 * _tol(P, _err(_dec(a1, P), r1))


@pytest.mark.parametrize('P', KG_MODES)
@pytest.mark.parametrize('tile', TILES)
def test_kg_splitk_and_bt_dgrad(cuda, P, tile):
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(77 + P)
    C, H, W, O = 256, 13, 21, 512
    x = torch.randn(1, C, H, W, generator=g)
    w = torch.randn(O, C, 3, 3, generator=g) * 0.03
    if not P:
        x, w = x.bfloat16().float(), w.bfloat16().float()
    xe = _enc(x, cuda, P)
    we, kw = _wargs(w, cuda, P)
    ref = F.conv2d(x.double(), w.double(), padding=1)
    base = _err(_dec(ext.conv_igemm_fwd(xe, we, None, 1, 1, False, 23, 2, **kw)[0], P), ref)
    got = ext.conv_igemm_fwd(xe, we, None, 1, 1, False, tile, 2, **kw)[0]  # split-K 2 on top of the groups
    assert _err(_dec(got, P), ref) <= _tol(P, base)
    # stride-1 data gradient straight from the forward filter (bt): dx = conv_transpose(dy, w)
    dy = torch.randn(1, O, H, W, generator=g)
    if not P:
        dy = dy.bfloat16().float()
    dye = _enc(dy, cuda, P)
    refd = torch.nn.grad.conv2d_input((1, C, H, W), w.double(), dy.double(), padding=1)
    d23 = ext.conv_igemm_fwd(dye, we, None, 1, 1, False, 23, 1, bt=True, **kw)[0]
    dkg = ext.conv_igemm_fwd(dye, we, None, 1, 1, False, tile, 1, bt=True, **kw)[0]
    assert _err(_dec(dkg, P), refd) <= _tol(P, _err(_dec(d23, P), refd))


@pytest.mark.parametrize('P', KG_MODES)
def test_kg_bn_backward_epilogue(cuda, P):
    """BN-backward epilogue (dgrad fused with the frozen BN + ReLU backward, fp32 column sums)."""
    from mx_rcnn_amd.ops import need_ext
    from mx_rcnn_amd.ops.conv import _flip_t
    ext = need_ext()
    g = torch.Generator().manual_seed(5 + P)
    C, H, W, O = 256, 14, 18, 256
    dy = torch.randn(1, O, H, W, generator=g)
    w = torch.randn(O, C, 3, 3, generator=g) * 0.03
    xbn = torch.randn(1, C, H, W, generator=g)
    if not P:
        dy, w, xbn = dy.bfloat16().float(), w.bfloat16().float(), xbn.bfloat16().float()
    gam, bet, mu, var = torch.rand(C) + 0.5, torch.randn(C) * 0.1, torch.randn(C) * 0.1, torch.rand(C) + 0.5
    bn = [t.to(cuda) for t in (gam, bet, mu, var)]
    wf, kw = _wargs(_flip_t(w), cuda, P)
    outs = {}
    for tile in (23, 27, 28, 29):
        dg, db = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
        dx = ext.conv_igemm_fwd(_enc(dy, cuda, P), wf, None, 1, 1, False, tile, 1, None, bn, 2e-5, False, True,
                                _enc(xbn, cuda, P), None, dg, db, **kw)[0]
        outs[tile] = (_dec(dx, P), dg.clone(), db.clone())
    dact = torch.nn.grad.conv2d_input((1, C, H, W), w.double(), dy.double(), padding=1)
    s = gam.double() / torch.sqrt(var.double() + 2e-5)
    pre = (xbn.double() - mu.double().view(1, -1, 1, 1)) * s.view(1, -1, 1, 1) + bet.double().view(1, -1, 1, 1)
    gm = dact * (pre > 0)
    for tile in (27, 28, 29):
        for i, ref in enumerate((gm * s.view(1, -1, 1, 1), None, gm.sum((0, 2, 3)))):
            if ref is None:
                continue
            base = _err(outs[23][i], ref)
            assert _err(outs[tile][i], ref) <= _tol(P, base) + 1e-6, (tile, i, base, _err(outs[tile][i], ref))


@pytest.mark.parametrize('P', MODES)
def test_grouped_bt_dgrad_wgrad(cuda, P):
    """The grouped data + weight gradient launch reading the forward filter transposed (bt) -- the
    fused one-pass form for fp32 triples -- against fp64: dgrad with the frozen BN-ReLU backward
    epilogue, and the weight gradient of a 3x3 conv over the same dY."""
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(31 + P)
    C, H, W, O = 128, 17, 23, 256
    dy = torch.randn(1, O, H, W, generator=g)
    w = torch.randn(O, C, 3, 3, generator=g) * 0.03
    xbn = torch.randn(1, C, H, W, generator=g)
    xin = torch.randn(1, 128, H, W, generator=g)
    if not P:
        dy, w, xbn, xin = (t.bfloat16().float() for t in (dy, w, xbn, xin))
    gam, bet, mu, var = torch.rand(C) + 0.5, torch.randn(C) * 0.1, torch.randn(C) * 0.1, torch.rand(C) + 0.5
    bn = [t.to(cuda) for t in (gam, bet, mu, var)]
    we, kw = _wargs(w, cuda, P)
    dgm, dbt = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
    gdt = torch.float32 if P else torch.bfloat16
    wg = _cl(torch.zeros(O, 128, 3, 3, device=cuda, dtype=gdt))
    dye = _enc(dy, cuda, P)
    out = ext.conv_dgrad_wgrad(dye, we, 1, None, bn, 2e-5, False, _enc(xbn, cuda, P), None, dgm, dbt, dye,
                               _enc(xin, cuda, P), 3, 3, 1, 1, wg, bt=True, **kw)
    dact = torch.nn.grad.conv2d_input((1, C, H, W), w.double(), dy.double(), padding=1)
    s = gam.double() / torch.sqrt(var.double() + 2e-5)
    pre = (xbn.double() - mu.double().view(1, -1, 1, 1)) * s.view(1, -1, 1, 1) + bet.double().view(1, -1, 1, 1)
    gm = dact * (pre > 0)
    ref_dw = torch.nn.grad.conv2d_weight(xin.double(), (O, 128, 3, 3), dy.double(), padding=1)
    tol = {0: 2e-2, 2: 4e-5, 3: 4e-6}[P]
    assert _err(_dec(out[0], P), gm * s.view(1, -1, 1, 1)) <= tol
    assert _err(dbt, gm.sum((0, 2, 3))) <= tol
    assert _err(wg.float(), ref_dw) <= tol
