"""Data gradients that read the forward filter transposed in-kernel (ConvEpi::bt), the fused ReLU /
dropout backward epilogue (ConvEpi::rmask), the standalone ReLU-mask kernel and the fused VGG16
trunk / head built on them (ops/vgg_fused.py).

bt reads the same filter elements in the same K order as the flipped / transposed copy it
replaces, so the two launches must agree BITWISE; the masked epilogue must equal the unmasked
result times the mask (exact: 0/1 times a power-of-two scale).  The fused VGG sequences are checked
against the per-layer autograd path (MXR_VGG_FUSED=0) on identical weights and inputs.
"""
import os

import pytest
import torch

from mx_rcnn_amd.ops import precision

pytestmark = pytest.mark.gpu


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _flip_t(w):
    return _cl(w.flip(2, 3).transpose(0, 1))


@pytest.mark.parametrize('k,O,I,H,W', [(3, 128, 64, 17, 23), (1, 256, 128, 9, 14), (3, 64, 256, 6, 7),
                                       (1, 4096, 512, 1, 1)])
def test_bt_dgrad_bitwise_equals_flipped_copy(cuda, k, O, I, H, W):
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(k + O + I)
    w = _cl(torch.randn(O, I, k, k, generator=g).to(cuda, torch.bfloat16))  # forward filter (O, I, k, k)
    N = 128 if H == 1 else 1
    dy = _cl(torch.randn(N, O, H, W, generator=g).to(cuda, torch.bfloat16))
    pad = (k - 1) // 2
    for tile in (0, 22, 23):
        ref = ext.conv_igemm_fwd(dy, _flip_t(w), None, 1, k - 1 - pad, False, tile, 1)[0]
        got = ext.conv_igemm_fwd(dy, w, None, 1, k - 1 - pad, False, tile, 1, bt=True)[0]
        assert got.shape == (N, I, H, W)
        assert torch.equal(got, ref), (tile, float((got.float() - ref.float()).abs().max()))
    # split-K plan (small grids) reduces the same partial sums
    got = ext.conv_igemm_fwd(dy, w, None, 1, k - 1 - pad, False, bt=True)[0]
    ref = torch.nn.grad.conv2d_input((N, I, H, W), w.float(), dy.float(), padding=pad)
    assert float((got.float() - ref).abs().max() / ref.abs().max()) < 2e-2


def test_bt_dgrad_x2_matches_fp32(cuda):
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(5)
    O, I, k, H, W = 128, 64, 3, 15, 21
    w = torch.randn(O, I, k, k, generator=g) * 0.05
    dy = torch.randn(1, O, H, W, generator=g)
    ref = torch.nn.grad.conv2d_input((1, I, H, W), w.double(), dy.double(), padding=1)
    wp = _cl(precision.split(_cl(w.to(cuda))))
    got = ext.conv_igemm_fwd(_cl(precision.split(_cl(dy.to(cuda)))), wp[:O], None, 1, 1, False, bt=True, x2=True,
                             w_plane=wp.numel() // 2)[0]
    err = float((precision.join(got).double().cpu() - ref).abs().max() / ref.abs().max())
    assert err <= 2e-5, err


def test_grouped_bt_matches_plain(cuda):
    """The grouped dgrad + wgrad launch with bt and an rmask epilogue against separate launches."""
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(9)
    O, I, H, W = 128, 64, 19, 25
    w = _cl(torch.randn(O, I, 3, 3, generator=g).to(cuda, torch.bfloat16) * 0.05)
    d = _cl(torch.randn(1, O, H, W, generator=g).to(cuda, torch.bfloat16))
    x = _cl(torch.relu(torch.randn(1, I, H, W, generator=g)).to(cuda, torch.bfloat16))  # a ReLU output
    tgt = _cl(torch.zeros(O, I, 3, 3, device=cuda, dtype=torch.bfloat16))
    dx = ext.conv_dgrad_wgrad(d, w, 1, None, None, 0.0, False, None, None, None, None, d, x, 3, 3, 1, 1, tgt, bt=True,
                              rmask=x, rmask_scale=2.0)[0]
    ref = ext.conv_igemm_fwd(d, _flip_t(w), None, 1, 1, False, 23, 1)[0]
    assert torch.equal(dx, (ref.float() * (x > 0) * 2.0).to(torch.bfloat16))
    dw = ext.conv_wgrad(d, x, 3, 3, 1, 1)
    assert torch.equal(tgt, dw)


def test_rmask_epilogue_and_relu_mask_kernel(cuda):
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(2)
    O, I, H, W = 64, 128, 13, 11
    w = _cl(torch.randn(O, I, 1, 1, generator=g).to(cuda, torch.bfloat16))
    d = _cl(torch.randn(1, O, H, W, generator=g).to(cuda, torch.bfloat16))
    x = _cl(torch.randn(1, I, H, W, generator=g).to(cuda, torch.bfloat16)).clamp_min(0)
    x[0, :, 0, 0] = 0
    plain = ext.conv_igemm_fwd(d, w, None, 1, 0, False, bt=True)[0]
    for tile in (22, 23):
        got = ext.conv_igemm_fwd(d, w, None, 1, 0, False, tile, 1, bt=True, rmask=x, rmask_scale=2.0)[0]
        assert torch.equal(got, (plain.float() * (x > 0) * 2.0).to(torch.bfloat16))
    # split-K: the mask in the reduce kernel
    ref4 = ext.conv_igemm_fwd(d, w, None, 1, 0, False, 23, 4, bt=True)[0]
    got = ext.conv_igemm_fwd(d, w, None, 1, 0, False, 23, 4, bt=True, rmask=x)[0]
    assert torch.equal(got, (ref4.float() * (x > 0)).to(torch.bfloat16))
    dd = _cl(torch.randn(1, I, H, W, generator=g).to(cuda, torch.bfloat16))
    m = ext.relu_mask_bwd(dd, x, 0.5)
    assert torch.equal(m, (dd.float() * (x > 0) * 0.5).to(torch.bfloat16))
    # x2: the hi plane's sign masks both planes
    dp = _cl(precision.split(_cl(torch.randn(1, I, H, W, generator=g).to(cuda))))
    xp = _cl(precision.split(_cl(x.float())))
    mp = ext.relu_mask_bwd(dp, xp, 1.0, True)
    ref = precision.join(dp) * (x.float() > 0)
    assert torch.equal(precision.join(mp), ref)


def _vgg_pair(cuda, precision_mode, fused):
    from mx_rcnn_amd.config import snapshot
    from mx_rcnn_amd.core.trainer import Trainer
    from mx_rcnn_amd.models import FasterRCNN
    torch.manual_seed(3)
    os.environ['MXR_VGG_FUSED'] = '1' if fused else '0'
    m = FasterRCNN('vgg16', 21, cfg=snapshot(), train_mode='rcnn')
    return Trainer(m, 'rcnn', fixed_param_prefix=['conv1', 'conv2'], lr=0.0, device=cuda, precision=precision_mode)


def test_vgg_fused_matches_per_layer(cuda):
    """bf16: the fused trunk / head against per-layer autograd (torch ReLU masks, flipped filters)."""
    from tests.test_parity import _rcnn_batch, _fwd_bwd
    b = _rcnn_batch()
    try:
        tf = _vgg_pair(cuda, 'bf16', True)
        of, gf = _fwd_bwd(tf, b)
        tu = _vgg_pair(cuda, 'bf16', False)
        ou, gu = _fwd_bwd(tu, b)
    finally:
        os.environ.pop('MXR_VGG_FUSED', None)
    for k in ('cls_loss', 'bbox_loss'):
        a, r = float(of[k].float().sum()), float(ou[k].float().sum())
        assert abs(a - r) <= 1e-3 * max(abs(r), 1e-6), (k, a, r)
    assert set(gf) == set(gu)
    for n in gu:
        a, r = gf[n], gu[n]
        cos = float(torch.dot(a, r) / (a.norm() * r.norm() + 1e-30))
        rel = float((a.norm() - r.norm()).abs() / (r.norm() + 1e-30))
        assert cos >= 0.999 and rel <= 0.01, (n, cos, rel)


def test_vgg_fp32_gpu_matches_fp32_cpu(cuda):
    """fp32-class fused VGG16 (dropout off: the CPU path draws its mask from torch's RNG) against the
    fp32 CPU step: losses to 1e-3, every layer's gradient cosine >= 0.99."""
    import copy
    from mx_rcnn_amd.config import snapshot
    from mx_rcnn_amd.core.trainer import Trainer
    from mx_rcnn_amd.models import FasterRCNN
    from tests.test_parity import _rcnn_batch, _fwd_bwd, _check_grads_tight, _rel
    torch.manual_seed(3)
    m = FasterRCNN('vgg16', 21, cfg=snapshot(), train_mode='rcnn')
    m.head.dropout = 0.0
    mg = copy.deepcopy(m)
    cpu = Trainer(m, 'rcnn', fixed_param_prefix=['conv1', 'conv2'], lr=0.0, device='cpu')
    gpu = Trainer(mg, 'rcnn', fixed_param_prefix=['conv1', 'conv2'], lr=0.0, device=cuda, precision='fp32')
    b = _rcnn_batch()
    oc, gc = _fwd_bwd(cpu, b)
    og, gg = _fwd_bwd(gpu, b)
    for k in ('cls_loss', 'bbox_loss'):
        assert _rel(og[k].float().cpu().sum(), oc[k].float().sum()) <= 1e-3, (k, og[k], oc[k])
    _check_grads_tight(gc, gg, min_layers=8)
