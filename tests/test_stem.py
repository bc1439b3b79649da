"""Fused stem convolution (csrc/hip/stem.hip, ops/stem.py): filter packing on the CPU, the HIP
kernel against an fp32 PyTorch oracle, and the trunks with the fused stem vs the unfused layers."""
import os

import pytest
import torch
import torch.nn.functional as F

from mx_rcnn_amd.models.layers import BatchNorm
from mx_rcnn_amd.ops.stem import bn_affine, pack_filter, stem_conv, stem_conv_reference


def _bn(name, c, fix_gamma, relu, g):
    bn = BatchNorm(name, c, fix_gamma=fix_gamma, relu=relu)
    with torch.no_grad():
        bn.gamma.copy_(torch.rand(c, generator=g) + 0.5)
        bn.beta.copy_(torch.randn(c, generator=g) * 0.2)
        bn.moving_mean.copy_(torch.randn(c, generator=g) * 10)
        bn.moving_var.copy_(torch.rand(c, generator=g) * 400 + 50)
    return bn.eval()


@pytest.mark.parametrize('k,s,p', [(7, 2, 3), (3, 1, 1)])
def test_pack_filter_is_im2col_order(k, s, p):
    """(64, KP) rows dotted with an im2col row in (fr, fc, c) order reproduce conv2d."""
    g = torch.Generator().manual_seed(0)
    w = torch.randn(64, 3, k, k, generator=g)
    x = torch.randn(1, 3, 13, 17, generator=g)
    wp = pack_filter(w, torch.float32)
    K = 3 * k * k
    assert wp.shape == (64, (K + 31) // 32 * 32) and torch.all(wp[:, K:] == 0)
    cols = F.unfold(x, k, padding=p, stride=s)  # (1, 3*k*k [c, fr, fc], L)
    cols = cols.view(3, k, k, -1).permute(1, 2, 0, 3).reshape(K, -1)  # -> (fr, fc, c)
    y = (wp[:, :K] @ cols).view(1, 64, *F.conv2d(x, w, stride=s, padding=p).shape[2:])
    torch.testing.assert_close(y, F.conv2d(x, w, stride=s, padding=p), rtol=1e-4, atol=1e-4)


def test_bn_affine_matches_batch_norm():
    g = torch.Generator().manual_seed(1)
    for fix in (True, False):
        bn = _bn('b', 5, fix, False, g)
        x = torch.randn(2, 5, 3, 4, generator=g)
        s, t = bn_affine(bn)
        gam = torch.ones(5) if fix else bn.gamma.detach()
        ref = F.batch_norm(x, bn.moving_mean, bn.moving_var, gam, bn.beta.detach(), False, 0.0, bn.eps)
        torch.testing.assert_close(x * s.view(1, -1, 1, 1) + t.view(1, -1, 1, 1), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('geom', ['resnet', 'vgg'])
@pytest.mark.parametrize('hw', [(67, 101), (130, 45)])
def test_stem_kernel_vs_fp32(cuda, dtype, geom, hw):
    g = torch.Generator().manual_seed(2)
    H, W = hw
    x = (torch.randn(2, 3, H, W, generator=g) * 50 + 100).to(cuda, dtype).contiguous(memory_format=torch.channels_last)
    if geom == 'resnet':
        w = (torch.randn(64, 3, 7, 7, generator=g) * 0.05).to(cuda, dtype)
        bd = _bn('bn_data', 3, True, False, g).to(cuda)
        b0 = _bn('bn0', 64, False, True, g).to(cuda)
        args = dict(stride=2, pad=3, in_bn=bd, out_bn=b0, relu=True)
    else:
        w = (torch.randn(64, 3, 3, 3, generator=g) * 0.05).to(cuda, dtype)
        b = (torch.randn(64, generator=g)).to(cuda, dtype)
        args = dict(stride=1, pad=1, bias=b, relu=True)
    with torch.no_grad():
        y = stem_conv(x, w, **args)
        ref = stem_conv_reference(x, w, **args)
    assert y.shape == ref.shape and y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    err = (y.float() - ref).abs().max().item()
    tol = 0.02 * ref.abs().max().item() + 0.05
    assert err <= tol, (err, tol)


@pytest.mark.gpu
def test_resnet_trunk_fused_stem_matches_unfused(cuda, monkeypatch):
    """bn_data -> conv0 -> bn0 -> relu in one launch == the three-layer path (frozen, eval)."""
    from mx_rcnn_amd.models.resnet import ResNetTrunk
    torch.manual_seed(3)
    m = ResNetTrunk(depth=18).to(cuda).eval()
    g = torch.Generator().manual_seed(4)
    for bn in (m.bn_data, m.bn0):
        with torch.no_grad():
            bn.moving_mean.copy_(torch.randn(bn.moving_mean.shape, generator=g).to(cuda))
            bn.moving_var.copy_((torch.rand(bn.moving_var.shape, generator=g) + 0.5).to(cuda))
    m = m.to(torch.bfloat16)
    for bn in (m.bn_data, m.bn0):
        bn.float()
    x = (torch.randn(1, 3, 96, 160, generator=g) * 50).to(cuda, torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    with torch.no_grad():
        monkeypatch.setenv('MXR_STEM', '1')
        y1 = m.bn0(m.conv0(m.bn_data(x)))
        y_f = stem_conv(x, m.conv0.weight, 2, 3, in_bn=m.bn_data, out_bn=m.bn0, relu=True)
        assert m._stem_fused(x)
        monkeypatch.setenv('MXR_STEM', '0')
        assert not m._stem_fused(x)
    err = (y_f.float() - y1.float()).abs().max().item()
    assert err <= 0.03 * y1.float().abs().max().item() + 0.05, err
