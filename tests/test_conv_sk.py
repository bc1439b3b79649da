"""Stream-K 64x64 conv (tile code 40, csrc/hip/conv_igemm.hip conv_igemm_sk_kernel): on grids a
little over the CU count (the batch-1 stage-3 GEMMs: 264 / 1056 tiles on 256 CUs) every
workgroup runs an equal share of (tile, K) steps; a tile split between two workgroups is summed
through a partial + flag.  Checked against the fp32 conv of the same operands (bf16, bf16x3 pairs,
fp32 triples), against the plain 64x64 kernel, run-to-run bitwise, and with the fused residual /
ReLU epilogue."""
import pytest
import torch
import torch.nn.functional as F

from mx_rcnn_amd.ops.precision import join, split


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.gpu
@pytest.mark.parametrize('mode', ['bf16', 'x2', 'x3'])
@pytest.mark.parametrize('cin,cout,k', [(256, 256, 3), (1024, 256, 1), (256, 1024, 1), (192, 320, 3)])
def test_stream_k_conv_matches_reference(cuda, mode, cin, cout, k):
    from mx_rcnn_amd.ops import need_ext
    ext = need_ext()
    g = torch.Generator().manual_seed(cin + cout + k)
    H, W = 50, 84  # M = 4200: 66 row tiles
    x = torch.randn(1, cin, H, W, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    res = torch.randn(1, cout, H, W, generator=g)
    p = k // 2
    planes = {'bf16': 0, 'x2': 2, 'x3': 3}[mode]
    if planes:
        xs, ws, rs = _cl(split(x.to(cuda), planes)), _cl(split(w.to(cuda), planes)), _cl(split(res.to(cuda), planes))
        kw = dict(x2=planes, w_plane=ws.numel() // planes)
        wk = ws[:cout]
        xr, wr, rr = join(xs, planes).float(), join(ws, planes).float(), join(rs, planes).float()
    else:
        xs, wk, rs = _cl(x.to(cuda).bfloat16()), _cl(w.to(cuda).bfloat16()), _cl(res.to(cuda).bfloat16())
        kw = {}
        xr, wr, rr = xs.float(), wk.float(), rs.float()
    ref = torch.relu(F.conv2d(xr.double(), wr.double(), padding=p) + rr.double())

    def run(tile):
        return ext.conv_igemm_fwd(xs, wk, None, 1, p, True, tile, 1, rs, **kw)[0]

    y40a = run(40)
    y40b = run(40)
    y23 = run(23)
    torch.cuda.synchronize()
    assert torch.equal(y40a, y40b), 'stream-K conv is not run-to-run deterministic'
    got = join(y40a, planes).double() if planes else y40a.double()
    base = join(y23, planes).double() if planes else y23.double()
    scale = ref.abs().max()
    tol = {0: 2e-2, 2: 2e-4, 3: 2e-5}[planes]
    assert float((got - ref).abs().max() / scale) < tol
    assert float((got - base).abs().max() / scale) < tol
