"""Single unit: fp32 torch oracle vs unfused kernels vs fused unit op (forward + all grads)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
from test_fused import _unit, _cl  # noqa: E402
from debug_fused import rep  # noqa: E402  (runs the first debug too; cheap)

dev = torch.device('cuda', 0)


def bn_relu32(x, bn):
    s = bn.gamma.float() * torch.rsqrt(bn.moving_var.float() + bn.eps)
    t = bn.beta.float() - bn.moving_mean.float() * s
    return torch.relu(x * s[None, :, None, None] + t[None, :, None, None])


def oracle(u, x, d_out):
    """fp32 autograd with leaf copies of every parameter."""
    P = {n: p.detach().float().clone().requires_grad_() for n, p in u.named_parameters()}

    class B:
        pass

    def bn(name):
        b = B()
        m = getattr(u, name)
        b.gamma, b.beta, b.moving_mean, b.moving_var, b.eps = P[name + '.gamma'], P[name + '.beta'], m.moving_mean, \
            m.moving_var, m.eps
        return b
    xx = x.detach().float().clone().requires_grad_()
    a1 = bn_relu32(xx, bn('bn1'))
    y = F.conv2d(a1, P['conv1.weight'])
    y = F.conv2d(bn_relu32(y, bn('bn2')), P['conv2.weight'], stride=u.conv2.stride, padding=1)
    y = F.conv2d(bn_relu32(y, bn('bn3')), P['conv3.weight'])
    sc = xx if u.dim_match else F.conv2d(a1, P['sc.weight'], stride=u.sc.stride)
    out = y + sc
    out.backward(d_out.float())
    return out, xx.grad, {n: p.grad for n, p in P.items()}


for cfg in [(256, 256, 1, True, True), (1024, 1024, 1, True, True)]:
    cin, cout, stride, dm, bottle = cfg
    u = _unit(cin, cout, stride, dm, dev, bottle)
    x0 = torch.randn(1, cin, 24, 40, generator=torch.Generator().manual_seed(6)).bfloat16()
    d_out = _cl(torch.randn(1, cout, 24, 40, generator=torch.Generator().manual_seed(7)).bfloat16(), dev)
    o_ref, xg_ref, g_ref = oracle(u, _cl(x0, dev), d_out)
    for mode in ('unfused', 'fused_unit'):
        os.environ['MXR_FUSE_UNIT'] = '1'
        x = _cl(x0, dev).requires_grad_()
        for p_ in u.parameters():
            p_.grad = None
        out = u(x) if mode == 'unfused' else u.forward_fused(x, None, None)[0]
        out.backward(d_out)
        print('==', cfg, mode)
        rep('out', out, o_ref)
        rep('x.grad', x.grad, xg_ref)
        for n, p_ in u.named_parameters():
            if p_.grad is not None:
                rep(n, p_.grad, g_ref[n])

print('--- chained u -> v: unfused vs fused vs fp32 oracle (relL2)')
import debug_fused  # noqa: E402,F401
for cfg in [(1024, 1024, 1, True, True)]:
    cin, cout, stride, dm, bottle = cfg
    u = _unit(cin, cout, stride, dm, dev, bottle)
    v = _unit(cout, cout, 1, True, dev, bottle)
    x0 = torch.randn(1, cin, 24, 40, generator=torch.Generator().manual_seed(6)).bfloat16()
    d_out = _cl(torch.randn(1, cout, 24, 40, generator=torch.Generator().manual_seed(7)).bfloat16(), dev)
    res = {}
    for mode in ('unfused', 'fused'):
        x = _cl(x0, dev).requires_grad_()
        for p_ in list(u.parameters()) + list(v.parameters()):
            p_.grad = None
        if mode == 'unfused':
            out = v(u(x))
        else:
            ou, act = u.forward_fused(x, None, v.bn1)
            out, _ = v.forward_fused(ou, act, None)
        out.backward(d_out)
        res[mode] = (x.grad.clone(), {('u.' + n): p_.grad.clone() for n, p_ in u.named_parameters()})
    rep('x.grad fused vs unfused', res['fused'][0], res['unfused'][0])
    for n in res['unfused'][1]:
        rep(n + ' f/u', res['fused'][1][n], res['unfused'][1][n])
