"""Stage-by-stage comparison of the fused ResNet-unit ops against the unfused modules (GPU)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))

from test_fused import _unit, _cl  # noqa: E402
from mx_rcnn_amd.ops.fused import conv_bn_relu, conv_add, conv_add_bn_relu  # noqa: E402


def rep(name, a, b):
    d = (a.float() - b.float()).abs()
    idx = d.argmax().item()
    loc = torch.unravel_index(torch.tensor(idx), d.shape)
    rel = (d.norm() / b.float().norm().clamp_min(1e-12)).item()
    print('%-28s relL2 %.4f maxdiff %.5f at %s (ref %.4f got %.4f) scale %.3f' % (
        name, rel, d.max().item(), tuple(int(v) for v in loc), b.flatten()[idx].item(), a.flatten()[idx].item(),
        b.float().abs().max().item()), flush=True)


if __name__ == '__main__':
    dev = torch.device('cuda', 0)
    for cfg in [(1024, 1024, 1, True, True), (256, 256, 1, True, True)]:
        cin, cout, stride, dm, bottle = cfg
        print('cfg', cfg)
        u = _unit(cin, cout, stride, dm, dev, bottle)
        x = _cl(torch.randn(1, cin, 24, 40, generator=torch.Generator().manual_seed(6)).bfloat16(), dev)
        with torch.no_grad():
            act1 = u.bn1(x)
            r1 = u.bn2(u.conv1(act1))
            f1 = conv_bn_relu(act1, u.conv1, u.bn2)
            rep('conv1+bn2', f1, r1)
            c1 = u.conv1(act1)
            rep('conv1 raw (igemm vs F)', c1, F.conv2d(act1.float(), u.conv1.weight.float()))
            r2 = u.bn3(u.conv2(r1))
            f2 = conv_bn_relu(r1, u.conv2, u.bn3)
            rep('conv2+bn3', f2, r2)
            r3 = u.conv3(r2) + x
            f3 = conv_add(r2, u.conv3, x)
            rep('conv3+res', f3, r3)
            f4, a4 = conv_add_bn_relu(r2, u.conv3, x, u.bn1)
            rep('conv3+res (bn out)', f4, r3)
            rep('next bn1', a4, u.bn1(r3))
            rep('unit fwd', u.forward_fused(x, None, None)[0], u(x))

    print('--- chained units, forward + backward')
    for unit_op in ('0', '1'):
        os.environ['MXR_FUSE_UNIT'] = unit_op
        for cfg in [(1024, 1024, 1, True, True), (256, 512, 1, False, True)]:
            cin, cout, stride, dm, bottle = cfg
            print('unit_op', unit_op, 'cfg', cfg)
            u = _unit(cin, cout, stride, dm, dev, bottle)
            v = _unit(cout, cout, 1, True, dev, bottle)
            x0 = torch.randn(1, cin, 24, 40, generator=torch.Generator().manual_seed(6)).bfloat16()
            res = []
            for fused in (False, True):
                x = _cl(x0, dev).requires_grad_()
                if fused:
                    ou, act = u.forward_fused(x, None, v.bn1)
                    out, _ = v.forward_fused(ou, act, None)
                else:
                    ou = u(x)
                    out = v(ou)
                d_out = torch.randn(out.shape, generator=torch.Generator().manual_seed(7)).bfloat16().to(dev)
                for p_ in list(u.parameters()) + list(v.parameters()):
                    p_.grad = None
                out.backward(d_out)
                gr = {t + n: p_.grad.float().clone() for t, m in (('u.', u), ('v.', v)) for n, p_ in m.named_parameters()
                      if p_.grad is not None}
                res.append((ou.detach(), out.detach(), x.grad.clone(), gr))
            rep('out_u', res[1][0], res[0][0])
            rep('out', res[1][1], res[0][1])
            rep('x.grad', res[1][2], res[0][2])
            for k in res[0][3]:
                if k in res[1][3]:
                    rep(k, res[1][3][k], res[0][3][k])
                else:
                    print('missing grad', k)
