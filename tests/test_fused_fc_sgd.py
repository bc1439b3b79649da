"""VGG16's FC weights updated inside their weight-gradient kernel (csrc conv_wgrad_sgd, ops/vgg_fused.py,
core/params.py enable_fused_sgd): the 120 M-element fc6 / fc7 gradient is never stored, and the
end-of-step SGD skips exactly those ranges.  The result must match the unfused step
(MXR_FUSED_FC_SGD=0) in every storage mode, with the shadow planes still the exact split of the
masters."""
import pytest
import torch

from mx_rcnn_amd.core.params import FlatParamStore
from mx_rcnn_amd.core.trainer import Trainer
from mx_rcnn_amd.models import FasterRCNN
from tests.test_model import _batch, _cfg


def test_sgd_step_skips_applied_fused_ranges_cpu():
    """The store's SGD over the complement of the applied fused ranges equals the full SGD there
    and leaves the fused ranges untouched (CPU: the range logic; the kernel is GPU-only)."""
    torch.manual_seed(0)
    m = FasterRCNN('vgg16', 21, cfg=_cfg())
    st = FlatParamStore(m, ['conv1', 'conv2'], torch.float32, 'cpu', False)
    ref = FlatParamStore(FasterRCNN('vgg16', 21, cfg=_cfg()), ['conv1', 'conv2'], torch.float32, 'cpu', False)
    for g, r in zip(st.groups, ref.groups):
        r.master.copy_(g.master)
        g.grad.normal_()
        r.grad.copy_(g.grad)
        g.mom.normal_()
        r.mom.copy_(g.mom)
    gi = max(range(len(st.groups)), key=lambda i: st.groups[i].numel)
    g = st.groups[gi]
    names = [e[0] for e in g.entries]
    picks = [names.index('fc7_weight'), names.index('fc6_weight')]
    specs = [{'off': g.offsets[i], 'numel': g.entries[i][3], 'applied': True} for i in picks]
    st._fused = {gi: specs}
    before = g.master.clone()
    lr = torch.tensor([0.01])
    st.sgd_step(lr, 0.9, 0.0005, 1.0, 1.0, refresh=False)
    ref.sgd_step(lr, 0.9, 0.0005, 1.0, 1.0, refresh=False)
    mask = torch.ones(g.numel, dtype=torch.bool)
    for sp in specs:
        mask[sp['off']:sp['off'] + sp['numel']] = False
        assert not sp['applied']  # reset for the next step
    assert torch.equal(g.master[~mask], before[~mask])
    assert torch.equal(g.master[mask], ref.groups[gi].master[mask])
    for a, b in zip(st.groups, ref.groups):
        if a is not g:
            assert torch.equal(a.master, b.master)


@pytest.mark.gpu
@pytest.mark.parametrize('prec', ['bf16', 'bf16x3', 'fp32'])
def test_fused_fc_update_matches_unfused_step(cuda, monkeypatch, prec):
    from mx_rcnn_amd.ops import precision
    b = {k: v.to(cuda) for k, v in _batch(224, 320).items()}

    def run(fused):
        monkeypatch.setenv('MXR_FUSED_FC_SGD', '1' if fused else '0')
        torch.manual_seed(0)
        m = FasterRCNN('vgg16', 21, cfg=_cfg())
        tr = Trainer(m, 'e2e', fixed_param_prefix=['conv1', 'conv2'], lr=0.01, device=cuda, precision=prec)
        assert sorted(tr.fused_fc_sgd) == (['fc6_weight', 'fc7_weight'] if fused else [])
        for i in range(2):
            torch.manual_seed(10 + i)
            tr.step(b)
        torch.cuda.synchronize()
        for gi, g in enumerate(tr.store.groups):
            if g.x2:
                parts = precision.split(g.master, g.x2)
                for k in range(g.x2):
                    assert torch.equal(g.shadow[k * g.plane:k * g.plane + g.numel],
                                       parts[k * g.numel:(k + 1) * g.numel]), (prec, fused, k)
            elif g.shadow is not None:
                assert torch.equal(g.shadow, g.master.to(g.shadow.dtype)), (prec, fused)
            for sp in tr.store._fused.get(gi, ()):  # the fused gradients were never written
                assert not bool(g.grad[sp['off']:sp['off'] + sp['numel']].any())
        return tr.store.state_arrays(), tr.store.optimizer_state()

    w1, m1 = run(True)
    w0, m0 = run(False)
    for k in w0:
        assert torch.allclose(w1[k], w0[k], rtol=1e-3, atol=1e-5), k
    for k in ('fc6_weight', 'fc7_weight'):
        scale = m0[k].abs().max().item() + 1e-12
        assert scale > 0, k
        assert (m1[k] - m0[k]).abs().max().item() <= 2e-2 * scale, k
