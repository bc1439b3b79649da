"""Precision contract of the headline path: one ResNet-50 training step on the bf16 HIP path vs
the fp32 CPU path from identical weights and identical (deterministic) samples.

* RPN mode on a 192x288 image with RPN_BATCH_SIZE 1024 > the labelled anchors, so the anchor
  subsampling keeps every labelled anchor (no RNG): compares rpn_cls_loss / rpn_bbox_loss.
* Fast R-CNN mode with a fixed RoI batch (no proposal sampling): compares cls_loss / bbox_loss.
* Per-parameter gradients: cosine similarity and relative norm over every trainable layer with a
  non-negligible gradient (bf16 activations and weights, fp32 accumulation and fp32 masters on the
  GPU; everything fp32 on the CPU).

Tolerances (stated in BASELINE.md): losses within 3 % relative; for every layer carrying >= 1e-3
of the largest gradient norm: total gradient norm within 5 % and median per-layer norm error
<= 10 %; loss-adjacent layers (rpn_*, cls_score, bbox_pred, bn1): cosine >= 0.97, norm within 5 %.  Deep-layer gradient DIRECTIONS of this random-init
network are chaotic under any rounding (see _check_grads), so only a loose median bound applies.
"""
import copy

import pytest
import torch

from mx_rcnn_amd.config import snapshot
from mx_rcnn_amd.core.trainer import Trainer
from mx_rcnn_amd.models import FasterRCNN

pytestmark = pytest.mark.gpu

FIXED = ['conv0', 'stage1', 'stage2', 'bn_data', 'bn0']


def _cfg():
    cfg = snapshot()
    cfg.TRAIN.BG_THRESH_LO = 0.0
    cfg.END2END = 1
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    cfg.TRAIN.RPN_BATCH_SIZE = 1024  # the largest the sampling kernel takes: keeps every labelled anchor here
    return cfg


def _image(H=192, W=288, seed=0):
    g = torch.Generator().manual_seed(seed)
    gt = torch.tensor([[[15., 18., 105., 135., 3.], [90., 30., 255., 165., 17.], [150., 105., 270., 180., 9.]]])
    return {'data': torch.randn(1, 3, H, W, generator=g) * 50, 'im_info': torch.tensor([[float(H), float(W), 1.0]]),
            'gt_boxes': gt, 'n_gt': torch.tensor([3], dtype=torch.int32)}, g


def _rcnn_batch(num_classes=21):
    b, g = _image(seed=1)
    R = 128
    x1 = torch.rand(R, generator=g) * 200
    y1 = torch.rand(R, generator=g) * 120
    wh = torch.rand(R, 2, generator=g) * 60 + 16
    rois = torch.stack([torch.zeros(R), x1, y1, x1 + wh[:, 0], y1 + wh[:, 1]], 1)
    label = torch.zeros(R, dtype=torch.int32)
    label[:32] = torch.randint(1, num_classes, (32,), generator=g).to(torch.int32)
    tgt = torch.zeros(R, 4 * num_classes)
    inside = torch.zeros(R, 4 * num_classes)
    for r in range(32):
        c = int(label[r])
        tgt[r, 4 * c:4 * c + 4] = torch.randn(4, generator=g) * 0.5
        inside[r, 4 * c:4 * c + 4] = 1.0
    return {'data': b['data'], 'rois': rois, 'label': label, 'bbox_target': tgt, 'bbox_inside_weight': inside,
            'bbox_outside_weight': inside.clone()}


def _pair(mode, cuda, precision='bf16'):
    torch.manual_seed(0)
    m = FasterRCNN('resnet50', 21, cfg=_cfg(), train_mode=mode)
    b, _ = _image()
    m.calibrate_bn(b['data'])  # frozen statistics from the data (stand-in for pretrained ones)
    m_gpu = copy.deepcopy(m)
    cpu = Trainer(m, mode, fixed_param_prefix=FIXED, lr=0.0, device='cpu')
    gpu = Trainer(m_gpu, mode, fixed_param_prefix=FIXED, lr=0.0, device=cuda, precision=precision)
    return cpu, gpu


def _fwd_bwd(tr, batch):
    from mx_rcnn_amd.ops.precision import x2_mode
    tr.model.train()
    tr.store.zero_grad()
    tr.reducer.prepare()
    with x2_mode(getattr(tr, 'x2', False)):
        out = tr.forward(tr.prepare_batch(batch))
        out['loss'].backward()
    tr.reducer.finish()
    if tr.device.type == 'cuda':
        torch.cuda.synchronize()
    grads = {n: p.grad.detach().float().cpu().flatten() for n, p in tr.store.params.items()
             if p.requires_grad and p.grad is not None}
    return out, grads


NEAR = ('rpn_', 'cls_score_', 'bbox_pred_', 'bn1_')  # layers adjacent to a loss


def _check_grads(gc, gg, median_floor):
    """Loss-adjacent layers: cosine >= 0.97 and norm within 5 %.  All non-negligible layers together:
    total gradient norm within 5 %, median per-layer norm error <= 10 %.
    Median cosine over all layers >= ``median_floor``, set 0.05 below the bf16-STORAGE floor: exact
    fp32 arithmetic with bf16-rounded inputs, weights, layer outputs and layer-output gradients gives
    a median cosine of 0.956 (RPN) / 0.521 (R-CNN) vs the fp32 step on this random-init network
    (deep-layer gradient directions are chaotic under any rounding); the HIP bf16 path measures
    0.962 / 0.563, i.e. it loses nothing beyond bf16 storage (tools/parity_probe.py,
    profiles/r3_parity_probe.txt).  The fp32-class mode removes the storage loss (the *_fp32_* tests)."""
    norms = {n: float(v.norm()) for n, v in gc.items()}
    big = max(norms.values())
    rows = []
    for n, v in gc.items():
        if norms[n] < 1e-3 * big:
            continue
        w = gg[n]
        cos = float(torch.dot(v, w) / (v.norm() * w.norm() + 1e-30))
        rel = abs(float(w.norm()) - norms[n]) / norms[n]
        rows.append((n, cos, rel))
        if n.startswith(NEAR):
            assert cos >= 0.97 and rel <= 0.05, (n, cos, rel)
    tot_c = sum(norms[n] ** 2 for n, _, _ in rows) ** 0.5
    tot_g = sum(float(gg[n].norm()) ** 2 for n, _, _ in rows) ** 0.5
    assert abs(tot_g - tot_c) <= 0.05 * tot_c, (tot_g, tot_c)
    rels = sorted(r[2] for r in rows)
    assert rels[len(rels) // 2] <= 0.10, rels[-5:]
    cos_all = sorted(r[1] for r in rows)
    print('median cos %.4f over %d layers; worst %s' % (cos_all[len(cos_all) // 2], len(rows),
                                                          sorted(rows, key=lambda r: r[1])[:3]))
    assert cos_all[len(cos_all) // 2] >= median_floor
    assert any(r[0].startswith(NEAR) for r in rows)


def _rel(a, b):
    return abs(float(a) - float(b)) / max(abs(float(b)), 1e-12)


def test_rpn_step_bf16_gpu_matches_fp32_cpu(cuda):
    cpu, gpu = _pair('rpn', cuda)
    b, _ = _image()
    oc, gc = _fwd_bwd(cpu, b)
    og, gg = _fwd_bwd(gpu, b)
    n_lab = int((oc['rpn_label'] >= 0).sum())
    assert 0 < n_lab < 1024, n_lab  # below the RPN batch: no subsampling, identical targets on both paths
    assert torch.equal(og['rpn_label'].cpu(), oc['rpn_label'])
    for k in ('rpn_cls_loss', 'rpn_bbox_loss'):
        assert _rel(og[k].float().cpu().sum(), oc[k].float().sum()) <= 0.03, (k, og[k], oc[k])
    _check_grads(gc, gg, 0.91)


def test_rcnn_step_bf16_gpu_matches_fp32_cpu(cuda):
    cpu, gpu = _pair('rcnn', cuda)
    b = _rcnn_batch()
    oc, gc = _fwd_bwd(cpu, b)
    og, gg = _fwd_bwd(gpu, b)
    for k in ('cls_loss', 'bbox_loss'):
        assert _rel(og[k].float().cpu().sum(), oc[k].float().sum()) <= 0.03, (k, og[k], oc[k])
    _check_grads(gc, gg, 0.47)


def _check_grads_tight(gc, gg, cos_min=0.99, rel_max=0.02, min_layers=10):
    """fp32-class contract: EVERY layer with a non-negligible gradient has cosine >= cos_min and
    norm within rel_max of the fp32 CPU step.  (The R-CNN step's deepest BN betas sit at cosine
    ~0.998 / norm ~1 %: a ReLU whose pre-activation is within rounding of zero flips between ANY
    two fp32 summation orders in this random-init network.)"""
    norms = {n: float(v.norm()) for n, v in gc.items()}
    big = max(norms.values())
    worst = []
    for n, v in gc.items():
        if norms[n] < 1e-3 * big:
            continue
        w = gg[n]
        cos = float(torch.dot(v, w) / (v.norm() * w.norm() + 1e-30))
        rel = abs(float(w.norm()) - norms[n]) / norms[n]
        worst.append((cos, rel, n))
        assert cos >= cos_min and rel <= rel_max, (n, cos, rel)
    worst.sort()
    print('fp32 mode: %d layers, worst cosine %s' % (len(worst), worst[:3]))
    assert len(worst) >= min_layers


# (precision, loss tolerance, per-layer cosine floor, per-layer norm error, median cosine floor)
# fp32: exact fp32 triples, six products -- the reference's precision; bf16x3: 16-bit pairs.
# The R-CNN step's per-layer floor is looser than its median: a ReLU whose pre-activation lies
# within rounding of zero flips between ANY two fp32 summation orders of this random-init network,
# which moves a few deep BN betas' directions (see _check_grads_tight).
RPN_TIGHT = {'fp32': (1e-4, 0.9999, 0.002, 0.99999), 'bf16x3': (1e-3, 0.99, 0.02, 0.999)}
RCNN_TIGHT = {'fp32': (1e-4, 0.995, 0.005, 0.9999), 'bf16x3': (1e-3, 0.99, 0.02, 0.99)}


def _median_cos(gc, gg):
    norms = {n: float(v.norm()) for n, v in gc.items()}
    big = max(norms.values())
    cs = sorted(float(torch.dot(v, gg[n]) / (v.norm() * gg[n].norm() + 1e-30))
                for n, v in gc.items() if norms[n] >= 1e-3 * big)
    return cs[len(cs) // 2]


@pytest.mark.parametrize('prec', ['fp32', 'bf16x3'])
def test_rpn_step_fp32_gpu_matches_fp32_cpu(cuda, prec):
    """The multi-plane GPU modes against the fp32 CPU step (the bf16 mode's deep layers fall to a
    median cosine of ~0.9 here)."""
    loss_tol, cos_min, rel_max, med_min = RPN_TIGHT[prec]
    cpu, gpu = _pair('rpn', cuda, prec)
    b, _ = _image()
    oc, gc = _fwd_bwd(cpu, b)
    og, gg = _fwd_bwd(gpu, b)
    assert torch.equal(og['rpn_label'].cpu(), oc['rpn_label'])
    for k in ('rpn_cls_loss', 'rpn_bbox_loss'):
        assert _rel(og[k].float().cpu().sum(), oc[k].float().sum()) <= loss_tol, (k, og[k], oc[k])
    _check_grads_tight(gc, gg, cos_min, rel_max)
    med = _median_cos(gc, gg)
    print('%s rpn: median cosine %.7f' % (prec, med))
    assert med >= med_min


@pytest.mark.parametrize('prec', ['fp32', 'bf16x3'])
def test_rcnn_step_fp32_gpu_matches_fp32_cpu(cuda, prec):
    loss_tol, cos_min, rel_max, med_min = RCNN_TIGHT[prec]
    cpu, gpu = _pair('rcnn', cuda, prec)
    b = _rcnn_batch()
    oc, gc = _fwd_bwd(cpu, b)
    og, gg = _fwd_bwd(gpu, b)
    for k in ('cls_loss', 'bbox_loss'):
        assert _rel(og[k].float().cpu().sum(), oc[k].float().sum()) <= loss_tol, (k, og[k], oc[k])
    _check_grads_tight(gc, gg, cos_min, rel_max)
    med = _median_cos(gc, gg)
    print('%s rcnn: median cosine %.7f' % (prec, med))
    assert med >= med_min
