"""Model families, parameter naming (SURVEY §2.12 counts), trainer step on CPU."""
import math
import pytest
import torch

from mx_rcnn_amd.config import snapshot
from mx_rcnn_amd.models import FasterRCNN
from mx_rcnn_amd.core.trainer import Trainer


def _cfg():
    cfg = snapshot()
    cfg.TRAIN.BG_THRESH_LO = 0.0
    cfg.END2END = 1
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    cfg.TRAIN.RPN_PRE_NMS_TOP_N = 800
    cfg.TRAIN.RPN_POST_NMS_TOP_N = 300
    return cfg


def test_param_counts_match_reference():
    m = FasterRCNN('vgg16', 21, cfg=_cfg())
    a = m.arg_params()
    assert len(a) == 40 and sum(v.numel() for v in a.values()) == 137078239
    shapes = m.arg_shapes()  # checkpoint layout: fc6 is held as the (4096, 512, 7, 7) filter of its rows
    assert shapes['fc6_weight'] == (4096, 25088) and a['fc6_weight'].shape == (4096, 512, 7, 7)
    assert shapes['rpn_cls_score_weight'] == (18, 512, 1, 1) == tuple(a['rpn_cls_score_weight'].shape)
    r = FasterRCNN('resnet101', 21, cfg=_cfg())
    assert len(r.arg_params()) == 318 and len(r.aux_params()) == 204
    assert sum(v.numel() for v in r.arg_params().values()) == 47463799
    r50 = FasterRCNN('resnet50', 21, cfg=_cfg())
    assert len(r50.arg_params()) == 165 and len(r50.aux_params()) == 102
    assert 'stage3_unit6_bn3_gamma' in r50.arg_params() and 'bn1_moving_var' in r50.aux_params()
    assert r.arg_params()['rpn_cls_score_weight'].shape[0] == 24


@pytest.mark.parametrize('net', ['resnet18', 'resnet34', 'resnet152'])
def test_other_depths_build(net):
    m = FasterRCNN(net, 2, cfg=_cfg())
    assert m.num_anchors == 12
    assert m.feat_shape(800, 1333) == (50, 84)


def _batch(H=160, W=224):
    gt = torch.tensor([[[10., 20., 80., 100., 3.], [50., 60., 150., 140., 7.], [-1, -1, -1, -1, -1]]])
    return {'data': torch.randn(1, 3, H, W) * 50, 'im_info': torch.tensor([[float(H), float(W), 1.0]]),
            'gt_boxes': gt, 'n_gt': torch.tensor([2], dtype=torch.int32)}


def test_vgg_e2e_loss_decreases_cpu():
    torch.manual_seed(0)
    cfg = _cfg()
    m = FasterRCNN('vgg16', 21, cfg=cfg)
    m.head.dropout = 0.0
    tr = Trainer(m, 'e2e', fixed_param_prefix=['conv1', 'conv2'], lr=0.002, device='cpu')
    b = _batch()
    outs = [tr.step(b) for _ in range(6)]
    assert all(torch.isfinite(o['loss']) for o in outs)
    # the sampled RoIs change every step, so compare the smooth parts of the objective
    for k in ('rpn_cls_loss', 'rpn_bbox_loss', 'cls_loss'):
        assert float(outs[-1][k]) < float(outs[0][k]), k


def test_resnet_rpn_and_rcnn_modes_cpu():
    torch.manual_seed(1)
    cfg = _cfg()
    m = FasterRCNN('resnet18', 21, cfg=cfg)
    tr = Trainer(m, 'rpn', fixed_param_prefix=['conv0', 'stage1'], device='cpu')
    out = tr.step(_batch())
    assert torch.isfinite(out['loss'])
    rois = torch.tensor([[0., 10, 20, 80, 100], [0., 30, 30, 90, 120]])
    rb = {'data': _batch()['data'], 'rois': rois, 'label': torch.tensor([3, 0], dtype=torch.int32),
          'bbox_target': torch.zeros(2, 84), 'bbox_inside_weight': torch.zeros(2, 84),
          'bbox_outside_weight': torch.zeros(2, 84)}
    tr2 = Trainer(m, 'rcnn', fixed_param_prefix=['conv0'], device='cpu')
    out = tr2.step(rb)
    assert torch.isfinite(out['loss'])
    m.eval()
    r, p, bb = m.detect(_batch()['data'], _batch()['im_info'])
    assert r.shape[1] == 5 and p.shape[1] == 21 and bb.shape[1] == 84


def test_frozen_prefix_substring_semantics():
    m = FasterRCNN('resnet18', 21, cfg=_cfg())
    tr = Trainer(m, 'e2e', fixed_param_prefix=['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'], device='cpu')
    assert 'conv0_weight' in tr.store.fixed_names
    assert 'stage3_unit1_conv1_weight' not in tr.store.fixed_names
    assert not tr.store.params['stage1_unit1_conv1_weight'].requires_grad
    assert tr.store.params['stage3_unit1_conv1_weight'].requires_grad


@pytest.mark.gpu
def test_e2e_step_gpu_graph(cuda):
    from mx_rcnn_amd.core.trainer import GraphedStep
    torch.manual_seed(0)
    cfg = _cfg()
    m = FasterRCNN('resnet50', 21, cfg=cfg)
    tr = Trainer(m, 'e2e', fixed_param_prefix=['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'], device=cuda)
    b = {k: v.to(cuda) for k, v in _batch(320, 480).items()}
    out = tr.step(b)
    torch.cuda.synchronize()
    assert torch.isfinite(out['loss'])
    g = GraphedStep(tr, b, warmup=2)
    for _ in range(3):
        o = g(b)
    torch.cuda.synchronize()
    assert torch.isfinite(o['loss'])


@pytest.mark.gpu
@pytest.mark.parametrize('prec', ['bf16', 'bf16x3', 'fp32'])
def test_overlapped_sgd_matches_end_of_step_sgd(cuda, monkeypatch, prec):
    """Bucket-by-bucket SGD under the backward pass (MXR_OVERLAP_SGD=1, parallel/reducer.py) gives the same weights
    and momenta as one update after the backward (MXR_OVERLAP_SGD=0), in every storage mode: the
    multi-plane stores update bucket slices at unpadded offsets with plane_stride, and
    their shadow planes must stay the exact split of the masters."""
    from mx_rcnn_amd.ops import precision
    fixed = ['conv0', 'stage1', 'stage2', 'bn_data', 'bn0']
    b = {k: v.to(cuda) for k, v in _batch(320, 480).items()}

    def run(overlap):
        monkeypatch.setenv('MXR_OVERLAP_SGD', '1' if overlap else '0')
        torch.manual_seed(0)
        m = FasterRCNN('resnet50', 21, cfg=_cfg())
        tr = Trainer(m, 'e2e', fixed_param_prefix=fixed, lr=0.01, device=cuda, precision=prec)
        assert tr.reducer.sgd_capable == overlap
        for i in range(2):
            torch.manual_seed(10 + i)
            tr.step(b)
        assert tr.reducer.sgd_applied == overlap
        torch.cuda.synchronize()
        for g in tr.store.groups:
            if g.x2:
                parts = precision.split(g.master, g.x2)
                for k in range(g.x2):
                    assert torch.equal(g.shadow[k * g.plane:k * g.plane + g.numel],
                                       parts[k * g.numel:(k + 1) * g.numel]), (prec, overlap, k)
        return tr.store.state_arrays(), tr.store.optimizer_state()

    w1, m1 = run(True)
    w0, m0 = run(False)
    for k in w0:
        assert torch.allclose(w1[k], w0[k], rtol=1e-3, atol=1e-5), k
    for k in m0:
        scale = m0[k].abs().max().item() + 1e-12
        assert (m1[k] - m0[k]).abs().max().item() <= 2e-2 * scale + 1e-7, k


@pytest.mark.gpu
def test_side_stream_grad_clear_matches_inline(cuda, monkeypatch):
    """Clearing the flat gradients on the dgrad-cache side stream (MXR_ZERO_GRAD_SIDE=1, joined
    before the first backward kernel) trains exactly like clearing them on the compute stream
    before the forward pass, eager and graph-replayed."""
    from mx_rcnn_amd.core.trainer import GraphedStep
    fixed = ['conv0', 'stage1', 'stage2', 'bn_data', 'bn0']
    b = {k: v.to(cuda) for k, v in _batch(320, 480).items()}

    def run(side):
        monkeypatch.setenv('MXR_ZERO_GRAD_SIDE', '1' if side else '0')
        torch.manual_seed(0)
        m = FasterRCNN('resnet50', 21, cfg=_cfg())
        tr = Trainer(m, 'e2e', fixed_param_prefix=fixed, lr=0.01, device=cuda)
        torch.manual_seed(10)
        tr.step(b)
        g = GraphedStep(tr, b, warmup=1)
        for _ in range(2):
            g(b)
        torch.cuda.synchronize()
        return tr.store.state_arrays(), [gr.grad.float().clone() for gr in tr.store.groups]

    w1, g1 = run(True)
    w0, g0 = run(False)
    for k in w0:
        assert torch.allclose(w1[k], w0[k], rtol=1e-3, atol=1e-5), k
    for a, c in zip(g1, g0):
        scale = c.abs().max().item() + 1e-12
        assert (a - c).abs().max().item() <= 2e-2 * scale + 1e-7


@pytest.mark.gpu
@pytest.mark.parametrize('precision', ['bf16', 'fp32'])
def test_flip_kernel_writes_parity_sub_filters(cuda, precision):
    """After the first backward registers the strided data gradient's parity sub-filters, the
    multi-filter flip kernel writes them in its own pass: every sub-filter equals its slice of the
    flipped filter after later updates, and the copy path is skipped for them (fp32-class pairs:
    one table entry per plane writes that plane's half of the pair sub-filter)."""
    from mx_rcnn_amd.ops import conv as conv_ops
    torch.manual_seed(0)
    m = FasterRCNN('resnet50', 21, cfg=_cfg())
    tr = Trainer(m, 'e2e', fixed_param_prefix=['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'], lr=0.01, device=cuda,
                 precision=precision)
    b = {k: v.to(cuda) for k, v in _batch(320, 480).items()}
    for _ in range(3):
        tr.step(b)
    torch.cuda.synchronize()
    assert tr.store._sub_in_table, 'no parity sub-filter was folded into the flip table'
    tr.store.refresh_dgrad_cache()
    torch.cuda.synchronize()
    checked = 0
    for p, view, buf in conv_ops.sub_filter_entries():
        if id(p) not in tr.store._sub_in_table:
            continue
        wf = conv_ops.cached_dgrad_weight(p)
        assert torch.equal(buf, view(wf).contiguous(memory_format=torch.channels_last))
        checked += 1
    assert checked >= 4


@pytest.mark.gpu
def test_graph_capture_has_no_training_side_effects(cuda):
    """GraphedStep's warm-up runs real steps to settle workspaces; weights, momentum, bf16
    shadows and BN moving statistics must be exactly as before the capture (a new shape must
    not apply unscheduled SGD updates), and replaying then trains like eager steps."""
    from mx_rcnn_amd.core.trainer import GraphedStep
    torch.manual_seed(0)
    m = FasterRCNN('resnet50', 21, cfg=_cfg())
    tr = Trainer(m, 'e2e', fixed_param_prefix=['conv0', 'stage1', 'stage2', 'bn_data', 'bn0'], lr=0.01, device=cuda)
    b = {k: v.to(cuda) for k, v in _batch(320, 480).items()}
    tr.step(b)
    torch.cuda.synchronize()
    before = tr.snapshot_state()
    GraphedStep(tr, b, warmup=3)
    torch.cuda.synchronize()
    for g, (mst, mom, sh) in zip(tr.store.groups, before['groups']):
        assert torch.equal(g.master, mst) and torch.equal(g.mom, mom)
        assert sh is None or torch.equal(g.shadow, sh)
    for buf, v in zip(tr.model.buffers(), before['buffers']):
        assert torch.equal(buf, v)


@pytest.mark.gpu
def test_vgg16_e2e_step_gpu_graph(cuda):
    """VGG16 end-to-end step on the GPU path (MFMA convs, HIP max-pool, fused FC + ReLU + dropout)
    eager then graph-replayed: finite loss, and dropout draws a new mask every update."""
    from mx_rcnn_amd.core.trainer import GraphedStep
    torch.manual_seed(0)
    m = FasterRCNN('vgg16', 21, cfg=_cfg())
    tr = Trainer(m, 'e2e', fixed_param_prefix=['conv1', 'conv2'], lr=0.001, device=cuda)
    b = {k: v.to(cuda) for k, v in _batch(320, 480).items()}
    out = tr.step(b)
    torch.cuda.synchronize()
    assert torch.isfinite(out['loss'])
    g = GraphedStep(tr, b, warmup=2)
    losses = []
    for _ in range(3):
        o = g(b)
        losses.append(float(o['loss'].float().item()))
    assert all(math.isfinite(v) for v in losses)
    assert int(tr.rng_step.item()) == tr.num_update


def _det_setup(net):
    """A random-init test-graph model with BN statistics / filter scales that keep activations O(1),
    its input and 64 fixed RoIs."""
    torch.manual_seed(0)
    m = FasterRCNN(net, 21, cfg=_cfg(), train_mode='test')
    g = torch.Generator().manual_seed(1)
    data = torch.randn(1, 3, 224, 320, generator=g) * 50
    if net.startswith('resnet'):
        m.calibrate_bn(data)
    else:  # He init keeps a BN-free VGG's activations O(1) (the 0.01-std init shrinks them into fp16 subnormals)
        with torch.no_grad():
            for c in m.trunk.convs:
                c.weight.normal_(0, (2.0 / (c.weight[0].numel())) ** 0.5, generator=g)
            data = data / 50.0
    with torch.no_grad():
        m.head.cls_score.weight.normal_(0, 0.05, generator=g)
        m.head.bbox_pred.weight.normal_(0, 0.05, generator=g)
    info = torch.tensor([[224., 320., 1.0]])
    x1 = torch.rand(64, generator=g) * 250
    y1 = torch.rand(64, generator=g) * 150
    rois = torch.stack([torch.zeros(64), x1, y1, x1 + 60, y1 + 60], 1)
    return m, data, info, rois


@pytest.mark.gpu
@pytest.mark.parametrize('net', ['resnet50', 'vgg16'])
def test_fp16_inference_matches_fp32(cuda, net):
    """The fp16 test graph (MFMA f16 convs / FC, fp16 BN, pooling, RoIPool) vs the fp32 graph on
    fixed RoIs: fp16 keeps 3 more mantissa bits than bf16, so with activations inside fp16's range it
    must land closer to fp32."""
    from mx_rcnn_amd.core.detector import Detector
    m, data, info, rois = _det_setup(net)
    outs = {}
    for name, dt in (('fp32', torch.float32), ('bf16', torch.bfloat16), ('fp16', torch.float16)):
        det = Detector(m, cuda, compute_dtype=dt)
        _, prob, box = det.forward(data, info, rois)
        outs[name] = (prob.float().cpu(), box.float().cpu())
    ref_p, ref_b = outs['fp32']

    def err(k):
        p, b = outs[k]
        return ((p - ref_p).abs().max().item(), ((b - ref_b).norm() / ref_b.norm()).item())
    e16, eb = err('fp16'), err('bf16')
    assert e16[0] <= 0.02 and e16[1] <= 0.02, e16
    assert e16[1] <= eb[1], (e16, eb)


@pytest.mark.gpu
@pytest.mark.parametrize('net', ['resnet50', 'vgg16'])
def test_fp32_detector_on_mfma_kernels_matches_torch_fp32(cuda, net, monkeypatch):
    """Detector(compute_dtype='fp32') runs the test graph in the three-plane mode on our kernels
    (F.conv2d / F.linear / vendor GEMM routes are made to raise while it runs), matches the plain
    fp32 PyTorch arm (MXR_FP32_EVAL=torch) to fp32 rounding, with RPN proposals and with fixed RoIs,
    and leaves the model it was built from untouched (its own weight copy; ADVICE r5 / VERDICT r5)."""
    import torch.nn.functional as Fn
    from mx_rcnn_amd.core.detector import Detector
    m, data, info, rois = _det_setup(net)
    m.to(cuda)
    before = {k: v.detach().clone() for k, v in m.state_dict().items()}
    Detector(m, cuda, compute_dtype='bf16')  # a low-precision detector must not convert m either
    monkeypatch.setenv('MXR_FP32_EVAL', 'torch')
    ref = Detector(m, cuda, compute_dtype='fp32')
    r_fixed = [t.float().cpu() for t in ref.forward(data, info, rois)]
    r_rpn = [t.float().cpu() for t in ref.forward(data, info)]
    monkeypatch.delenv('MXR_FP32_EVAL')
    det = Detector(m, cuda, compute_dtype='fp32')
    assert det.planes == 3

    def boom(*a, **k):
        raise AssertionError('vendor conv / GEMM fallback in the fp32 test graph')
    monkeypatch.setattr(Fn, 'conv2d', boom)
    monkeypatch.setattr(Fn, 'linear', boom)
    monkeypatch.setattr(torch, '_addmm_activation', boom)
    got_fixed = [t.float().cpu() for t in det.forward(data, info, rois)]
    got_rpn = [t.float().cpu() for t in det.forward(data, info)]
    torch.cuda.synchronize()
    monkeypatch.undo()
    assert torch.equal(got_fixed[0], r_fixed[0])
    assert (got_fixed[1] - r_fixed[1]).abs().max().item() <= 1e-4, (got_fixed[1] - r_fixed[1]).abs().max().item()
    rel = ((got_fixed[2] - r_fixed[2]).norm() / r_fixed[2].norm()).item()
    assert rel <= 1e-4, rel
    # RPN proposals: near-tied scores may order differently under another fp32 summation order, so
    # compare the proposal sets (most boxes shared) rather than rows
    assert got_rpn[0].shape == r_rpn[0].shape and bool(torch.isfinite(got_rpn[1]).all())
    a = {tuple(v) for v in (got_rpn[0][:, 1:] * 4).round().tolist()}
    b = {tuple(v) for v in (r_rpn[0][:, 1:] * 4).round().tolist()}
    assert len(a & b) >= 0.9 * len(b), (len(a & b), len(b))
    for k, v in m.state_dict().items():
        assert v.dtype == before[k].dtype and torch.equal(v, before[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', ['bf16', 'fp32'])
def test_pool_post_bn_fusion_keeps_detections(cuda, dtype, monkeypatch):
    """The inference fusions of stage1_unit1_bn1 into pool0 and stage4_unit1_bn1 into the RoI pooling
    (ops/pool.py post_bn_ok) leave the detector's outputs unchanged: bit for bit in bf16, to fp32
    rounding in the three-plane fp32 mode; and the fused kernels do run (no bn_relu_fwd launch)."""
    from mx_rcnn_amd.core.detector import Detector
    from mx_rcnn_amd.ops import need_ext
    m, data, info, rois = _det_setup('resnet50')
    outs = {}
    for flag in ('0', '1'):
        monkeypatch.setenv('MXR_POOL_POST_BN', flag)
        det = Detector(m, cuda, compute_dtype=dtype)
        ext = need_ext()
        calls = []
        real = ext.bn_relu_fwd
        monkeypatch.setattr(ext, 'bn_relu_fwd', lambda *a, **k: calls.append(1) or real(*a, **k))
        outs[flag] = ([t.float().cpu() for t in det.forward(data, info, rois)],
                      [t.float().cpu() for t in det.forward(data, info)], len(calls))
        monkeypatch.setattr(ext, 'bn_relu_fwd', real)
    (f0, r0, n0), (f1, r1, n1) = outs['0'], outs['1']
    assert n0 >= 4 and n1 == 0, (n0, n1)  # pool0 + RoI pooling, per forward
    for a, b in zip(f0 + r0, f1 + r1):
        if dtype == 'bf16':
            assert torch.equal(a, b)
        else:
            assert torch.allclose(a, b, atol=1e-4, rtol=1e-4), (a - b).abs().max().item()


def test_unit_seed_backward_matches_default():
    """A backward seeded with ops._ext.unit_grad (loss ops skip their scale-by-1) gives the same
    gradients as the default seed, and a non-unit seed still scales."""
    from mx_rcnn_amd.ops._ext import unit_grad
    from mx_rcnn_amd.ops.losses import combine_losses, smooth_l1, softmax_ce
    g = torch.Generator().manual_seed(3)
    pred0 = torch.randn(16, 8, generator=g)
    logits0 = torch.randn(16, 5, generator=g)
    tgt = torch.randn(16, 8, generator=g)
    w = torch.ones(16, 8)
    lab = torch.randint(0, 5, (16,), generator=g)

    def grads(seed):
        pred = pred0.clone().requires_grad_()
        logits = logits0.clone().requires_grad_()
        l1 = smooth_l1(pred, tgt, w, w, sigma=1.0, grad_scale=0.5, slot=2)
        ce, _ = softmax_ce(logits, lab)
        loss, _ = combine_losses([l1, ce], [1.0, 1.0])
        loss.backward(seed)
        return pred.grad.clone(), logits.grad.clone()

    a = grads(unit_grad(torch.device('cpu')))
    b = grads(torch.ones(()))
    c = grads(torch.full((), 2.0))
    for x, y, z in zip(a, b, c):
        assert torch.equal(x, y)
        assert torch.allclose(z, 2 * y)


def test_fused_gradient_clear_matches_fill_cpu():
    """The update zeroes the gradients it consumed (Trainer.fused_clear) instead of a fill at the
    next step's start: three rcnn-mode steps give the same weights either way, the buffers are
    zero after each fused step, and a step after the step API (gradients left written) clears."""
    rois = torch.tensor([[0., 10, 20, 80, 100], [0., 30, 30, 90, 120]])
    rb = {'data': _batch()['data'], 'rois': rois, 'label': torch.tensor([3, 0], dtype=torch.int32),
          'bbox_target': torch.zeros(2, 84), 'bbox_inside_weight': torch.zeros(2, 84),
          'bbox_outside_weight': torch.zeros(2, 84)}
    outs = []
    for fused in (True, False):
        torch.manual_seed(2)
        m = FasterRCNN('resnet18', 21, cfg=_cfg())
        tr = Trainer(m, 'rcnn', fixed_param_prefix=['conv0'], lr=0.01, device='cpu')
        tr.fused_clear = fused
        for _ in range(3):
            tr.step(rb)
            if fused:
                assert not tr.grads_dirty and all(not g.any() for g in tr.store.grad_buffers())
        outs.append([g.master.clone() for g in tr.store.groups])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # dirty buffers (e.g. the forward / backward / update API) are cleared by the next step
    tr.grads_dirty = True
    for g in tr.store.grad_buffers():
        g.fill_(1e3)
    tr.fused_clear = True
    before = [g.master.clone() for g in tr.store.groups]
    tr.step(rb)
    assert all(float((g.master - b).abs().max()) < 1.0 for g, b in zip(tr.store.groups, before))


def test_linear_in_shape_layout_cpu():
    """Linear(in_shape=(C, H, W)) (VGG fc6): the weight is the (cout, C, H, W) filter of the MXNet
    (cout, C*H*W) matrix -- same logical elements, so loading a checkpoint matrix and flattening
    (C, H, W) inputs gives the plain FullyConnected result; the checkpoint shape stays 2-D."""
    from mx_rcnn_amd.models.layers import Linear
    torch.manual_seed(3)
    lin = Linear('fc6', 8 * 7 * 7, 16, in_shape=(8, 7, 7))
    assert lin.weight.shape == (16, 8, 7, 7) and lin.mx_arg_shapes()['fc6_weight'] == (16, 392)
    w2 = torch.randn(16, 392)
    with torch.no_grad():
        lin.weight.copy_(w2.reshape(lin.weight.shape))  # the loader's reshape
    x = torch.randn(5, 8, 7, 7)
    ref = x.reshape(5, -1) @ w2.t() + lin.bias
    assert torch.allclose(lin(x), ref, atol=1e-5)
    # held channels_last (the parameter store's layout): rows of the channels_last map match
    wcl = lin.weight.detach().contiguous(memory_format=torch.channels_last)
    rows_w = wcl.permute(0, 2, 3, 1).reshape(16, -1)
    rows_x = x.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(5, -1)
    assert torch.allclose(rows_x @ rows_w.t() + lin.bias, ref, atol=1e-5)


def test_inference_copy_leaves_the_trained_model_untouched():
    """core/detector.py _inference_copy (what a GPU Detector runs): a private copy of the model's
    weights in the test precision; the model it came from keeps its dtype, values and the trainer's
    attachments (dropout counter, non-finite counter), and the copy carries none of them."""
    from mx_rcnn_amd.core.detector import _inference_copy, resolve_dtype
    torch.manual_seed(0)
    m = FasterRCNN('vgg16', 21, cfg=_cfg())
    tr = Trainer(m, 'e2e', fixed_param_prefix=['conv1', 'conv2'], device='cpu')
    before = {k: v.clone() for k, v in m.state_dict().items()}
    c = _inference_copy(m, resolve_dtype('bf16'))
    assert c is not m and not c.training
    assert c.trunk.convs[3].weight.dtype == torch.bfloat16 and c.head.fc6.weight.dtype == torch.bfloat16
    assert c.trunk.convs[3].weight.is_contiguous(memory_format=torch.channels_last)
    assert c.head.fc6.rng_step is None and c.nonfinite_counter is None
    assert m.head.fc6.rng_step is tr.rng_step and m.nonfinite_counter is tr.nonfinite
    for k, v in m.state_dict().items():
        assert v.dtype == before[k].dtype and torch.equal(v, before[k]), k
    with pytest.raises(ValueError):
        resolve_dtype('int8')
