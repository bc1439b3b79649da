"""Host-side caches derived from parameters must never outlive or outsmart their parameter.

Round 4's driver GPU suite failed on a stem packed-filter cache keyed by ``id(weight)``: a freed
filter's id / address / version were reused by the next one and the stale packing was served
(`ops/stem.py`).  These CPU tests pin the fixes: packings stored on the tensor itself, a reload
epoch for ``.data`` writes, weakly held dgrad caches and per-parameter gradient hooks, and dead
trainers that are actually freed (bench.py builds three in one process).
"""
import gc
import weakref

import pytest
import torch

from mx_rcnn_amd.ops import conv as conv_ops
from mx_rcnn_amd.ops import grad_sink, precision
from mx_rcnn_amd.ops.stem import _packed_filter, pack_filter


def _expected(w, dtype, planes):
    if dtype != torch.float32:
        return pack_filter(w, dtype)
    pf = precision.split(pack_filter(w, torch.float32), planes)
    if planes == 3:
        pf = torch.cat([pf[64:128], pf[:64], pf[128:]], 0)
    return pf


@pytest.mark.parametrize('dtype,planes', [(torch.float16, 0), (torch.bfloat16, 0), (torch.float32, 2),
                                          (torch.float32, 3)])
def test_stem_packing_never_stale_across_reallocation(dtype, planes):
    """Allocate, pack, free and re-allocate same-shape filters: every packing is of the live one
    (the id()-keyed cache returned a stale packing ~half the time here)."""
    g = torch.Generator().manual_seed(0)
    with precision.x2_mode(planes):
        for i in range(50):
            w = torch.randn(64, 3, 7, 7, generator=g).to(dtype if dtype != torch.float32 else torch.float32)
            got = _packed_filter(w, dtype)
            assert torch.equal(got, _expected(w, dtype, planes)), 'stale packing at iteration %d' % i
            del w, got


def test_stem_packing_follows_data_reload():
    """``p.data.copy_`` does not move the version counter: forget_weight's reload epoch must, and
    the rebuild is in place (a captured graph keeps reading the live buffer)."""
    p = torch.nn.Parameter(torch.randn(64, 3, 7, 7).half())
    a = _packed_filter(p, torch.float16)
    assert _packed_filter(p, torch.float16) is a  # cached
    new = torch.randn(64, 3, 7, 7).half()
    p.data.copy_(new)
    precision.forget_weight(p)
    b = _packed_filter(p, torch.float16)
    assert b is a, 'rebuild must reuse the buffer'
    assert torch.equal(b, pack_filter(new, torch.float16))
    # an ordinary in-place write moves the version counter by itself
    with torch.no_grad():
        p.mul_(2)
    assert torch.equal(_packed_filter(p, torch.float16), pack_filter(p, torch.float16))


def test_packing_dies_with_its_parameter():
    p = torch.nn.Parameter(torch.randn(64, 3, 3, 3))
    ref = weakref.ref(_packed_filter(p, torch.bfloat16))
    del p
    gc.collect()
    assert ref() is None


def test_dgrad_caches_hold_parameters_weakly():
    p = torch.nn.Parameter(torch.randn(64, 64, 3, 3))
    buf = torch.empty(64, 64, 3, 3)
    conv_ops.register_dgrad_weight(p, buf)
    assert conv_ops.cached_dgrad_weight(p) is buf
    wf = conv_ops.cached_dgrad_weight(p)
    conv_ops.sub_filter(p, wf, [0, 2], [0, 2], 2)
    assert len(conv_ops.sub_filters_of(p)) == 1
    pref, pid = weakref.ref(p), id(p)
    del p, wf
    gc.collect()
    assert pref() is None, 'the dgrad cache pinned its parameter'
    assert pid not in conv_ops._DGRAD_W
    assert not [k for k in conv_ops._SUBW if k[0] == pid]


def test_grad_hooks_live_on_the_parameter():
    p = torch.nn.Parameter(torch.randn(4))
    fired = []
    grad_sink.add_hook(p, lambda _p: fired.append('old'))
    grad_sink.clear_hooks([p])
    grad_sink.add_hook(p, lambda _p: fired.append('new'))
    grad_sink.delivered(p)
    assert fired == ['new']
    q = torch.nn.Parameter(torch.randn(4))
    grad_sink.delivered(q)  # nothing registered: no-op
    assert grad_sink.target(q) is None
    grad_sink.enable_direct(q)
    grad_sink.enable_direct(q)  # idempotent: one engine hook
    q.grad = torch.zeros(4)
    assert grad_sink.target(q) is q.grad


def test_sequential_trainers_are_collectable():
    """bench.py builds fp32, bf16x3 and bf16 trainers in one process: each earlier store (masters,
    momentum, gradients, shadow planes) must be freed when its trainer goes."""
    from mx_rcnn_amd.config import snapshot
    from mx_rcnn_amd.core.trainer import Trainer
    from mx_rcnn_amd.models import FasterRCNN
    refs = []
    for _ in range(3):
        torch.manual_seed(0)
        m = FasterRCNN('resnet18', 6, cfg=snapshot())
        tr = Trainer(m, 'rcnn', fixed_param_prefix=['conv0'], lr=0.01, device='cpu')
        for p in tr.store.params.values():  # as a reducer does
            grad_sink.add_hook(p, lambda _p, s=tr.store: None)
        refs.append((weakref.ref(tr.store), weakref.ref(m)))
        del tr, m, p
        gc.collect()
    for store_ref, model_ref in refs:
        assert store_ref() is None and model_ref() is None, 'a dead trainer is still reachable'


def test_training_generation_keys_only_trainable_parameters():
    """precision.train_generation: moves with every training step for trainable parameters (the
    SGD kernels rewrite them in place), stays 0 for frozen ones (their values change only through
    loads, which bump the reload epoch) -- the key the inference-time filter folds use."""
    from mx_rcnn_amd.ops import precision
    frozen = torch.nn.Parameter(torch.ones(2), requires_grad=False)
    live = torch.nn.Parameter(torch.ones(2))
    g0 = precision.train_generation(live)
    assert precision.train_generation(frozen) == 0
    precision.bump_generation()
    assert precision.train_generation(live) == g0 + 1
    assert precision.train_generation(frozen, None) == 0
    assert precision.train_generation(frozen, live) == g0 + 1


def test_trainer_step_moves_the_training_generation():
    """Every training step (eager here; GraphedStep replays bump it too) advances the generation,
    so an evaluation between steps rebuilds the folds of trainable filters."""
    from mx_rcnn_amd.core.trainer import Trainer
    from tests.test_dist import _batch, _make_model
    tr = Trainer(_make_model(), 'rcnn', fixed_param_prefix=['conv0'], lr=0.01, wd=0.0, clip_gradient=-1, device='cpu')
    w = tr.model.trunk.conv0.weight if hasattr(tr.model.trunk, 'conv0') else next(tr.model.parameters())
    live = next(p for p in tr.model.parameters() if p.requires_grad)
    g0 = precision.train_generation(live)
    tr.step(_batch(0))
    assert precision.train_generation(live) > g0
    assert precision.train_generation(w) == (0 if not w.requires_grad else precision.train_generation(live))
