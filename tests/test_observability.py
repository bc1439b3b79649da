"""Aux subsystems: norm monitor, stage profiler, non-finite guard + fault
injection, RCNN_SYNC proxy, Speedometer JSONL sink."""
import json
import logging
import os

import numpy as np
import pytest
import torch


def _tiny_module(tmp_path=None, monitor=None):
    from mx_rcnn_amd.config import config
    from mx_rcnn_amd.core.module import MutableModule
    from mx_rcnn_amd.data.load_data import load_synthetic_roidb
    from mx_rcnn_amd.data.loader import AnchorLoader
    from mx_rcnn_amd.models import FasterRCNN
    config.TRAIN.BG_THRESH_LO = 0.0
    config.TRAIN.HAS_RPN = True
    config.END2END = 1
    config.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    config.SCALES = (160,)
    config.MAX_SIZE = 240
    imdb, roidb = load_synthetic_roidb(4, 160, 240, 5)
    torch.manual_seed(0)
    model = FasterRCNN('resnet18', 5)
    data = AnchorLoader(model, roidb, batch_size=1, shuffle=False, anchor_scales=model.anchor_scales)
    model.calibrate_bn(torch.as_tensor(data.get_batch()['data']))
    mod = MutableModule(model, ['data', 'im_info'], ['gt_boxes'], context='cpu',
                        fixed_param_prefix=['conv0', 'bn_data'], mode='e2e')
    return mod, data


def test_norm_monitor_reports_outputs_weights_grads(caplog):
    from mx_rcnn_amd.utils.monitor import Monitor
    mod, data = _tiny_module()
    mon = Monitor(interval=2, pattern='.*')
    with caplog.at_level(logging.INFO):
        mod.fit(data, num_epoch=1, monitor=mon, max_steps=3,
                optimizer_params={'learning_rate': 1e-3, 'momentum': 0.9, 'wd': 5e-4})
    lines = [r.getMessage() for r in caplog.records if r.getMessage().startswith('Batch:')]
    names = {l.split()[2] for l in lines}
    assert any(n.endswith('_output') for n in names)
    assert 'rpn_conv_3x3_weight' in names and 'rpn_conv_3x3_weight_grad' in names
    steps = {int(l.split()[1]) for l in lines}
    assert steps == {1, 3}  # steps 0 and 2 (reported after tic) with interval 2
    vals = [float(l.split()[3]) for l in lines]
    assert all(np.isfinite(vals))


def test_nonfinite_guard_and_fault_injection(monkeypatch):
    monkeypatch.setenv('MXR_FAULT_INJECT', 'nan@1')
    mod, data = _tiny_module()
    with pytest.raises(FloatingPointError, match='non-finite'):
        mod.fit(data, num_epoch=1, max_steps=3, check_every=2,
                optimizer_params={'learning_rate': 1e-3, 'momentum': 0.9, 'wd': 5e-4})


def test_no_fault_no_raise(monkeypatch):
    monkeypatch.delenv('MXR_FAULT_INJECT', raising=False)
    mod, data = _tiny_module()
    mod.fit(data, num_epoch=1, max_steps=2, check_every=1,
            optimizer_params={'learning_rate': 1e-3, 'momentum': 0.9, 'wd': 5e-4})
    assert int(mod.trainer.nonfinite) == 0


def test_parse_fault():
    from mx_rcnn_amd.core.module import parse_fault
    assert parse_fault('nan@7') == (7, 'nan')
    assert parse_fault(None) == (None, None)


def test_profiler_disabled_is_noop():
    from mx_rcnn_amd.utils import profiler as prof
    prof.enable(False)
    with prof.range('x'):
        pass
    assert prof.report() == {}


def test_speedometer_jsonl(tmp_path):
    from mx_rcnn_amd.core.callback import BatchEndParam, Speedometer
    from mx_rcnn_amd.core.metric import e2e_metrics
    path = str(tmp_path / 'speed.jsonl')
    sp = Speedometer(8, frequent=2, jsonl=path)
    m = e2e_metrics()
    for i in range(5):
        sp(BatchEndParam(0, i, m))
    recs = [json.loads(l) for l in open(path)]
    assert len(recs) == 2 and recs[0]['batch'] == 2 and 'samples_per_sec' in recs[0]


def test_rcnn_sync_proxy(monkeypatch):
    from mx_rcnn_amd.ops import _ext
    monkeypatch.setenv('RCNN_SYNC', '1')

    class Fake:
        def k(self, x):
            return x + 1
    p = _ext._SyncProxy(Fake())
    assert p.k(1) == 2


@pytest.mark.gpu
def test_profiler_stage_breakdown_gpu(cuda):
    from mx_rcnn_amd.config import snapshot
    from mx_rcnn_amd.core.trainer import Trainer
    from mx_rcnn_amd.models import FasterRCNN
    from mx_rcnn_amd.utils import profiler as prof
    import bench
    cfg = snapshot()
    cfg.END2END = 1
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    m = FasterRCNN('resnet50', 21, cfg=cfg)
    batch = bench.synthetic_batch(1, 320, 480, 21, cuda, torch.Generator().manual_seed(0))
    t = Trainer(m, 'e2e', fixed_param_prefix=['conv0', 'stage1', 'bn_data', 'bn0'], device=cuda)
    prof.enable(True)
    try:
        for _ in range(2):
            t.step(batch)
        rep = prof.report()
    finally:
        prof.enable(False)
    for k in ('trunk', 'proposal', 'roi_pool', 'head', 'backward+allreduce', 'sgd'):
        assert k in rep and rep[k] >= 0.0


def test_exact_resume_from_states(tmp_path):
    """2 epochs straight == 1 epoch + resume (params + momentum + update count + RNG + order)."""
    from mx_rcnn_amd.utils.load_model import load_checkpoint
    opt = {'learning_rate': 1e-3, 'momentum': 0.9, 'wd': 5e-4}
    from mx_rcnn_amd.core.lr_scheduler import FactorScheduler
    from mx_rcnn_amd.utils.load_model import do_checkpoint
    a_pref, b_pref = str(tmp_path / 'a'), str(tmp_path / 'b')
    torch.manual_seed(11)
    mod, data = _tiny_module()
    mod.fit(data, num_epoch=2, epoch_end_callback=do_checkpoint(a_pref), states_prefix=a_pref,
            optimizer_params=dict(opt, lr_scheduler=FactorScheduler(3, 0.5)))
    torch.manual_seed(11)
    mod, data = _tiny_module()
    mod.fit(data, num_epoch=1, epoch_end_callback=do_checkpoint(b_pref), states_prefix=b_pref,
            optimizer_params=dict(opt, lr_scheduler=FactorScheduler(3, 0.5)))
    from mx_rcnn_amd.utils.load_model import load_param
    arg, aux, _ = load_param(b_pref, 1)  # unfolds bbox_pred like the reference resume path
    mod2, data2 = _tiny_module()
    mod2.fit(data2, num_epoch=2, begin_epoch=1, arg_params=arg, aux_params=aux,
             epoch_end_callback=do_checkpoint(b_pref), resume_states=b_pref + '-0001.states',
             optimizer_params=dict(opt, lr_scheduler=FactorScheduler(3, 0.5)))
    assert mod2.trainer.num_update == 8
    a2, _ = load_checkpoint(a_pref, 2)
    b2, _ = load_checkpoint(b_pref, 2)
    for k in a2:
        np.testing.assert_allclose(a2[k], b2[k], rtol=1e-2, atol=1e-5, err_msg=k)


def test_old_states_file_rederives_dropout_counter(tmp_path):
    """A states file written before the dropout counter was saved ('rng_step' absent) resumes the
    counter from the update count instead of restarting at 0."""
    from mx_rcnn_amd.utils import ndarray_io
    from mx_rcnn_amd.utils.load_model import do_checkpoint
    pref = str(tmp_path / 'c')
    torch.manual_seed(3)
    mod, data = _tiny_module()
    mod.fit(data, num_epoch=1, epoch_end_callback=do_checkpoint(pref), states_prefix=pref,
            optimizer_params={'learning_rate': 1e-3, 'momentum': 0.9, 'wd': 5e-4})
    n = mod.trainer.num_update
    assert n > 0 and int(mod.trainer.rng_step.item()) == n
    st = ndarray_io.load(pref + '-0001.states')
    del st['rng_step']
    ndarray_io.save(pref + '-old.states', st)
    mod2, _ = _tiny_module()
    mod2.init_optimizer(optimizer_params={'learning_rate': 1e-3, 'momentum': 0.9, 'wd': 5e-4})
    mod2.load_optimizer_states(pref + '-old.states')
    assert int(mod2.trainer.rng_step.item()) == n


def test_watchdog_in_fit_reports_slow_steps_and_stops(monkeypatch):
    """MXR_WATCHDOG=<s> arms the heartbeat inside Module.fit: CPU steps slower than the stall
    limit are reported (the loop itself is not disturbed) and the thread ends with fit."""
    import threading
    from mx_rcnn_amd.parallel import watchdog
    seen = []
    monkeypatch.setattr(watchdog.Heartbeat, '_report', lambda self, *a: seen.append(a))
    monkeypatch.setenv('MXR_WATCHDOG', '0.02')
    mod, data = _tiny_module()
    mod.fit(data, num_epoch=1, max_steps=2, optimizer_params={'learning_rate': 1e-3, 'momentum': 0.9, 'wd': 5e-4})
    assert seen and all(k == 'local' for k, *_ in seen)
    assert not any(t.name == 'mxr-heartbeat' for t in threading.enumerate())


def test_watchdog_pause_covers_long_host_phases():
    """pause()/resume() brackets known long phases (graph capture, epoch-end checkpointing): no
    local stall is reported while paused, and the stall clock restarts on resume."""
    import time
    from mx_rcnn_amd.parallel.watchdog import Heartbeat
    seen = []
    hb = Heartbeat(0.05, period_s=0.01, store=None, on_stall=lambda *a: seen.append(a))
    hb.start()
    hb.beat(0)
    with hb.paused():
        time.sleep(0.25)
    assert not seen
    time.sleep(0.25)  # unpaused and silent: reported
    hb.stop()
    assert seen and seen[0][0] == 'local'
