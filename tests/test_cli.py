"""CLI entry points on synthetic data, CPU (reference test strategy: the shell launchers and
train/test scripts are the integration tests).  Each runs as a subprocess so
global config mutations stay isolated."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SYN = ['--synthetic', '4', '--synthetic-shape', '320x480', '--max-steps', '2']


def _run(args, cwd, timeout=600):
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='')
    r = subprocess.run([sys.executable] + args, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout + r.stderr


@pytest.fixture(scope='module')
def alt_model(tmp_path_factory):
    d = tmp_path_factory.mktemp('alt')
    log = _run([os.path.join(ROOT, 'train_alternate.py')] + SYN +
               ['--rpn_epoch', '1', '--rcnn_epoch', '1', '--model-dir', str(d / 'model'), '--root_path', str(d),
                '--pretrained', 'none'], cwd=str(d))
    return d, log


def test_train_alternate_all_stages(alt_model):
    d, log = alt_model
    for stage in ('TRAIN RPN WITH IMAGENET INIT', 'TRAIN RCNN WITH IMAGENET INIT', 'TRAIN RPN WITH RCNN INIT',
                  'COMBINE RPN2 WITH RCNN1', 'TRAIN RCNN WITH RPN INIT', 'COMBINE RPN2 WITH RCNN2'):
        assert stage in log
    for f in ('rpn1-0001', 'rcnn1-0001', 'rpn2-0001', 'rcnn2-0000', 'rcnn2-0001', 'final-0000'):
        assert (d / 'model' / (f + '.params')).exists(), f
    assert (d / 'rpn_data' / 'synthetic_rpn.npz').exists()


def test_final_model_contains_both_halves(alt_model):
    from mx_rcnn_amd.utils.load_model import load_checkpoint
    d, _ = alt_model
    arg, _ = load_checkpoint(str(d / 'model' / 'final'), 0)
    rpn2, _ = load_checkpoint(str(d / 'model' / 'rpn2'), 1)
    rcnn2, _ = load_checkpoint(str(d / 'model' / 'rcnn2'), 1)
    np.testing.assert_array_equal(arg['rpn_cls_score_weight'], rpn2['rpn_cls_score_weight'])
    np.testing.assert_array_equal(arg['cls_score_weight'], rcnn2['cls_score_weight'])


def test_eval_demo_predict(alt_model):
    d, _ = alt_model
    log = _run([os.path.join(ROOT, 'test.py'), '--has_rpn', '--prefix', str(d / 'model' / 'final'), '--epoch', '0',
                '--synthetic', '4', '--synthetic-shape', '320x480'], cwd=str(d))
    assert 'Mean AP' in log
    from mx_rcnn_amd.data.synthetic import synthetic_image
    from mx_rcnn_amd.processing.image_processing import imwrite
    imwrite(str(d / 'img.jpg'), synthetic_image({'synthetic_seed': 3, 'height': 300, 'width': 420,
                                                 'boxes': np.array([[10, 10, 100, 120]])}))
    _run([os.path.join(ROOT, 'demo.py'), '--image', str(d / 'img.jpg'), '--prefix', str(d / 'model' / 'final'),
          '--epoch', '0', '--out', str(d / 'demo.jpg'), '--cfg', 'SCALES=[300]', 'MAX_SIZE=500'], cwd=str(d))
    assert (d / 'demo.jpg').exists()
    _run([os.path.join(ROOT, 'predict.py'), '--img', str(d / 'img.jpg'), '--prefix', str(d / 'model' / 'final'),
          '--epoch', '0', '--out', str(d / 'pred.jpg'), '--thresh', '0.0'], cwd=str(d))
    assert (d / 'pred.jpg').exists()


def test_train_end2end_resnet_synthetic(tmp_path):
    log = _run([os.path.join(ROOT, 'train_end2end.py')] + SYN +
               ['--network', 'resnet18', '--num_epoch', '1', '--prefix', str(tmp_path / 'e2e'), '--pretrained',
                'none', '--frequent', '1'], cwd=str(tmp_path))
    assert (tmp_path / 'e2e-0001.params').exists(), log[-2000:]


def test_eval_in_memory_perfect_and_empty():
    from mx_rcnn_amd.data.voc_eval import eval_in_memory
    gt = [{'boxes': np.array([[0, 0, 10, 10], [20, 20, 40, 50]]), 'gt_classes': np.array([1, 2])},
          {'boxes': np.array([[5, 5, 30, 30]]), 'gt_classes': np.array([1])}]
    classes = ['bg', 'a', 'b']
    det = [[], [np.array([[0, 0, 10, 10, .9]]), np.array([[5, 5, 30, 30, .8]])],
           [np.array([[20, 20, 40, 50, .7]]), np.zeros((0, 5))]]
    assert eval_in_memory(gt, det, classes) == pytest.approx(1.0)
    empty = [[], [np.zeros((0, 5))] * 2, [np.zeros((0, 5))] * 2]
    assert eval_in_memory(gt, empty, classes) == 0.0


def test_bench_rpn_cpu_json(tmp_path):
    """BASELINE config 1 harness (VGG16 RPN-only CPU forward) prints one well-formed JSON line."""
    import json
    out = _run([os.path.join(ROOT, 'bench_rpn_cpu.py'), '--image', '224x320', '--steps', '1', '--warmup', '0'],
               cwd=str(tmp_path))
    rec = json.loads([ln for ln in out.splitlines() if ln.startswith('{')][-1])
    assert rec['unit'] == 'ms/image' and rec['higher_is_better'] is False and rec['value'] > 0
    assert rec['config']['rois'] == [1, 300, 5]
