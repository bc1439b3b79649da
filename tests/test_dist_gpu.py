"""The data-parallel step on the GPU: a 1-rank RCCL (backend 'nccl') process group, with every
gradient bucket all-reduced inside the captured hipGraph (fp32 wire), must produce the same
weights as the same graphed step without a process group (reference semantics: kvstore 'device'
sums gradients, `train_end2end.py:150`; one rank sums one term).

Each configuration runs in its own process (tools/dp_step_check.py): a process group cannot be
torn down and re-created cleanly inside one process, and the non-DP step must not see one.
"""
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, name, precision, dp, port, steps, plan_file=None):
    out = str(tmp_path / (name + '.pt'))
    env = dict(os.environ)
    for k in ('MXR_FORCE_DIST', 'WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    if plan_file is None:
        # the per-shape conv autotune picks split-K variants by timing, i.e. per process: fix the plan
        env['MXR_CONV_TUNE'] = '0'
    else:  # autotune on, its plan persisted to / loaded from this file (ops/tune_plan.py)
        env.pop('MXR_CONV_TUNE', None)
        env['MXR_TUNE_FILE'] = str(plan_file)
    if dp:
        env.update({'MXR_FORCE_DIST': '1', 'WORLD_SIZE': '1', 'RANK': '0', 'LOCAL_RANK': '0',
                    'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port)})
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'dp_step_check.py'), out, '--precision', precision,
                        '--steps', str(steps)],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    return torch.load(out, weights_only=True), r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize('precision', ['bf16', 'bf16x3', 'fp32'])
def test_rccl_one_rank_graphed_step_matches_single_process(tmp_path, precision):
    """One graphed step (fresh momentum: the update is lr * clip(grad) + wd term, so any gradient
    difference shows directly).  The step is bitwise deterministic (no float atomics anywhere on
    the gradient path: the frozen-BN gamma / beta column sums go to per-tile partial rows folded
    in a fixed order, the RoI-pool backward accumulates in 64-bit fixed point, the BN-ReLU backward
    reduces in thread order), so two plain runs and the RCCL run must agree bit for bit on EVERY
    weight.  The conv autotune is off (its timing-based split-K choices differ between
    processes)."""
    a, _ = _run(tmp_path, 'plain', precision, False, 0, 1)
    b, _ = _run(tmp_path, 'plain2', precision, False, 0, 1)
    d, log = _run(tmp_path, 'dp', precision, True, 29650 + ['bf16', 'bf16x3', 'fp32'].index(precision), 1)
    assert int(a['_dp'][0]) == 0
    assert int(d['_dp'][0]) == 1 and int(d['_dp'][1]) >= 1, log  # the reducer really ran its buckets
    keys = [k for k in a if not k.startswith('_')]
    assert len(keys) > 20 and set(keys) == {k for k in d if not k.startswith('_')}
    nondet = [k for k in keys if not torch.equal(a[k], b[k])]
    assert not nondet, 'plain run-to-run differences: %s (max abs %s)' % (
        nondet[:5], [float((a[k].float() - b[k].float()).abs().max()) for k in nondet[:5]])
    diff = [k for k in keys if not torch.equal(a[k], d[k])]
    assert not diff, 'DP step differs: %s (max abs %s)' % (
        diff[:5], [float((a[k].float() - d[k].float()).abs().max()) for k in diff[:5]])


@pytest.mark.gpu
def test_autotuned_reruns_are_bitwise_equal_through_the_plan_file(tmp_path):
    """With the conv autotune ON, the first run times its candidates and persists the plan
    (ops/tune_plan.py); a second run loads it, takes the same kernels and must produce the same
    weights bit for bit (fp32 precision, one graphed step)."""
    plan = tmp_path / 'plan.json'
    a, _ = _run(tmp_path, 'tuned1', 'fp32', False, 0, 1, plan_file=plan)
    assert plan.exists(), 'the first run did not persist its conv plan'
    b, _ = _run(tmp_path, 'tuned2', 'fp32', False, 0, 1, plan_file=plan)
    keys = [k for k in a if not k.startswith('_')]
    diff = [k for k in keys if not torch.equal(a[k], b[k])]
    assert not diff, 'autotuned reruns differ: %s' % diff[:5]
