"""The data-parallel step on the GPU: a 1-rank RCCL (backend 'nccl') process group, with every
gradient bucket all-reduced inside the captured hipGraph (fp32 wire), must produce the same
weights as the same graphed step without a process group (reference semantics: kvstore 'device'
sums gradients, `train_end2end.py:150`; one rank sums one term).

Each configuration runs in its own process (tools/dp_step_check.py): a process group cannot be
torn down and re-created cleanly inside one process, and the non-DP step must not see one.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, name, precision, dp, port, steps, plan_file=None, extra=()):
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
                        '--steps', str(steps)] + list(extra),
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
@pytest.mark.parametrize('precision', ['bf16', 'fp32'])
def test_vgg16_fc_update_after_allreduce_matches_fused_single_process(tmp_path, precision):
    """VGG16 e2e under a 1-rank RCCL group: fc6 / fc7 take their SGD on the reducer's optimizer
    stream right after their buckets' all-reduce (parallel/reducer.py sgd_names), the rest at the
    end of the step; the single-process step fuses the same update into the weight gradient.  Two
    graphed steps, every weight bitwise equal."""
    ex = ('--mode', 'e2e', '--network', 'vgg16', '--image', '224x320')
    a, la = _run(tmp_path, 'vgg_plain', precision, False, 0, 2, extra=ex)
    d, ld = _run(tmp_path, 'vgg_dp', precision, True, 29660 + ['bf16', 'fp32'].index(precision), 2, extra=ex)
    assert int(a['_dp'][4]) == 2, la  # fused into the wgrad in the single process
    assert int(d['_dp'][0]) == 1 and int(d['_dp'][3]) >= 2, ld  # DP: early bucket updates
    keys = [k for k in a if not k.startswith('_')]
    diff = [k for k in keys if not torch.equal(a[k], d[k])]
    assert not diff, 'DP fc update differs: %s (max abs %s)' % (
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


def _two_ranks(tmp_path, name, precision, same_batch, steps=2, extra=()):
    """Two worker processes (tools/dp_two_rank_check.py), both on cuda:0, gloo rendezvous on
    127.0.0.1; returns both ranks' saved states."""
    sk = socket.socket()
    sk.bind(('127.0.0.1', 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(2):
        env = dict(os.environ)
        env.pop('MXR_FORCE_DIST', None)
        env.update({'MXR_CONV_TUNE': '0', 'WORLD_SIZE': '2', 'RANK': str(r), 'LOCAL_RANK': '0',
                    'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port)})
        cmd = [sys.executable, os.path.join(ROOT, 'tools', 'dp_two_rank_check.py'), str(tmp_path / ('%s_r%d.pt' % (name, r))),
               '--precision', precision, '--steps', str(steps)] + (['--same-batch'] if same_batch else []) + list(extra)
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=480)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    return [torch.load(str(tmp_path / ('%s_r%d.pt' % (name, r))), weights_only=True) for r in range(2)], outs


def _plain(tmp_path, name, precision, rescale, steps=2, extra=()):
    env = dict(os.environ)
    for k in ('MXR_FORCE_DIST', 'WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    env['MXR_CONV_TUNE'] = '0'
    out = str(tmp_path / (name + '.pt'))
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'dp_two_rank_check.py'), out, '--precision', precision,
                        '--steps', str(steps), '--rescale', str(rescale)] + list(extra),
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=480)
    assert r.returncode == 0, r.stdout[-3000:]
    return torch.load(out, weights_only=True)


@pytest.mark.gpu
@pytest.mark.parametrize('precision', ['fp32', 'bf16'])
def test_two_ranks_on_one_gpu_sum_gradients(tmp_path, precision):
    """World size 2 on the device kernels.  Both ranks train on the SAME batches, so the summed
    gradient is exactly 2g, and one plain process with rescale_grad = 2 must produce the same
    weights and momenta bit for bit (x + x and 2 * x are both exact); both replicas must be
    identical.  RCCL refuses two ranks on one GPU: the ranks talk over gloo (device buckets staged
    through host memory), everything else is the production DP path (hooks, buckets, SUM, SGD)."""
    (r0, r1), logs = _two_ranks(tmp_path, 'same', precision, True)
    assert r0['_info'].tolist()[:3] == [1, int(r0['_info'][1]), 2] and int(r0['_info'][1]) > 1, logs[0][-2000:]
    ref = _plain(tmp_path, 'plain2x', precision, 2.0)
    assert int(ref['_info'][0]) == 0
    keys = [k for k in ref if not k.startswith('_')]
    assert len(keys) > 10
    for k in keys:
        assert torch.equal(r0[k], r1[k]), ('replicas differ', k)
    diff = [k for k in keys if not torch.equal(ref[k], r0[k])]
    assert not diff, 'DP sum differs from the plain 2x-rescaled step: %s (max abs %s)' % (
        diff[:5], [float((ref[k].float() - r0[k].float()).abs().max()) for k in diff[:5]])


@pytest.mark.gpu
def test_two_ranks_on_one_gpu_stay_in_sync_on_different_batches(tmp_path):
    """Per-rank batches: different objectives, one synchronous update -- the replicas stay
    bit-identical, and they moved away from the single-rank result."""
    (r0, r1), logs = _two_ranks(tmp_path, 'diff', 'fp32', False)
    assert not torch.equal(r0['_objective'], r1['_objective']), logs[0][-2000:]
    keys = [k for k in r0 if not k.startswith('_')]
    for k in keys:
        assert torch.equal(r0[k], r1[k]), ('replicas differ', k)
    ref = _plain(tmp_path, 'plain1x', 'fp32', 1.0)
    assert any(not torch.equal(ref[k], r0[k]) for k in keys)


@pytest.mark.gpu
def test_two_ranks_on_one_gpu_e2e_resnet101_headline_shape(tmp_path):
    """the production-shaped DP step -- e2e ResNet-101 at 800x1333 (anchor targets,
    the proposal chain 12000 -> 6000 and its RoI sampling, the stage-4 head), 25 MB buckets -- with
    two ranks on the box's one GPU (gloo between them), same batches: bit for bit the weights of one
    process with rescale_grad = 2, identical replicas."""
    ex = ('--mode', 'e2e', '--network', 'resnet101', '--image', '800x1333', '--bucket-mb', '25')
    (r0, r1), logs = _two_ranks(tmp_path, 'e2e', 'fp32', True, steps=2, extra=ex)
    info = r0['_info'].tolist()
    assert info[0] == 1 and info[1] >= 5 and info[2] == 2, logs[0][-2000:]  # production-size buckets
    ref = _plain(tmp_path, 'e2e_plain2x', 'fp32', 2.0, steps=2, extra=ex)
    keys = [k for k in ref if not k.startswith('_')]
    assert len(keys) > 300
    for k in keys:
        assert torch.equal(r0[k], r1[k]), ('replicas differ', k)
    diff = [k for k in keys if not torch.equal(ref[k], r0[k])]
    assert not diff, 'e2e DP sum differs from the plain 2x-rescaled step: %s (max abs %s)' % (
        diff[:5], [float((ref[k].float() - r0[k].float()).abs().max()) for k in diff[:5]])
