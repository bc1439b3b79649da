"""Data parallelism at the BASELINE rank counts on the CPU (gloo): config 3 runs 8 ranks
(`train_end2end.py:117,168`, bench N=8), config 4 four (`face.sh`, `train_alternate.py:15-63`).

* bench.py under torchrun at world 8 -- the driver's N=8 launch shape -- with the real e2e Trainer
  (ResNet-18, small images): one JSON line, dp8, every gradient bucket's collective measured, and
  the 8 replicas bitwise equal after the timed steps (weights digest all-reduced);
* the same at world 4 with VGG16 (the other BASELINE trunk);
* train_alternate.py under 4 ranks: rank-0 checkpoints read by every rank at the next stage, the
  proposal dump sharded over 4 ranks and gathered, combine_model, the final model;
* an uneven ``work_load_list`` over 4 ranks: the slices tile the global batch, every rank runs the
  same number of steps.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_PORT')}
    # one intra-op thread per rank: 8 ranks on the container's 8 CPUs
    env.update(PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='', OMP_NUM_THREADS='1')
    return env


def _torchrun(n, script, args, cwd, timeout=900):
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(n),
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.join(ROOT, script)] + args
    return subprocess.run(cmd, cwd=str(cwd), env=_env(), capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize('world,network,image', [(8, 'resnet18', '160x224'), (4, 'vgg16', '160x224')])
def test_bench_e2e_at_baseline_rank_counts(tmp_path, world, network, image):
    r = _torchrun(world, 'bench.py', ['--gpus', str(world), '--steps', '2', '--warmup', '1', '--network', network,
                                      '--image', image, '--num-classes', '6', '--bucket-mb', '4'], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    cfg = rec['config']
    assert rec['n_gpus'] == world and cfg['parallelism'] == 'dp%d' % world and cfg['global_batch'] == world
    assert cfg['backend'] == 'gloo' and cfg['train_mode'] == 'e2e'
    ar = cfg['allreduce']
    assert ar and len(ar['bucket_ms']) == len(ar['bucket_bytes']) >= 2  # several buckets at 4 MB
    assert cfg['replicas']['agree'] is True, cfg['replicas']
    assert all(np.isfinite(v) for v in cfg['objective_first_last'])


def test_alternate_training_four_ranks(tmp_path):
    """BASELINE config 4's pipeline at its rank count: 4-step alternate training under torchrun with
    4 gloo ranks; the proposal dumps cover every image once (9 images sharded rank::4 -- 3, 2, 2, 2 --
    and gathered back in image order)."""
    r = _torchrun(4, 'train_alternate.py',
                  ['--synthetic', '9', '--synthetic-shape', '160x224', '--max-steps', '2', '--rpn_epoch', '1',
                   '--rcnn_epoch', '1', '--model-dir', str(tmp_path / 'model'), '--root_path', str(tmp_path),
                   '--pretrained', 'none', '--network', 'resnet18'], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    for stage in ('rpn1', 'rcnn1', 'rpn2', 'rcnn2', 'final'):
        assert list((tmp_path / 'model').glob('%s-*.params' % stage)), stage
    from mx_rcnn_amd.data.cache import load_box_list
    boxes = load_box_list(str(tmp_path / 'rpn_data' / 'synthetic_rpn.npz'))
    assert len(boxes) == 9 and all(b.shape[1] == 5 and len(b) > 0 for b in boxes)


def test_uneven_work_load_list_four_ranks():
    """work_load_list '1,2,2,3' at world 4, 2 images per rank on average (global batch 8): rank k
    gets its share of every global batch, the four slices tile it in order, and all ranks step
    the same number of times (reference: MXNet _split_input_slice over the device list)."""
    from mx_rcnn_amd.config import config
    from mx_rcnn_amd.data.load_data import load_synthetic_roidb
    from mx_rcnn_amd.data.loader import AnchorLoader
    _, roidb = load_synthetic_roidb(24, 96, 128, 4)
    config.SCALES = (96,)
    config.MAX_SIZE = 128
    ld = [AnchorLoader(None, roidb, 2, True, rank=r, world_size=4, work_load_list='1,2,2,3', prefetch=1, workers=1)
          for r in range(4)]
    assert len({len(x) for x in ld}) == 1 and len(ld[0]) == 3
    for k, want in enumerate((1, 2, 2, 3)):
        assert all(len(b) == want for b in ld[k]._batches), k
    for step in range(len(ld[0])):
        parts = [list(x._batches[step]) for x in ld]
        assert sum(parts, []) == list(ld[0]._global[step])
    # the batches a rank yields carry its share
    b = ld[3].get_batch()
    assert np.asarray(b['data']).shape[0] == 3


def test_train_end2end_four_ranks_uneven_work_load(tmp_path):
    """The real training CLI at world 4 with an uneven work_load_list ('1,1,2,4' of a global batch
    of 8: ranks hold 1, 1, 2 and 4 images per step): every rank captures/steps in lockstep and rank 0
    writes the checkpoint."""
    r = _torchrun(4, 'train_end2end.py',
                  ['--synthetic', '16', '--synthetic-shape', '160x224', '--max-steps', '2', '--network', 'resnet18',
                   '--num_epoch', '1', '--prefix', str(tmp_path / 'e2e'), '--pretrained', 'none', '--frequent', '1',
                   '--ims-per-gpu', '2', '--work_load_list', '1,1,2,4', '--gpus', '0,1,2,3'], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (tmp_path / 'e2e-0001.params').exists(), (r.stdout + r.stderr)[-2000:]
