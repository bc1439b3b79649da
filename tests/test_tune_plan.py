"""Conv autotune plans (ops/tune_plan.py): persisted across runs, identical across DP ranks.

The autotune picks tiles / K splits by timing, and K splits change summation order, so the plan
decides the low bits of every conv output.  Host-only: the plan table lives in the extension's
host code, no GPU needed.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from mx_rcnn_amd.ops import tune_plan
from mx_rcnn_amd.ops._ext import ext_available, need_ext

pytestmark = pytest.mark.skipif(not ext_available(), reason='extension not built')


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_plan_file_roundtrip_and_hash(tmp_path, monkeypatch):
    ext = need_ext()
    monkeypatch.setenv('MXR_TUNE_FILE', str(tmp_path / 'plan.json'))
    ext.conv_tune_set([('1,50,84,256,256,3,3,1,1|x', 23, 1), ('1,50,84,1024,256,1,1,1,0|y', 30, 2)], True)
    path = tune_plan.save()
    assert path == str(tmp_path / 'plan.json')
    got = tune_plan.read_plan(path)
    assert got == tune_plan.table()
    h = tune_plan.plan_hash()
    # a fresh table loaded from the file is the same plan
    ext.conv_tune_set([], True)
    assert tune_plan.plan_hash() != h
    ext.conv_tune_set(got, True)
    assert tune_plan.plan_hash() == h
    # another version / arch is ignored
    with open(path, 'w') as f:
        f.write('{"arch": "gfx950", "version": -1, "plan": {"k": [1, 1]}}')
    assert tune_plan.read_plan(path) == []


def _worker(rank, world, port, out):
    os.environ.update({'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'RANK': str(rank),
                       'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank), 'MXR_TUNE_PLAN': '0'})
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    ext = need_ext()
    # the same shapes tuned to DIFFERENT winners on each rank (timing noise), plus a rank-only shape
    ext.conv_tune_set([('shapeA', 23 + rank, 1), ('shapeB', 30, 1 + rank), ('only%d' % rank, 22, 1)], True)
    h = tune_plan.sync_from_rank0(torch.device('cpu'))
    torch.save({'hash': h, 'table': tune_plan.table()}, os.path.join(out, 'r%d.pt' % rank))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_ranks_capture_rank0_plan():
    world = 3
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, 'r%d.pt' % r), weights_only=True) for r in range(world)]
    assert len({r['hash'] for r in res}) == 1
    assert all(r['table'] == res[0]['table'] for r in res)
    assert ('shapeA', 23, 1) in res[0]['table'] and ('only0', 22, 1) in res[0]['table']
    assert not any(k.startswith('only1') or k.startswith('only2') for k, _, _ in res[1]['table'])
