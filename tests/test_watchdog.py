"""Step heartbeat / stall watchdog (mx_rcnn_amd/parallel/watchdog.py): a local
stall is reported once per stalled step and re-armed by the next beat; with 2 gloo ranks,
rank 0 names the peer whose training loop stopped while its heartbeat thread still runs."""
import os
import tempfile
import time

import torch.multiprocessing as mp

from mx_rcnn_amd.parallel.watchdog import Heartbeat
from tests.test_dist import _free_port


def _wait(cond, timeout=5.0):
    t0 = time.time()
    while not cond() and time.time() - t0 < timeout:
        time.sleep(0.02)
    return cond()


def test_local_stall_fires_once_per_step():
    seen = []
    hb = Heartbeat(stall_s=0.25, period_s=0.03, store=None, on_stall=lambda *a: seen.append(a))
    with hb:
        hb.beat(0)
        assert _wait(lambda: len(seen) == 1)
        time.sleep(0.3)
        assert len(seen) == 1 and seen[0][:3] == ('local', 0, 0) and seen[0][3] > 0.25
        for s in range(1, 6):  # steady progress: no report
            hb.beat(s)
            time.sleep(0.05)
        assert len(seen) == 1
        assert _wait(lambda: len(seen) == 2)
        assert seen[1][:3] == ('local', 0, 5)


def _worker(rank, world, port, out_dir):
    os.environ.update({'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'RANK': str(rank),
                       'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank)})
    from mx_rcnn_amd.parallel import dist as pdist
    pdist.init_distributed(backend='gloo')
    seen = []
    hb = Heartbeat(stall_s=0.6, period_s=0.05, on_stall=lambda *a: seen.append(a)).start()
    steps = 40 if rank == 0 else 3  # rank 1's loop "hangs" after step 2 (thread keeps publishing)
    for s in range(steps):
        hb.beat(s)
        time.sleep(0.05)
    if rank == 1:
        time.sleep(2.0 - 3 * 0.05)
    hb.stop()
    with open(os.path.join(out_dir, 'r%d.txt' % rank), 'w') as f:
        f.write(repr([(k, r, s) for k, r, s, _ in seen]))
    pdist.barrier()
    pdist.destroy()


def test_peer_stall_reported_by_rank0():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        r0 = open(os.path.join(d, 'r0.txt')).read()
        r1 = open(os.path.join(d, 'r1.txt')).read()
    assert "('peer', 1, 2)" in r0, r0
    assert "('local', 1, 2)" in r1, r1
    assert 'local' not in r0, r0
