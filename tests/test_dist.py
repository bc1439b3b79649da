"""Data-parallel correctness on CPU with the gloo backend, world_size 2 (multi-process):
bucketed all-reduce SUM of flat gradient buffers + fused SGD must equal one process
accumulating both ranks' gradients (reference kvstore 'device' semantics: grads summed)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(rank):
    g = torch.Generator().manual_seed(100 + rank)
    rois = torch.tensor([[0., 10, 20, 80, 100], [0., 30, 30, 90, 120], [0., 5, 5, 60, 60]])
    return {'data': torch.randn(1, 3, 96, 128, generator=g) * 50, 'rois': rois,
            'label': torch.tensor([3, 0, 5], dtype=torch.int32),
            'bbox_target': torch.randn(3, 24, generator=g) * 0.1,
            'bbox_inside_weight': torch.ones(3, 24), 'bbox_outside_weight': torch.ones(3, 24)}


def _make_model():
    from mx_rcnn_amd.config import snapshot
    from mx_rcnn_amd.models import FasterRCNN
    torch.manual_seed(0)
    return FasterRCNN('resnet18', 6, cfg=snapshot())


def _worker(rank, world, port, out_dir, bucket_mb):
    os.environ.update({'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'RANK': str(rank),
                       'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank)})
    from mx_rcnn_amd.parallel import dist as pdist
    from mx_rcnn_amd.core.trainer import Trainer
    pdist.init_distributed(backend='gloo')
    tr = Trainer(_make_model(), 'rcnn', fixed_param_prefix=['conv0'], lr=0.01, wd=0.0, clip_gradient=-1,
                 device='cpu', bucket_mb=bucket_mb)
    assert len(tr.reducer.buckets) >= 1
    tr.step(_batch(rank))
    torch.save({k: v.clone() for k, v in tr.store.state_arrays().items()}, os.path.join(out_dir, 'r%d.pt' % rank))
    pdist.barrier()
    pdist.destroy()


@pytest.mark.parametrize('bucket_mb', [64, 0.05])
def test_dp_gloo_matches_single_process(bucket_mb):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d, bucket_mb), nprocs=world, join=True)
        r0 = torch.load(os.path.join(d, 'r0.pt'), weights_only=True)
        r1 = torch.load(os.path.join(d, 'r1.pt'), weights_only=True)
    # replicas identical after the synchronous update
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    # single process: accumulate both ranks' gradients, one SGD step
    from mx_rcnn_amd.core.trainer import Trainer
    tr = Trainer(_make_model(), 'rcnn', fixed_param_prefix=['conv0'], lr=0.01, wd=0.0, clip_gradient=-1,
                 device='cpu')
    tr.model.train()
    tr.store.zero_grad()
    for r in range(world):
        out = tr.forward(tr.prepare_batch(_batch(r)))
        out['loss'].backward()
    tr.update_lr()
    tr.store.sgd_step(tr.lr_t, tr.momentum, tr.wd, tr.rescale, tr.clip)
    ref = tr.store.state_arrays()
    for k in ref:
        assert torch.allclose(ref[k], r0[k], atol=1e-5, rtol=1e-4), k


def test_alternate_training_two_ranks(tmp_path):
    """4-step alternate training under torchrun with 2 gloo ranks (BASELINE config 4 shape on the
    CPU): checkpoints written by rank 0 are read by every rank at the next stage, the proposal
    dump is sharded over ranks and gathered, and the final combined model exists."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.join(root, 'train_alternate.py'),
           '--synthetic', '5', '--synthetic-shape', '320x480', '--max-steps', '2', '--rpn_epoch', '1',
           '--rcnn_epoch', '1', '--model-dir', str(tmp_path / 'model'), '--root_path', str(tmp_path),
           '--pretrained', 'none', '--network', 'resnet18']
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (tmp_path / 'model' / 'final-0000.params').exists()
    from mx_rcnn_amd.data.cache import load_box_list
    boxes = load_box_list(str(tmp_path / 'rpn_data' / 'synthetic_rpn.npz'))
    assert len(boxes) == 5 and all(b.shape[1] == 5 for b in boxes)


def _bcast_worker(rank, world, port, out_dir):
    os.environ.update({'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'RANK': str(rank),
                       'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank)})
    from mx_rcnn_amd.config import snapshot
    from mx_rcnn_amd.core.trainer import Trainer
    from mx_rcnn_amd.models import FasterRCNN
    from mx_rcnn_amd.parallel import dist as pdist
    pdist.init_distributed(backend='gloo')
    torch.manual_seed(rank)  # deliberately different initialisations
    m = FasterRCNN('resnet18', 6, cfg=snapshot())
    for b in m.buffers():
        if b.is_floating_point():
            b.add_(float(rank))
    tr = Trainer(m, 'e2e', fixed_param_prefix=['conv0', 'stage1'], device='cpu')
    st = {k: v.clone() for k, v in tr.store.state_arrays().items()}
    st.update({'buf%d' % i: b.clone() for i, b in enumerate(tr.model.buffers())})
    torch.save(st, os.path.join(out_dir, 'b%d.pt' % rank))
    pdist.barrier()
    pdist.destroy()


def test_dp_ranks_start_from_rank0_weights():
    """Data parallel training starts every rank from rank 0's parameters and buffers."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_bcast_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        r0 = torch.load(os.path.join(d, 'b0.pt'), weights_only=True)
        r1 = torch.load(os.path.join(d, 'b1.pt'), weights_only=True)
    assert r0.keys() == r1.keys()
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k


def test_bench_two_ranks_contract(tmp_path):
    """bench.py under torchrun with 2 gloo ranks (the driver's N>1 launch shape, on the CPU):
    one JSON line from rank 0 with the whole-job value and dp2 config."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.join(root, 'bench.py'),
           '--gpus', '2', '--steps', '2', '--warmup', '1', '--network', 'resnet18', '--image', '256x320',
           '--num-classes', '6']
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == 2 and rec['steps'] == 2 and rec['warmup'] == 1 and rec['scaling'] == 'weak'
    assert rec['config']['parallelism'] == 'dp2' and rec['config']['global_batch'] == 2
    assert abs(rec['value'] - 2 * 2 / (rec['ms_per_step'] * 2 / 1e3)) <= 0.01 * rec['value'] + 1e-3


class _FakeImdb:
    num_images, num_classes, name = 5, 3, 'fake'

    def evaluate_detections(self, all_boxes):
        # image k of class j carries the score k + j / 10; the result encodes the order
        return [[float(all_boxes[j][k][0, 4]) for k in range(self.num_images)] for j in range(1, self.num_classes)]


class _FakeLoader:
    shuffle = False

    def __init__(self, image_ids):
        self.ids = image_ids

    def __iter__(self):
        for k in self.ids:
            yield {'data': None, 'im_info': None, 'k': k}


class _FakeDetector:
    def __init__(self, loader):
        self.it = iter(loader.ids)

    def detect_batch(self, data, im_info, thresh, nms, max_per_image, rois=None):
        k = next(self.it)
        boxes = torch.tensor([[0., 0, 10, 10], [1., 1, 11, 11]])
        return [(boxes, torch.tensor([k + 0.1, k + 0.2]), torch.tensor([1, 2]))]


def _eval_worker(rank, world, port, out_dir):
    os.environ.update({'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'RANK': str(rank),
                       'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank)})
    from mx_rcnn_amd.parallel import dist as pdist
    from mx_rcnn_amd.core.tester import pred_eval
    from mx_rcnn_amd.config import config
    pdist.init_distributed(backend='gloo')
    config.TEST.HAS_RPN = True
    loader = _FakeLoader(list(range(rank, _FakeImdb.num_images, world)))
    res = pred_eval(_FakeDetector(loader), loader, _FakeImdb(), shard=(rank, world))
    torch.save(torch.tensor(res), os.path.join(out_dir, 'e%d.pt' % rank))
    pdist.barrier()
    pdist.destroy()


def test_sharded_pred_eval_two_ranks():
    """Images rank::world per rank are gathered back in image order; every rank gets rank 0's
    evaluation."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_eval_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        e0 = torch.load(os.path.join(d, 'e0.pt'), weights_only=True)
        e1 = torch.load(os.path.join(d, 'e1.pt'), weights_only=True)
    want = torch.tensor([[k + 0.1 for k in range(5)], [k + 0.2 for k in range(5)]])
    assert torch.allclose(e0, want) and torch.equal(e0, e1)


def test_bench_spawns_ranks_itself(tmp_path):
    """``python bench.py --gpus 2`` with no launcher starts 2 rank processes itself (the
    reference's single-command multi-GPU launch) and reports n_gpus from the process group,
    plus the measured per-bucket all-reduce time."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_PORT')}
    env.update(PYTHONPATH=root, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='')
    cmd = [sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '2', '--warmup', '1',
           '--network', 'resnet18', '--image', '256x320', '--num-classes', '6']
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == 2 and rec['config']['parallelism'] == 'dp2' and rec['config']['backend'] == 'gloo'
    ar = rec['config']['allreduce']
    assert ar and len(ar['bucket_ms']) == len(ar['bucket_bytes']) >= 1 and ar['total_ms'] > 0


def test_bench_rejects_mismatched_world(tmp_path):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, CUDA_VISIBLE_DEVICES='', RANK='0', WORLD_SIZE='1', LOCAL_RANK='0',
               MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '1'],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and 'WORLD_SIZE=1' in (r.stderr + r.stdout)


class _FakeGroup:
    def __init__(self, grad):
        self.grad = grad
        self.numel = grad.numel()
        self.entries = [('p%d' % i, None, 'weight', 25, (25,), False) for i in range(grad.numel() // 25)]
        self.offsets = [25 * i for i in range(grad.numel() // 25)]
        self.decay = True


class _FakeStore:
    def __init__(self, grad):
        self.groups = [_FakeGroup(grad)]
        self.params = {}
        self.device = grad.device


def _wire_worker(rank, world, port, out_dir, comm):
    os.environ.update({'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'RANK': str(rank),
                       'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank)})
    from mx_rcnn_amd.parallel import dist as pdist
    from mx_rcnn_amd.parallel.reducer import BucketReducer
    pdist.init_distributed(backend='gloo')
    g = torch.Generator().manual_seed(7 + rank)
    grad = (torch.randn(200, generator=g) * torch.logspace(-3, 3, 200)).to(torch.bfloat16)
    red = BucketReducer(_FakeStore(grad), bucket_mb=0.0002, tail_mb=0.0001,
                        comm_dtype=torch.float32 if comm == 'fp32' else torch.bfloat16)
    assert len(red.buckets) > 1
    orig = grad.clone()  # the bf16 wire reduces in place
    red.prepare()
    red.finish()
    out = red.grad_for(red.store.groups[0]).clone()
    torch.save({'grad': orig, 'sum': out}, os.path.join(out_dir, 'w%d.pt' % rank))
    pdist.barrier()
    pdist.destroy()


@pytest.mark.parametrize('comm', ['fp32', 'bf16'])
def test_bf16_gradients_summed_in_fp32_on_the_wire(comm):
    """bf16 gradient buffers are widened per bucket and all-reduced in fp32 (the reference
    kvstore sums fp32); the optimizer reads the fp32 sum.  bf16 wire is the opt-in."""
    world = 3
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_wire_worker, args=(world, _free_port(), d, comm), nprocs=world, join=True)
        rs = [torch.load(os.path.join(d, 'w%d.pt' % r), weights_only=True) for r in range(world)]
    exact = sum(r['grad'].double() for r in rs)
    scale = sum(r['grad'].double().abs() for r in rs)  # error bounds scale with sum |g|
    for r in rs:
        assert torch.equal(r['sum'], rs[0]['sum'])
    err = ((rs[0]['sum'].double() - exact).abs() / scale).max().item()
    if comm == 'fp32':
        assert rs[0]['sum'].dtype == torch.float32
        assert err <= 2 ** -22
    else:
        assert rs[0]['sum'].dtype == torch.bfloat16
        assert err <= 2 ** -6


def _aux_worker(rank, world, port, out_dir):
    os.environ.update({'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'RANK': str(rank),
                       'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank)})
    from mx_rcnn_amd.config import snapshot
    from mx_rcnn_amd.core.module import MutableModule
    from mx_rcnn_amd.models import FasterRCNN
    from mx_rcnn_amd.parallel import dist as pdist
    pdist.init_distributed(backend='gloo')
    torch.manual_seed(0)
    m = FasterRCNN('resnet18', 6, cfg=snapshot())
    mod = MutableModule(m, context='cpu', mode='e2e')
    mod.bind()
    with torch.no_grad():  # per-rank train-mode statistics diverge between checkpoints
        for k, t in mod._model_aux().items():
            t.fill_(float(rank + 1))
    _, aux = mod.get_params()
    torch.save({k: torch.from_numpy(v) for k, v in aux.items()}, os.path.join(out_dir, 'a%d.pt' % rank))
    pdist.barrier()
    pdist.destroy()


def test_checkpoint_averages_bn_moving_stats_over_ranks():
    """get_params (the checkpoint source) averages BN moving statistics across ranks, like
    MXNet's get_params over device copies (rcnn/module.py:84-86)."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_aux_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        a0 = torch.load(os.path.join(d, 'a0.pt'), weights_only=True)
        a1 = torch.load(os.path.join(d, 'a1.pt'), weights_only=True)
    assert a0 and any('stage4' in k or 'bn1' in k for k in a0)
    for k in a0:
        assert torch.allclose(a0[k], torch.full_like(a0[k], 1.5)), k
        assert torch.equal(a0[k], a1[k])


@pytest.mark.parametrize('mode', ['rpn', 'rcnn'])
def test_bench_alternate_stage_modes_two_ranks(tmp_path, mode):
    """``bench.py --train-mode rpn|rcnn`` (BASELINE config 4: the alternate scheme's stages) with
    2 self-spawned gloo ranks: one JSON line with the stage metric, n_gpus 2, finite objective."""
    import json
    import math
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_PORT')}
    env.update(PYTHONPATH=root, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='')
    cmd = [sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '2', '--warmup', '1',
           '--network', 'resnet18', '--image', '256x320', '--num-classes', '6', '--train-mode', mode]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec['metric'] == 'imgs/sec alternate-stage %s train resnet18' % mode
    assert rec['n_gpus'] == 2 and rec['config']['train_mode'] == mode
    assert all(math.isfinite(v) for v in rec['config']['objective_first_last'])


def test_gpus_names_devices_like_the_reference(monkeypatch):
    """--gpus is a device list as in the reference (train_end2end.py:168): '2,3' runs two ranks
    on GPUs 2 and 3 (HIP_VISIBLE_DEVICES for the children), '3' one process on GPU 3."""
    from mx_rcnn_amd.parallel import spawn
    for k in ('RANK', 'WORLD_SIZE', 'HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES', 'ROCR_VISIBLE_DEVICES'):
        monkeypatch.delenv(k, raising=False)
    assert spawn.device_ids('2,3') == [2, 3] and spawn.device_ids('3') == [3] and spawn.device_ids(4) == [0, 1, 2, 3]
    assert spawn.parse_gpus('2,3') == 2 and spawn.parse_gpus('0') == 1
    assert spawn.select_devices('2,3') == '2,3'
    assert 'HIP_VISIBLE_DEVICES' not in os.environ
    assert spawn.select_devices('0') is None and 'HIP_VISIBLE_DEVICES' not in os.environ
    assert spawn.select_devices('3') is None
    assert os.environ['HIP_VISIBLE_DEVICES'] == '3'


def test_gpus_index_an_existing_visibility_mask(monkeypatch):
    """under a scheduler's HIP_VISIBLE_DEVICES=4,5,6,7, '--gpus 2,3' means the 3rd and
    4th VISIBLE devices (physical 6, 7), like mx.gpu(i); an id past the mask is an error."""
    import pytest as _pt
    from mx_rcnn_amd.parallel import spawn
    for k in ('RANK', 'WORLD_SIZE', 'CUDA_VISIBLE_DEVICES', 'ROCR_VISIBLE_DEVICES'):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv('HIP_VISIBLE_DEVICES', '4,5,6,7')
    assert spawn.select_devices('2,3') == '6,7'
    assert spawn.select_devices('0') is None and os.environ['HIP_VISIBLE_DEVICES'] == '4'
    monkeypatch.setenv('HIP_VISIBLE_DEVICES', '4,5,6,7')
    with _pt.raises(SystemExit):
        spawn.select_devices('1,5')
    # a launched rank is placed by its launcher: nothing changes
    monkeypatch.setenv('RANK', '0')
    monkeypatch.setenv('WORLD_SIZE', '2')
    assert spawn.select_devices('2,3') is None and os.environ['HIP_VISIBLE_DEVICES'] == '4,5,6,7'


def test_gpus_under_rocr_and_cuda_masks(monkeypatch):
    """ROCR_VISIBLE_DEVICES renumbers the devices below HIP, so the HIP mask written for
    the ranks holds INDICES into it ('--gpus 0' under ROCR=4,5,6,7 leaves the env alone; '1,2' ->
    '1,2'); a CUDA_VISIBLE_DEVICES mask is HIP's own alias and maps like HIP_VISIBLE_DEVICES."""
    import pytest as _pt
    from mx_rcnn_amd.parallel import spawn
    for k in ('RANK', 'WORLD_SIZE', 'HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES', 'ROCR_VISIBLE_DEVICES'):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv('ROCR_VISIBLE_DEVICES', '4,5,6,7')
    assert spawn.select_devices('0') is None and 'HIP_VISIBLE_DEVICES' not in os.environ
    assert spawn.select_devices('1,2') == '1,2'
    assert spawn.select_devices('3') is None and os.environ['HIP_VISIBLE_DEVICES'] == '3'
    monkeypatch.delenv('HIP_VISIBLE_DEVICES')
    with _pt.raises(SystemExit):
        spawn.select_devices('4')
    monkeypatch.delenv('ROCR_VISIBLE_DEVICES')
    monkeypatch.setenv('CUDA_VISIBLE_DEVICES', '2,3')
    assert spawn.select_devices('0,1') == '2,3'
    assert spawn.select_devices('1') is None and os.environ['HIP_VISIBLE_DEVICES'] == '3'


def test_capture_sync_key_ignores_uneven_slices():
    """an uneven work_load_list gives ranks different batch sizes; the cross-rank
    capture check must compare only the slice-independent dims (module.sync_key)."""
    from mx_rcnn_amd.core.module import sync_key
    k1 = (('data', (1, 3, 608, 1024)), ('gt_boxes', (1, 20, 5)), ('im_info', (1, 3)))
    k3 = (('data', (3, 3, 608, 1024)), ('gt_boxes', (3, 20, 5)), ('im_info', (3, 3)))
    assert k1 != k3 and sync_key(k1) == sync_key(k3)
    k_other = (('data', (1, 3, 600, 1024)), ('gt_boxes', (1, 20, 5)), ('im_info', (1, 3)))
    assert sync_key(k_other) != sync_key(k1)


def test_two_rank_check_tool_sums_like_rescale_two_on_cpu(tmp_path):
    """The worker of the GPU two-rank test (tools/dp_two_rank_check.py) on the CPU: two gloo ranks
    on the same batch sum their gradients to exactly 2g, so they match one process with
    rescale_grad = 2 bit for bit, and the replicas agree."""
    from tests.test_dist_gpu import _plain, _two_ranks
    (r0, r1), logs = _two_ranks(tmp_path, 'cpu', 'fp32', True, steps=1)
    assert r0['_info'].tolist()[0] == 1 and r0['_info'].tolist()[2] == 2, logs[0][-2000:]
    ref = _plain(tmp_path, 'cpu_plain2x', 'fp32', 2.0, steps=1)
    keys = [k for k in ref if not k.startswith('_')]
    assert len(keys) > 10
    for k in keys:
        assert torch.equal(r0[k], r1[k]), ('replicas differ', k)
        assert torch.equal(ref[k], r0[k]), ('DP sum differs from the 2x-rescaled step', k)


def _fc_worker(rank, world, port, out_dir, early):
    os.environ.update({'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'RANK': str(rank),
                       'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank), 'MXR_FUSED_FC_SGD': '1' if early else '0'})
    from mx_rcnn_amd.config import snapshot
    from mx_rcnn_amd.core.trainer import Trainer
    from mx_rcnn_amd.models import FasterRCNN
    from mx_rcnn_amd.parallel import dist as pdist
    pdist.init_distributed(backend='gloo')
    torch.manual_seed(0)
    cfg = snapshot()
    cfg.TRAIN.BG_THRESH_LO = 0.0
    cfg.END2END = 1
    cfg.TRAIN.BBOX_NORMALIZATION_PRECOMPUTED = True
    cfg.TRAIN.RPN_PRE_NMS_TOP_N = 600
    cfg.TRAIN.RPN_POST_NMS_TOP_N = 200
    m = FasterRCNN('vgg16', 6, cfg=cfg)
    m.head.dropout = 0.0
    tr = Trainer(m, 'e2e', fixed_param_prefix=['conv1', 'conv2'], lr=0.01, device='cpu', bucket_mb=64)
    names = tr.reducer.early_names
    g = torch.Generator().manual_seed(50 + rank)
    gt = torch.tensor([[[10., 20., 80., 100., 3.], [50., 60., 150., 140., 2.]]])
    for step in range(2):
        torch.manual_seed(100 * step + rank)
        tr.step({'data': torch.randn(1, 3, 128, 192, generator=g) * 50, 'im_info': torch.tensor([[128., 192., 1.0]]),
                 'gt_boxes': gt, 'n_gt': torch.tensor([2], dtype=torch.int32)})
    st = {k: v.clone() for k, v in tr.store.state_arrays().items()}
    st.update({'mom:' + k: v.clone() for k, v in tr.store.optimizer_state().items()})
    st['_early'] = torch.tensor([len(names), int('fc6_weight' in names)])
    torch.save(st, os.path.join(out_dir, 'f%d_%d.pt' % (int(early), rank)))
    pdist.barrier()
    pdist.destroy()


def test_vgg16_fc_update_after_allreduce_gloo():
    """under data parallelism VGG16's fc6 / fc7 buckets take their SGD as soon as
    their all-reduce completes (parallel/reducer.py sgd_names) and the end-of-step SGD skips them;
    two gloo ranks, two steps: weights and momenta bitwise equal to the plain end-of-step update, and
    the replicas agree."""
    with tempfile.TemporaryDirectory() as d:
        for early in (True, False):
            mp.spawn(_fc_worker, args=(2, _free_port(), d, early), nprocs=2, join=True)
        e0, e1 = [torch.load(os.path.join(d, 'f1_%d.pt' % r), weights_only=True) for r in range(2)]
        p0 = torch.load(os.path.join(d, 'f0_0.pt'), weights_only=True)
    assert int(e0['_early'][1]) == 1 and int(p0['_early'][0]) == 0
    keys = [k for k in p0 if not k.startswith('_')]
    assert len(keys) > 20
    for k in keys:
        assert torch.equal(e0[k], e1[k]), ('replicas differ', k)
        assert torch.equal(e0[k], p0[k]), ('early fc update differs from the end-of-step SGD', k)
