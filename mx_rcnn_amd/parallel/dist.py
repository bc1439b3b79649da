"""Process-group bootstrap.  Reads RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT from the environment (torchrun / torch.distributed.run)."""
import datetime
import os

import torch
import torch.distributed as dist


def is_distributed():
    return dist.is_available() and dist.is_initialized()


def get_rank():
    return dist.get_rank() if is_distributed() else 0


def get_world_size():
    return dist.get_world_size() if is_distributed() else 1


# RCCL / torch ProcessGroup defaults for one 8 x MI355X node (set before the communicator is created;
# a value already in the environment wins):
# * NCCL_MIN_NCHANNELS=16: every GPU has 7 point-to-point xGMI links (~153 GB/s each); one RCCL
#   channel drives one ring, i.e. one link per hop.  The gradient buckets are 4-25 MB all-reduces
#   (parallel/reducer.py), large enough to be bandwidth-bound, so at least two channels per link
#   keep all 7 links busy; each channel costs one workgroup (16 of 256 CUs) that the overlapped
#   backward kernels lose while a collective runs.
# * TORCH_NCCL_ASYNC_ERROR_HANDLING=1: a failed or timed-out collective aborts the communicator
#   and raises on every rank (torchrun then tears the job down) instead of hanging the step.
# * TORCH_NCCL_CUDA_EVENT_CACHE=0: the process group's watchdog polls the completion events of the
#   eager (warm-up) collectives; with the event cache a finished work's event object is handed to a
#   collective recorded inside the step's hipGraph capture, and the watchdog's next poll of the old
#   work then fails with hipErrorCapturedEvent and aborts the process (seen on the 1-rank RCCL
#   graphed-step test, bf16x3).  Fresh events per work cost nothing measurable here (a few dozen
#   collectives per step, all inside the replayed graph).
# * collective timeout MXR_COLL_TIMEOUT (default 600 s) for init_process_group.
RCCL_DEFAULTS = {
    'NCCL_MIN_NCHANNELS': '16',
    'TORCH_NCCL_ASYNC_ERROR_HANDLING': '1',
    'TORCH_NCCL_CUDA_EVENT_CACHE': '0',
}


def rccl_env():
    """The effective RCCL settings (recorded in bench.py's JSON line)."""
    keys = list(RCCL_DEFAULTS) + ['NCCL_MAX_NCHANNELS', 'NCCL_ALGO', 'NCCL_PROTO', 'MXR_COLL_TIMEOUT']
    return {k: os.environ[k] for k in keys if k in os.environ}


def init_distributed(backend=None, timeout_s=None):
    """Initialise from env if WORLD_SIZE > 1.  Returns (rank, world_size, local_rank, device)."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    use_gpu = torch.cuda.is_available() and backend != 'gloo'
    device = torch.device('cuda', local_rank) if use_gpu else torch.device('cpu')
    if use_gpu:
        torch.cuda.set_device(device)
    force = os.environ.get('MXR_FORCE_DIST', '0') == '1'  # 1-rank process group (tests the RCCL paths)
    if (world > 1 or force) and not is_distributed():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        backend = backend or ('nccl' if use_gpu else 'gloo')
        kw = {}
        if backend == 'nccl':
            kw['device_id'] = device
            for k, v in RCCL_DEFAULTS.items():
                os.environ.setdefault(k, v)
        if timeout_s is None:
            timeout_s = int(os.environ.get('MXR_COLL_TIMEOUT', '600'))
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world, local_rank, device


def backend_name():
    """'nccl' (RCCL on ROCm), 'gloo', or None when not distributed."""
    return dist.get_backend() if is_distributed() else None


def barrier():
    if is_distributed():
        if dist.get_backend() == 'nccl':
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_max(value, device):
    """Max of a python float across ranks."""
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if is_distributed():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def destroy():
    if is_distributed():
        dist.destroy_process_group()
