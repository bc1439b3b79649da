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


def init_distributed(backend=None, timeout_s=600):
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
