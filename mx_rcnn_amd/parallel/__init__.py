"""Data-parallel runtime: one process per GPU, torch.distributed over RCCL (backend
"nccl" resolves to RCCL on ROCm) or gloo on CPU, with our own bucketed gradient reducer."""
from .dist import init_distributed, get_rank, get_world_size, is_distributed, barrier, all_reduce_max  # noqa: F401
from .reducer import BucketReducer  # noqa: F401
from .watchdog import Heartbeat  # noqa: F401
