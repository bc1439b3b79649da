"""Hold ``--gb`` GB of device memory for ``--seconds`` (another process's cached allocations, as a
pytest parent holds them while a test runs subprocesses on the same card)."""
import argparse
import time

import torch

ap = argparse.ArgumentParser()
ap.add_argument('--gb', type=float, default=100)
ap.add_argument('--seconds', type=float, default=120)
ap.add_argument('--nan', action='store_true', help='fill with NaN (then exit: the freed pages keep it)')
a = ap.parse_args()
blocks = [torch.full((1 << 28,), float('nan') if a.nan else 1.0, device='cuda', dtype=torch.float32)
          for _ in range(int(a.gb))]
torch.cuda.synchronize()
print('holding', len(blocks), 'GB', flush=True)
time.sleep(a.seconds)
