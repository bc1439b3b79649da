"""Background GPU load for race hunting: keeps the device busy with bandwidth-heavy copies and
GEMMs for ``--seconds`` (a concurrently running test then sees perturbed stream timing, as when
other processes share the card).  Exits on its own.

    python tools/gpu_noise.py --seconds 120 &
"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--seconds', type=float, default=60)
    a = ap.parse_args()
    x = torch.randn(4096, 4096, device='cuda', dtype=torch.bfloat16)
    big = torch.empty(256 << 20, device='cuda', dtype=torch.uint8)
    big2 = torch.empty_like(big)
    t0 = time.time()
    while time.time() - t0 < a.seconds:
        for _ in range(20):
            big2.copy_(big)
            x = (x @ x).clamp_(-1, 1)
        torch.cuda.synchronize()


if __name__ == '__main__':
    main()
