"""Device-side random subset selection with the reference's structure (no host sync).

numpy.random.choice cannot be bit-reproduced on the GPU; the contract
kept here is distributional + structural: uniform subsets without replacement, the
with-replacement pad PREPENDED exactly where the reference puts it
(`rcnn/rpn/proposal_target.py:148-180`), and exact counts.
"""
import torch

from .rng import uniform


def random_rank(mask, generator=None):
    """Per-row random rank of each True entry among the row's True entries (others >= count)."""
    keys = uniform(mask.shape, mask.device, generator)
    keys = torch.where(mask, keys, torch.full_like(keys, 2.0))
    order = torch.argsort(keys, dim=-1)
    rank = torch.empty_like(order)
    ar = torch.arange(mask.shape[-1], device=mask.device).expand_as(order)
    rank.scatter_(-1, order, ar)
    return rank, order


def keep_random(mask, limit, generator=None):
    """Keep a uniform random subset of at most ``limit`` (int or (B,) tensor) True entries per row."""
    rank, _ = random_rank(mask, generator)
    if not torch.is_tensor(limit):
        limit = torch.full(mask.shape[:-1], int(limit), device=mask.device, dtype=torch.long)
    return mask & (rank < limit[..., None])


def sample_slots(mask, n, generator=None):
    """Reference `npr.choice(w/o replacement, min(n, cnt))` + prepended with-replacement pad to n.

    Returns (idx (B, n) int64, take (B,) int64) where slots [0, n-take) are the pad (drawn
    from the sampled set) and [n-take, n) the sampled entries.
    """
    B, N = mask.shape
    _, order = random_rank(mask, generator)
    cnt = mask.sum(dim=-1)
    take = torch.clamp(cnt, max=n)
    pad = n - take
    j = torch.arange(n, device=mask.device)[None, :].expand(B, n)
    u = uniform((B, n), mask.device, generator)
    pick = torch.minimum((u * take[:, None].clamp_min(1)).long(), take[:, None].clamp_min(1) - 1)
    src = torch.where(j < pad[:, None], pick, j - pad[:, None])
    src = src.clamp(0, N - 1)
    return torch.gather(order, 1, src), take
