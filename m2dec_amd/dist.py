"""Multi-GPU work-queue hand-off: independent streams, one per rank.

The data path has no collective.  The only exchanges are
  * a broadcast of the job table (one stream seed per rank) from rank 0, and
  * an all-gather of per-rank counters (pictures decoded, seconds) at the end,
over torch.distributed: backend "nccl" (= RCCL over xGMI) with device tensors on the GPU box,
"gloo" with CPU tensors in the CPU tests.
"""
from typing import List, Tuple


def job_table(dist, world: int, rank: int, device: str, first_seed: int = 1) -> List[int]:
    import torch

    seeds = list(range(first_seed, first_seed + world))
    if dist is None or world == 1:
        return seeds
    t = torch.tensor(seeds if rank == 0 else [0] * world, dtype=torch.int64, device=device)
    dist.broadcast(t, 0)
    return [int(x) for x in t.tolist()]


def gather_counters(dist, world: int, frames: int, seconds: float, device: str) -> Tuple[int, float, List[Tuple[int, float]]]:
    """Returns (total frames over ranks, max seconds over ranks, per-rank list)."""
    import torch

    if dist is None or world == 1:
        return frames, seconds, [(frames, seconds)]
    c = torch.tensor([float(frames), float(seconds)], dtype=torch.float64, device=device)
    outs = [torch.zeros_like(c) for _ in range(world)]
    dist.all_gather(outs, c)
    per = [(int(o[0].item()), float(o[1].item())) for o in outs]
    return sum(p[0] for p in per), max(p[1] for p in per), per


def all_ranks(dist, world: int, ok: bool, device: str) -> bool:
    """True iff `ok` holds on every rank (all-reduce MIN of one int); used for the per-rank parity gate."""
    import torch

    if dist is None or world == 1:
        return bool(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())
