"""Chain-parallel sampling across GPUs: one process per GPU, no collective on the data path.

The reference runs chains as separate SLURM jobs (Operator_network/VI_HMC/main_VI_HMC_burgers.py:252)
or sequentially (Neural_network/VI_HMC/main_VI_HMC.py:458-460) and pools them offline
(post_process_burgers.py:261-289). Here rank r of a torch.distributed job owns the contiguous chain
block [r*C/G, (r+1)*C/G); chain c is seeded by ``seed_base + c`` regardless of G, so a chain's samples
do not depend on the world size. The only exchange is one all-gather of the per-rank sample pools
(RCCL over xGMI with the ``nccl`` backend, ``gloo`` on CPU) at the end, plus an all-reduce of
accept counts / posterior-predictive sums.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def chain_block(total_chains: int, rank: int, world_size: int) -> range:
    """Contiguous chain ids owned by ``rank`` (balanced when world_size does not divide total)."""
    base, rem = divmod(total_chains, world_size)
    start = rank * base + min(rank, rem)
    return range(start, start + base + (1 if rank < rem else 0))


def chain_seeds(chains: range, seed_base: int = 1000) -> List[int]:
    return [seed_base + c for c in chains]


def gather_pool(local: torch.Tensor, total_chains: Optional[int] = None) -> torch.Tensor:
    """All-gather per-rank [C_local, S, K] sample pools into [C_total, S, K] on every rank.
    Ranks may own different chain counts; blocks are padded to the largest and trimmed."""
    rank, ws = world()
    if ws == 1:
        return local
    n_local = torch.tensor([local.shape[0]], device=local.device, dtype=torch.long)
    counts = [torch.zeros_like(n_local) for _ in range(ws)]
    dist.all_gather(counts, n_local)
    counts = [int(c.item()) for c in counts]
    cmax = max(counts)
    if local.shape[0] < cmax:
        pad = torch.zeros((cmax - local.shape[0],) + tuple(local.shape[1:]), device=local.device, dtype=local.dtype)
        local = torch.cat([local, pad])
    out = torch.empty((ws * cmax,) + tuple(local.shape[1:]), device=local.device, dtype=local.dtype)
    dist.all_gather_into_tensor(out, local.contiguous())
    blocks = [out[r * cmax:r * cmax + counts[r]] for r in range(ws)]
    return torch.cat(blocks)


def all_reduce_sum(t: torch.Tensor) -> torch.Tensor:
    if world()[1] > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t
