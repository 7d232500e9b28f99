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


def gather_ragged_pool(samples: torch.Tensor, counts: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """All-gather per-rank sample stores ``samples`` [C_local, S_cap, K] whose chain c holds ``counts[c]``
    valid samples. Chains that hit a ``LogProbError`` store fewer samples (hamiltorch appends nothing for
    them), so ranks differ in both the chain count and the stored length: every rank trims to its own
    longest chain, the blocks are padded to the job-wide maxima (one small all-gather of the shapes first)
    and exchanged by ONE all_gather_into_tensor. Returns the pool [C_total, S_max, K] (padding rows zero)
    and the per-chain counts [C_total], in rank order on every rank."""
    rank, ws = world()
    n_valid = int(counts.max().item()) if counts.numel() else 0
    valid = torch.arange(n_valid, device=samples.device)[None, :] < counts.to(samples.device)[:, None]
    local = torch.where(valid[:, :, None], samples[:, :n_valid], torch.zeros((), dtype=samples.dtype,
                                                                             device=samples.device))
    if ws == 1:
        return local, counts.clone()
    shape = torch.tensor([local.shape[0], local.shape[1]], device=local.device, dtype=torch.long)
    shapes = [torch.zeros_like(shape) for _ in range(ws)]
    dist.all_gather(shapes, shape)
    shapes = [(int(s[0].item()), int(s[1].item())) for s in shapes]
    cmax = max(s[0] for s in shapes)
    smax = max(s[1] for s in shapes)
    K = samples.shape[2]
    blk = torch.zeros((cmax, smax, K), device=local.device, dtype=local.dtype)
    blk[:local.shape[0], :local.shape[1]] = local
    cnt = torch.zeros(cmax, device=local.device, dtype=torch.long)
    cnt[:counts.numel()] = counts
    out = torch.empty((ws * cmax, smax, K), device=local.device, dtype=local.dtype)
    dist.all_gather_into_tensor(out, blk)
    out_cnt = torch.empty(ws * cmax, device=local.device, dtype=torch.long)
    dist.all_gather_into_tensor(out_cnt, cnt)
    keep = torch.cat([torch.arange(r * cmax, r * cmax + shapes[r][0], device=local.device) for r in range(ws)])
    return out[keep], out_cnt[keep]


def max_over_ranks(x: float, device) -> float:
    """The job's time for a per-rank wall time: the maximum over ranks (bench.py's contract)."""
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    if world()[1] > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_sum(t: torch.Tensor) -> torch.Tensor:
    if world()[1] > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t
