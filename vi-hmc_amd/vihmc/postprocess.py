"""Posterior-predictive evaluation of saved or in-memory HMC samples on the HIP engine.

Mirrors the reference's post-processing with the same file formats:
* ``get_list_fnames`` -- the uids listed in ``{out_dir}/fnames.txt`` (Operator_network/VI_HMC/post_process_burgers.py:261-282),
  and ``load_pooled_samples`` -- ``hmc_params_{uid}.npy`` [S_ret, K] fp32 per uid, ``[burn:]`` of each (:285-288);
* ``predictive`` -- the forward over every pooled sample (``predict_model`` / ``eval_VI_HMC``,
  main_VI_HMC_burgers.py:183-241,304-349), batched ``engine.max_chains`` samples per launch, returning the
  per-sample MSE and log-probability lists the reference prints, the fp64 posterior-predictive mean, and
  the per-sample per-function relative L2 errors of ``print_error`` (post_process_burgers.py:105-146);
* ``post_burn_per_chain`` -- each chain's own stored samples after burn (chains that hit a LogProbError
  store fewer samples; nothing requires equal counts).

Across ranks (chain-sharded runs) ``pool_ranks`` all-reduces the prediction sums and counts and all-gathers
the per-sample MSE / log-probability lists; the sample pool itself never moves.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Sequence

import numpy as np
import torch


def get_list_fnames(out_dir: str) -> List[str]:
    with open(os.path.join(out_dir, "fnames.txt")) as f:
        return [ln.strip() for ln in f if ln.strip()]


def append_fname(out_dir: str, uid: str):
    """Record a saved run's uid the way post_process_burgers.py expects to find it."""
    with open(os.path.join(out_dir, "fnames.txt"), "a") as f:
        f.write(uid + "\n")


def load_pooled_samples(out_dir: str, uids: Sequence[str], burn: int) -> List[torch.Tensor]:
    """``hmc_params_{uid}.npy`` [burn:] per uid (numpy.load without pickles)."""
    return [torch.from_numpy(np.load(os.path.join(out_dir, f"hmc_params_{u}.npy"), allow_pickle=False)[burn:])
            for u in uids]


def post_burn_per_chain(samples: torch.Tensor, counts: torch.Tensor, burn: int) -> List[torch.Tensor]:
    """Chain i's stored samples [burn:counts[i]] of a ChainResult (no equal-count requirement)."""
    return [samples[i, burn:int(counts[i])] for i in range(samples.shape[0])]


def l2_relative_error_t(y_true: torch.Tensor, y_pred: torch.Tensor) -> torch.Tensor:
    """post_process_burgers.py:105-121 on [..., N, P] tensors: per-function ||y - f|| / ||y||."""
    return torch.linalg.vector_norm(y_true - y_pred, dim=-1) / torch.linalg.vector_norm(y_true, dim=-1)


@dataclass
class Predictive:
    n: int = 0                                             # samples evaluated
    pred_sum: torch.Tensor = None                          # fp64 [N, P] sum of predictions
    mse: List[float] = field(default_factory=list)         # per-sample mean squared error (reference order)
    log_prob: List[float] = field(default_factory=list)    # per-sample log-probability on the data
    rel_l2: List[np.ndarray] = field(default_factory=list)  # per-sample [N] relative L2 errors

    def mean(self) -> torch.Tensor:
        return self.pred_sum / max(self.n, 1)


def predictive(engine, sample_sets: Sequence[torch.Tensor], y: torch.Tensor, with_rel_l2: bool = False) -> Predictive:
    """Forward of every sample of every set (sets = chains or saved files, in order) on ``engine`` (a
    DeepONetEngine / MLPEngine whose data are the evaluation set), ``engine.max_chains`` samples per launch."""
    dev = engine.device
    yd = y.to(dev).reshape(engine.out_shape)
    res = Predictive(pred_sum=torch.zeros(engine.out_shape, dtype=torch.float64, device=dev))
    B = engine.max_chains
    with torch.no_grad():
        for s in sample_sets:
            s = s.to(dev, torch.float32)
            for i in range(0, s.shape[0], B):
                lp, out = engine.forward(s[i:i + B])
                res.pred_sum += out.double().sum(0)
                res.n += out.shape[0]
                res.mse += ((out - yd) ** 2).mean(dim=tuple(range(1, out.dim()))).tolist()
                res.log_prob += lp.tolist()
                if with_rel_l2:
                    res.rel_l2 += list(l2_relative_error_t(yd.double(), out.double()).cpu().numpy())
    return res


def pool_ranks(p: Predictive) -> Predictive:
    """Job-wide predictive of a chain-sharded run: the prediction sums and counts all-reduced, the per-sample
    MSE / log-probability lists all-gathered in rank order (a few floats per sample), so every summary line
    covers every rank's samples. No-op in a single-process run."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return p
    n = torch.tensor([float(p.n)], dtype=torch.float64, device=p.pred_sum.device)
    dist.all_reduce(p.pred_sum)
    dist.all_reduce(n)
    p.n = int(n.item())
    lists = [None] * dist.get_world_size()
    dist.all_gather_object(lists, (p.mse, p.log_prob, p.rel_l2))
    p.mse = [v for l in lists for v in l[0]]
    p.log_prob = [v for l in lists for v in l[1]]
    p.rel_l2 = [v for l in lists for v in l[2]]
    return p


def print_summary(p: Predictive, y: torch.Tensor, with_rel_l2: bool = False):
    """The lines main_VI_HMC_burgers.py:293-300 / :343-349 and post_process_burgers.py print_error print."""
    print("\nExpected validation log probability: {:.2f}".format(float(np.mean(p.log_prob))))
    print("\nExpected MSE: {:.6f}".format(float(np.mean(p.mse))))
    print("\nFinal MSE: {:.6f}".format(p.mse[-1]))
    print("\nMin MSE:{:.6f}".format(min(p.mse)))
    mean = p.mean().cpu()
    err = l2_relative_error_t(y.double().reshape(mean.shape), mean)
    print("\nMean relative L2 error of the posterior-predictive mean: {:.6f}".format(float(err.mean())))
    if with_rel_l2 and p.rel_l2:
        e = np.stack(p.rel_l2)
        print("Mean Relative L2 error: ", float(e.mean()))
        print("MAP error: ", float(np.min(e.mean(axis=1))))
        print("Min error index: ", np.unravel_index(e.argmin(), e.shape))
        print("Max error index: ", np.unravel_index(e.argmax(), e.shape))
