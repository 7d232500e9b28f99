"""Sampling diagnostics: effective sample size (Geyer initial monotone sequence) and ESS/s.

The reference has no ESS or acceptance diagnostics beyond hamiltorch's printed acceptance rate
(SURVEY.md §5), so ESS/s is build-defined: Geyer's initial-monotone-sequence ESS of
(i) the log-prob trace and (ii) every sampled coordinate (min / median reported), per chain,
summed over chains.
"""
from __future__ import annotations

import torch


def autocorr(x: torch.Tensor) -> torch.Tensor:
    """Normalised autocorrelation along the last axis (FFT, biased estimator)."""
    x = x.to(torch.float64)
    n = x.shape[-1]
    x = x - x.mean(-1, keepdim=True)
    f = torch.fft.rfft(x, n=2 * n)
    ac = torch.fft.irfft(f * f.conj(), n=2 * n)[..., :n]
    v = ac[..., :1]
    return torch.where(v > 0, ac / torch.where(v > 0, v, torch.ones_like(v)), torch.zeros_like(ac))


def ess(x: torch.Tensor) -> torch.Tensor:
    """Geyer initial-monotone-sequence ESS along the last axis; any leading batch shape."""
    n = x.shape[-1]
    if n < 4:
        return torch.full(x.shape[:-1], float("nan"), dtype=torch.float64, device=x.device)
    rho = autocorr(x)
    m = n // 2
    G = rho[..., 0:2 * m:2] + rho[..., 1:2 * m:2]                  # Γ_k = ρ_2k + ρ_2k+1
    pos = G > 0
    first_neg = torch.where(pos.all(-1), torch.full(G.shape[:-1], m, device=x.device),
                            (~pos).to(torch.int64).argmax(-1))
    k = torch.arange(m, device=x.device)
    keep = k < first_neg[..., None]
    G = torch.where(keep, G, torch.zeros_like(G))
    G = torch.cummin(G, dim=-1).values                              # monotone
    G = torch.where(keep, G, torch.zeros_like(G))
    tau = -1.0 + 2.0 * G.sum(-1)
    tau = torch.clamp(tau, min=1.0 / max(n, 1))
    const = rho[..., 0] == 0                                        # constant chain (e.g. all rejected)
    out = n / tau
    return torch.where(const, torch.zeros_like(out), out)


def summarize(samples: torch.Tensor, logp_trace: torch.Tensor, wall_s: float) -> dict:
    """samples [C, S, K], logp_trace [C, S] -> ESS and ESS/s (summed over chains)."""
    e_lp = ess(logp_trace).sum().item()
    e_coord = ess(samples.transpose(1, 2)).sum(0)                    # [K]
    e_min = e_coord.min().item()
    e_med = e_coord.median().item()
    return {"ess_logp": e_lp, "ess_min": e_min, "ess_median": e_med,
            "ess_logp_per_s": e_lp / wall_s, "ess_min_per_s": e_min / wall_s, "ess_median_per_s": e_med / wall_s}
