"""Time the paths next to the gradient evaluation (SURVEY §8 "next" rows) at Burgers shapes on the GPU.

    python profiles/scripts/probes/probe_paths.py [--chains 16] [--iters 10]

* value-only log-prob (hamiltorch's Hamiltonian evaluations at the accept step) -- engine.logp
* posterior-predictive forward (predict_model: out [C, N, P]) -- engine.forward
* half-data gradient evaluation (the splitting integrator's shard closures, N/2 functions each)
* sensitivity scores over N validation functions x p points (the step that writes gradient_indices)
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "vi-hmc_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc import sensitivity as S  # noqa: E402
from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402


def timed(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=16)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--sens-p", type=int, nargs="+", default=[100, 10201])
    args = ap.parse_args()
    C = args.chains
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    feats = trunk_features(prob.trunk_in)
    th_np = np.tile(prob.mu[prob.grad_ind], (C, 1))
    eng = DeepONetEngine(spec, prob.branch_in, feats, prob.y, prob.mu, prob.grad_ind, 0.0, 0.1, "NLL", 1.0,
                         max_chains=C, device="cuda:0")
    th = torch.tensor(th_np, device="cuda:0") + 0.001 * torch.randn(C, th_np.shape[1], device="cuda:0")
    t_g = timed(lambda: eng.logp_grad(th), args.iters)
    t_v = timed(lambda: eng.logp(th), args.iters)
    t_f = timed(lambda: eng.forward(th), max(2, args.iters // 2))
    print(f"C={C}  N={prob.N} P={prob.P}")
    print(f"  log-prob + gradient      {t_g * 1e3:8.3f} ms  ({C / t_g:9.1f} grad-evals/s)")
    print(f"  log-prob value only      {t_v * 1e3:8.3f} ms  ({C / t_v:9.1f} evals/s)")
    print(f"  predictive forward       {t_f * 1e3:8.3f} ms  ({C / t_f:9.1f} posterior samples/s, "
          f"{C * prob.N * prob.P / t_f / 1e9:.2f} G outputs/s)")
    eng.close()
    half = prob.N // 2
    eh = DeepONetEngine(spec, prob.branch_in[:half], feats, prob.y[:half], prob.mu, prob.grad_ind, 0.0, 0.1, "NLL",
                        1.0, max_chains=C, device="cuda:0")
    t_h = timed(lambda: eh.logp_grad(th), args.iters)
    print(f"  half-data grad (split)   {t_h * 1e3:8.3f} ms  ({C / t_h:9.1f} shard grad-evals/s; N/2 = {half})")
    eh.close()
    sd = np.full(prob.mu.size, 0.01, np.float32)
    for p in args.sens_p:
        pts = S.sample_points(prob.N, prob.P, min(p, prob.P), seed=3)
        S.sensitivity_scores(spec, prob.branch_in, prob.trunk_in, pts, prob.mu, sd)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        S.sensitivity_scores(spec, prob.branch_in, prob.trunk_in, pts, prob.mu, sd)
        t_s = time.perf_counter() - t0
        print(f"  sensitivity scores       {t_s * 1e3:8.1f} ms  (N = {prob.N} functions x p = {min(p, prob.P)} points, "
              f"{prob.N * min(p, prob.P) / t_s / 1e6:.2f} M output-gradients/s, plan build included)")


if __name__ == "__main__":
    main()
