"""HMC iterations per second with the Metropolis step in one vihmc_hmc_accept launch vs its torch form
(HMCRunner._accept_native), alternating, at 16 chains and at one chain (bench workload, Burgers DeepONet, L = 7).

    python profiles/scripts/probes/probe_accept.py --reps 2
"""
import argparse
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd")]

import torch  # noqa: E402

from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402
from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    for C in (16, 1):
        eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0,
                             0.1, "NLL", 1.0, max_chains=C, device=dev)
        th0 = torch.tensor(prob.mu[prob.grad_ind], device=dev).repeat(C, 1)
        for rep in range(a.reps):
            for native in (True, False):
                r = HMCRunner(EngineEvaluator(eng), th0, a.steps + 3, 7, 1e-4, burn=0,
                              rng=ChainRNG(C, eng.K, dev, seeds=[1000 + c for c in range(C)]))
                r._accept_native = native
                for _ in range(3):
                    r.step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    r.step()
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                print(f"C={C} rep {rep} native={int(native)}: {C * 7 * a.steps / dt:9.1f} leapfrog-steps/s "
                      f"({dt / a.steps * 1e3:.3f} ms per HMC iteration)", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
