"""Gradient-only evaluation time, Gram form vs residual form, per chain count (Burgers shapes; N = 1000 and the
splitting integrator's half shard N = 500). One plan per (N, C), max_chains = C, the form chosen by plan options.

    python profiles/scripts/probes/probe_crossover.py --chains 1 2 4 8 16 --iters 40
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "vi-hmc_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, nargs="+", default=[1, 2, 4, 8, 16])
    ap.add_argument("--rows", type=int, nargs="+", default=[1000, 500])
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    tf = trunk_features(prob.trunk_in)
    rng = np.random.default_rng(0)
    for rows in a.rows:
        for C in a.chains:
            th = torch.tensor(np.stack([prob.mu[prob.grad_ind] + 0.01 * rng.standard_normal(prob.grad_ind.size)
                                        for _ in range(C)]).astype(np.float32), device=dev)
            res = {}
            for form in ("residual", "gram"):
                eng = DeepONetEngine(spec, prob.branch_in[:rows], tf, prob.y[:rows], prob.mu, prob.grad_ind, 0.0, 0.1,
                                     "NLL", 1.0, max_chains=C, device=dev)
                if form == "gram":
                    eng.option("gram_min_chains", 1)
                else:
                    eng.option("gram", 0)
                best = 1e9
                for _ in range(a.reps):
                    for _ in range(3):
                        eng.grad(th)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(a.iters):
                        eng.grad(th)
                    torch.cuda.synchronize()
                    best = min(best, (time.perf_counter() - t0) / a.iters * 1e3)
                ran = eng.get_option("gram")
                assert bool(ran & 2) == (form == "gram"), (form, ran)
                res[form] = best
                eng.close()
            print(f"N={rows} C={C}: residual {res['residual']:.4f} ms, gram {res['gram']:.4f} ms per gradient-only "
                  f"evaluation (gram/residual {res['gram'] / res['residual']:.3f})", flush=True)


if __name__ == "__main__":
    main()
