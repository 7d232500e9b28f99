"""Per-kernel-class HIP-event times of the batched DeepONet evaluation (Burgers shapes), for A/B runs:

    python profiles/scripts/probes/probe_classes.py --chains 16 --iters 20 [--tag NAME]

Prints one line: eval ms and per-class ms per evaluation (include/vihmc.h VIHMC_T_*), measured with every class
timed (events add ~4 % to the evaluation), then the untimed wall per evaluation.
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
    ap.add_argument("--chains", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tag", default="")
    ap.add_argument("--opt", action="append", default=[], help="plan option key=value (repeatable)")
    ap.add_argument("--grad", action="store_true", help="gradient-only evaluations (vihmc_grad: the Gram form)")
    ap.add_argument("--config4", action="store_true",
                    help="config 4's evaluation: one data shard of N/2 functions, every parameter sampled")
    args = ap.parse_args()
    spec = DeepONetSpec()
    C = args.chains
    if args.config4:        # bench.py leg_split_c1's first shard
        prob = deeponet_problem(seed=0, k=None)
        half = prob.N // 2
        eng = DeepONetEngine(spec, prob.branch_in[:half], trunk_features(prob.trunk_in), prob.y[:half], prob.mu,
                             prob.grad_ind, 0.0, 0.1, "NLL", 1.0, prior_scale=2.0, max_chains=C, device="cuda:0")
    else:
        prob = deeponet_problem(seed=0)
        eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0,
                             0.1, "NLL", 1.0, max_chains=C, device="cuda:0")
    for kv in args.opt:
        k, v = kv.split("=")
        eng.option(k, int(v))
    th = torch.tensor(np.tile(prob.mu[prob.grad_ind], (C, 1)), device="cuda:0")
    th += 0.001 * torch.randn_like(th)
    ev = (lambda t: eng.grad(t)) if args.grad else (lambda t: eng.logp_grad(t))
    for _ in range(5):
        ev(th)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        ev(th)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.iters * 1e3
    eng.timing(-1, True)
    for _ in range(args.iters):
        ev(th)
    torch.cuda.synchronize()
    names = {0: "contract_a", 1: "contract_b", 2: "bwd", 3: "fwd", 4: "eval", 6: "gram"}
    out = {n: eng.timing_class(i)[0] / args.iters for i, n in names.items()}
    eng.timing(-1, False)
    print(f"{args.tag:12s} C={C} wall {wall:.4f} ms/eval | " + " ".join(f"{n} {v:.4f}" for n, v in out.items()),
          flush=True)


if __name__ == "__main__":
    main()
