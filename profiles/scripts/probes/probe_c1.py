"""Single-chain evaluation latency with and without HIP-event timing / hipGraph replay (the round-1 note:
C = 1 ran 2x faster under rocprofv3 than plain).

    python profiles/scripts/probes/probe_c1.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "vi-hmc_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402


def run(eng, th, iters, mode):
    if mode == "events":
        eng.timing(eng.T_EVAL, True)
    elif mode == "graph":
        eng.graph(True)
    elif mode == "sync":
        pass
    for _ in range(3):
        eng.logp_grad(th)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        eng.logp_grad(th)
        if mode == "sync":
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    ev = eng.timing_class(eng.T_EVAL) if mode == "events" else (0.0, 0)
    eng.timing(-1, False)
    eng.graph(False)
    return dt, ev


def main():
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0, 0.1,
                         "NLL", 1.0, max_chains=16, device="cuda:0")
    for C in (1, 2, 4, 16):
        th = torch.tensor(np.tile(prob.mu[prob.grad_ind], (C, 1)), device="cuda:0")
        th += 0.001 * torch.randn_like(th)
        for mode in ("plain", "events", "plain", "graph", "sync"):
            dt, (ms, n) = run(eng, th, 50, mode)
            print(f"C={C:3d} {mode:7s} wall {dt * 1e3:7.3f} ms/eval" +
                  (f"   events {ms / max(n, 1):7.3f} ms/eval" if n else ""), flush=True)


if __name__ == "__main__":
    main()
