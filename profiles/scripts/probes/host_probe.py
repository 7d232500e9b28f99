"""Host enqueue time vs GPU wall time per DeepONet evaluation (is a small-C evaluation launch-bound?)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."), "vi-hmc_amd"))
import numpy as np, torch
from vihmc.data import deeponet_problem
from vihmc.engine import DeepONetEngine, trunk_features
from vihmc.layout import DeepONetSpec
spec = DeepONetSpec(); prob = deeponet_problem(seed=0)
eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0, 0.1, "NLL", 1.0, max_chains=16, device="cuda:0")
for C in (1, 16):
    th = torch.tensor(np.tile(prob.mu[prob.grad_ind], (C, 1)), device="cuda:0")
    lp = torch.empty(C, device="cuda:0"); g = torch.empty(C, eng.K, device="cuda:0")
    for _ in range(5): eng.logp_grad(th, lp, g)
    torch.cuda.synchronize()
    n = 50
    t0 = time.perf_counter()
    for _ in range(n): eng.logp_grad(th, lp, g)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"C={C}: host enqueue {(t1-t0)/n*1e3:.3f} ms/call, wall {(t2-t0)/n*1e3:.3f} ms/call", flush=True)
