"""Host time per HMC iteration of config 4's fused splitting runner at one chain, by phase (momentum draw, accept
draw, trajectory enqueue, Metropolis enqueue), against the device wall time -- which host call, if any, blocks.

    python profiles/scripts/probes/host_step_probe.py
"""
import collections
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd")]

import torch  # noqa: E402

from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402
from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner, Integrator  # noqa: E402

spec = DeepONetSpec()
prob = deeponet_problem(seed=0, k=None)
half = prob.N // 2
tf = trunk_features(prob.trunk_in)
engs = [DeepONetEngine(spec, prob.branch_in[m * half:(m + 1) * half], tf, prob.y[m * half:(m + 1) * half], prob.mu,
                       prob.grad_ind, 0.0, 0.1, "NLL", 1.0, prior_scale=2.0, max_chains=1, device="cuda:0")
        for m in range(2)]
evs = [EngineEvaluator(e) for e in engs]
th0 = torch.tensor(prob.mu, device="cuda:0")[None]
r = HMCRunner(evs, th0, 40, 7, 1e-4, integrator=Integrator.SPLITTING, rng=ChainRNG(1, spec.n_params, "cuda:0",
                                                                                   seeds=[1000]))
acc = collections.defaultdict(float)


def timed(obj, name, key):
    f = getattr(obj, name)

    def w(*a, **k):
        t = time.perf_counter()
        out = f(*a, **k)
        acc[key] += time.perf_counter() - t
        return out
    setattr(obj, name, w)


timed(r.rng, "draw_momentum", "draw_momentum")
timed(r.rng, "draw_logu", "draw_logu")
timed(r, "_trajectory", "trajectory")
timed(r, "_accept_fused", "accept")
timed(engs[0], "split_step", "split_step e0")
timed(engs[1], "split_step", "split_step e1")
timed(engs[1], "logp", "logp e1")
for _ in range(3):
    r.step()
torch.cuda.synchronize()
acc.clear()
n = 20
t0 = time.perf_counter()
for _ in range(n):
    t = time.perf_counter()
    r.step()
    acc["step"] += time.perf_counter() - t
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"per iteration: host {(t1 - t0) / n * 1e3:.3f} ms, wall {(t2 - t0) / n * 1e3:.3f} ms", flush=True)
for k, v in acc.items():
    print(f"  {k:16s} {v / n * 1e3:.3f} ms", flush=True)
