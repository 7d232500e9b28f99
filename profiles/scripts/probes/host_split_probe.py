"""Host time of config 4's fused splitting step (vihmc_split_step through _Engine.split_step) at one chain: the python
wrapper vs the C entry point, enqueue only (no synchronisation inside the loop), and the device wall time per call.

    python profiles/scripts/probes/host_split_probe.py
"""
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd")]

import torch  # noqa: E402

from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

spec = DeepONetSpec()
prob = deeponet_problem(seed=0, k=None)
half = prob.N // 2
tf = trunk_features(prob.trunk_in)
engs = [DeepONetEngine(spec, prob.branch_in[m * half:(m + 1) * half], tf, prob.y[m * half:(m + 1) * half], prob.mu,
                       prob.grad_ind, 0.0, 0.1, "NLL", 1.0, prior_scale=2.0, max_chains=1, device="cuda:0")
        for m in range(2)]
th = torch.tensor(prob.mu, device="cuda:0")[None].contiguous()
p = torch.zeros_like(th)
e0, e1 = engs
for _ in range(3):
    e0.split_step(th, p, 1, 1e-6, 1e-6, scatter_into=e1)
torch.cuda.synchronize()
for n in (8, 8, 8):
    t0 = time.perf_counter()
    for i in range(n):
        e0.split_step(th, p, 1, 1e-6, 1e-6, scatter_into=e1, scattered_in=i > 0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"split_step: host {(t1 - t0) / n * 1e3:.3f} ms/call, wall {(t2 - t0) / n * 1e3:.3f} ms/call", flush=True)
# the C entry point alone (same arguments as _Engine.split_step builds)
grad = torch.empty_like(th)
L = e0.L
stream = e0._stream()
for n in (8, 8):
    t0 = time.perf_counter()
    for i in range(n):
        L.vihmc_split_step(e0._plan, th.data_ptr(), p.data_ptr(), 1, grad.data_ptr(), None, 1, 1e-6, 1e-6, e1._plan,
                           int(i > 0), stream)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"vihmc_split_step (C call): host {(t1 - t0) / n * 1e3:.3f} ms/call, wall {(t2 - t0) / n * 1e3:.3f}", flush=True)
t0 = time.perf_counter()
for i in range(50):
    g = torch.empty(1, e0.K, device="cuda:0")
t1 = time.perf_counter()
print(f"torch.empty [1, K]: {(t1 - t0) / 50 * 1e6:.1f} us", flush=True)
