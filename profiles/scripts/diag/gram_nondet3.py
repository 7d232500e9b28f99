"""Which internal buffer first differs between repeated Gram-form gradient calls? (the guard test's 64-function teacher
shape, 4 distinct chains, layer-wise backward). After every grad call the plan's buffers are copied out
(vihmc_plan_debug_copy) and compared with the first call's, per chain."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

dev = torch.device("cuda", 0)
spec = DeepONetSpec()
p = deeponet_problem(seed=5, n=64, nt=21, nx=21, noise=1e-6, mu_noise=0.0)
t = p.teacher[p.grad_ind].astype(np.float32)
rng = np.random.default_rng(4)
pert = [(t + 0.05 * rng.standard_normal(t.size)).astype(np.float32) for _ in range(2)]
th = torch.tensor(np.stack([t, t] + pert), device=dev)
C = 4
NAMES = ["bimg", "timg", "act_b", "act_t", "gram_tb", "gram_gt_part", "gram_gt", "gram_gb", "gram_tt", "gram_stats",
         "dzb", "dzt"]
for opts in ({"bwd_chain": 0}, {}):
    eng = DeepONetEngine(spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, 0.0, 0.1, "NLL", 1.0,
                         max_chains=C, device=dev)
    eng.option("gram_guard", 0)
    for k, v in opts.items():
        eng.option(k, v)
    first = None
    g0 = None
    for call in range(6):
        g = eng.grad(th).cpu().numpy()
        bufs = {n: eng.debug_buffer(n) for n in NAMES}
        if first is None:
            first, g0 = bufs, g
            print(f"{opts}: sizes " + ", ".join(f"{n}={0 if b is None else b.size}" for n, b in bufs.items()), flush=True)
            continue
        diffs = []
        for n in NAMES:
            a, b = first[n], bufs[n]
            if a is None:
                continue
            cs = a.size // C
            per = [int(np.count_nonzero(a[c * cs:(c + 1) * cs] != b[c * cs:(c + 1) * cs])) for c in range(C)]
            if any(per):
                # first differing byte offset within the chain
                c = next(i for i in range(C) if per[i])
                off = int(np.nonzero(a[c * cs:(c + 1) * cs] != b[c * cs:(c + 1) * cs])[0][0])
                diffs.append(f"{n}: bytes per chain {per}, first at chain {c} +{off}")
        gd = np.abs(g - g0).max(axis=1)
        print(f"{opts} call {call}: grad maxdiff per chain {gd.tolist()}; " + ("; ".join(diffs) or "buffers same"),
              flush=True)
    eng.close()
