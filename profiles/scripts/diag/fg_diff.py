"""Where the fused-gather trajectory differs from the separate gather (debug aid): per L, the indices of differing
positions / momenta / gradients and their values. VIHMC_LIB selects the library."""
import os
import sys
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "vi-hmc_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from goldens import deeponet_case  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402

dev = torch.device("cuda", 0)
c = deeponet_case(sys.argv[1] if len(sys.argv) > 1 else "deeponet_burgers")
C = int(sys.argv[2]) if len(sys.argv) > 2 else 1
p = c.prob
rng = np.random.default_rng(17)
th0 = np.asarray(c.thetas[0], np.float32)
th = torch.tensor(np.stack([th0 + (0.01 * rng.standard_normal(th0.size)).astype(np.float32) for _ in range(C)]),
                  device=dev)
K = th.shape[1]
mom = torch.randn(C, K, generator=torch.Generator().manual_seed(5)).to(dev)
im = torch.linspace(0.5, 1.5, K, device=dev)
print("K", K, "D", c.spec.n_params, "grad_ind[:5]", p.grad_ind[:5])
for L in [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,3").split(",")]:
    out = []
    for fuse in (1, 0):
        eng = DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu,
                             c.prior_sd, c.loss, c.tau_out, max_chains=C, device=dev)
        eng.option("fuse_gather", fuse)
        _, g0 = eng.logp_grad(th)
        out.append([x.cpu() for x in eng.trajectory(th, mom, g0, 2e-3, L, inv_mass=im)] + [g0.cpu()])
        eng.close()
    for name, a, b in zip(("theta", "p", "logp", "grad", "g0"), out[0], out[1]):
        d = (a != b)
        n = int(d.sum())
        print(f"L={L} {name}: {n} differ", end="")
        if n and a.dim() == 2:
            idx = torch.nonzero(d)[:6].tolist()
            print(" at", idx, [(float(a[i][j]), float(b[i][j])) for i, j in idx[:3]], end="")
        print()
