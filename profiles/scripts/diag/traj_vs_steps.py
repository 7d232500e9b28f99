"""Debug: one BNN trajectory through vihmc_mlp_trajectory vs the step-by-step torch updates (first diff)."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "vi-hmc_amd"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "tests")]
import torch  # noqa: E402

from goldens import bnn_case  # noqa: E402
from vihmc.engine import MLPEngine  # noqa: E402

dev = torch.device("cuda", 0)
c = bnn_case("bnn_vi_hmc")
eng = MLPEngine(c.spec, c.data["x_train"], c.data["y_train"], c.g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                c.tau_out, max_chains=2, device=dev)
th0 = torch.tensor(c.thetas[0], device=dev)[None].repeat(2, 1)
lp0, g0 = eng.logp_grad(th0)
p0 = torch.randn(th0.shape, generator=torch.Generator().manual_seed(0)).to(dev)
eps = 1e-3
for L in (1, 2, 5):
    tf, pf, lf, gf = eng.trajectory(th0, p0, g0, eps, L)
    th, p, g = th0.clone(), p0 + (0.5 * eps) * g0, g0
    for s in range(L):
        th = th + eps * p
        lp, g = eng.logp_grad(th)
        p = p + eps * g
    p = p - (0.5 * eps) * g
    print(f"L={L} theta eq {torch.equal(tf, th)} maxdiff {float((tf - th).abs().max()):.3e}  p eq {torch.equal(pf, p)} "
          f"{float((pf - p).abs().max()):.3e}  g eq {torch.equal(gf, g)} {float((gf - g).abs().max()):.3e}  "
          f"lp {lf.tolist()} vs {lp.tolist()}")
# the evaluation alone at th0: trajectory with eps = 0 -> theta unchanged, g = grad(th0)
tf, pf, lf, gf = eng.trajectory(th0, p0, g0, 0.0, 1)
print("eps=0: theta eq", torch.equal(tf, th0), "g eq", torch.equal(gf, g0), float((gf - g0).abs().max()),
      "lp", lf.tolist(), lp0.tolist())
