"""Where does the Gram form's gradient error sit? Full Burgers shape, perturbed golden theta: |g - g_fp64| per
parameter group (the output bias b0, then each layer of both nets) for the Gram and the residual form."""
import os
import sys
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from goldens import deeponet_case  # noqa: E402
from oracle.deeponet_ref import deeponet_layout, np_logp_grad  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402

c = deeponet_case("deeponet_burgers")
p, s = c.prob, c.spec
th0 = np.asarray(c.thetas[0], np.float32)
th1 = (th0 + 0.01 * np.random.default_rng(11).standard_normal(th0.size)).astype(np.float32)
eng = DeepONetEngine(s, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu, c.prior_sd,
                     c.loss, c.tau_out, max_chains=2, device="cuda:0")
th = torch.tensor(np.stack([th0, th1]), device="cuda:0")
gg = eng.grad(th).cpu().numpy().astype(np.float64)
gr = eng.logp_grad(th)[1].cpu().numpy().astype(np.float64)
lay = deeponet_layout(s.in_branch, s.width_branch, s.depth_branch, s.in_trunk, s.width_trunk, s.depth_trunk, s.out)
br, tr, D = lay
flat_of = np.full(D, -1, np.int64)
flat_of[np.asarray(p.grad_ind)] = np.arange(len(p.grad_ind))
groups = [("b0", [0])]
for name, layers in (("branch", br), ("trunk", tr)):
    for j, l in enumerate(layers):
        groups.append((f"{name}{j}.W", list(range(l.w_off, l.w_off + l.n_out * l.n_in))))
        groups.append((f"{name}{j}.b", list(range(l.b_off, l.b_off + l.n_out))))
for i, t in enumerate([th0, th1]):
    _, rg, _ = np_logp_grad(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, t, c.prior_mu, c.prior_sd, c.loss,
                            c.tau_out)
    print(f"theta{i}: max|g| {np.abs(rg).max():.4e} at {int(np.abs(rg).argmax())}; |g| {np.linalg.norm(rg):.4e}")
    for gname, fl in groups:
        k = flat_of[np.asarray(fl)]
        k = k[k >= 0]
        if k.size == 0:
            continue
        ref = rg[k]
        eg = np.abs(gg[i][k] - ref).max()
        er = np.abs(gr[i][k] - ref).max()
        print(f"  {gname:12s} n={k.size:6d} max|ref| {np.abs(ref).max():.3e}  gram err {eg:.3e}  residual err {er:.3e}")
