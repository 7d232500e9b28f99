"""Where does the Gram form's gradient error sit at the fit-table problem (round 5)? Full Burgers shape, theta at the
teacher, frozen weights at the teacher, data noise `noise` (tests/test_gpu_gram.py::test_gram_precision_vs_fit): the
norm of |g - g_fp64| per parameter group (b0, each layer's W and b of both nets) for the Gram form, the residual form
and the reference's fp32 closure (TorchDeepONetRef, CPU). Usage: python gram_fit_err.py [noise] [chains]"""
import os
import sys
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from oracle.deeponet_ref import TorchDeepONetRef, deeponet_layout, np_logp_grad  # noqa: E402
from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

noise = float(sys.argv[1]) if len(sys.argv) > 1 else 1e-2
C = int(sys.argv[2]) if len(sys.argv) > 2 else 3
s = DeepONetSpec()
sd = 1e3
p = deeponet_problem(seed=3, noise=noise, mu_noise=0.0)
th = p.teacher[p.grad_ind].astype(np.float32)
eng = DeepONetEngine(s, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, 0.0, sd, "NLL", 1.0,
                     max_chains=C, device="cuda:0")
eng.option("gram_min_chains", 1)
eng.option("gram_guard", 0)
tt = torch.tensor(np.stack([th] * C), device="cuda:0")
gg = eng.grad(tt)[0].cpu().numpy().astype(np.float64)
gr = eng.logp_grad(tt)[1][0].cpu().numpy().astype(np.float64)
lay = deeponet_layout(s.in_branch, s.width_branch, s.depth_branch, s.in_trunk, s.width_trunk, s.depth_trunk, s.out)
_, rg, _ = np_logp_grad(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, th, 0.0, sd, "NLL", 1.0)
_, g32 = TorchDeepONetRef(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, 0.0, sd, "NLL", 1.0).logp_grad(th)
g32 = np.asarray(g32, np.float64)
br, tr, D = lay
flat_of = np.full(D, -1, np.int64)
flat_of[np.asarray(p.grad_ind)] = np.arange(len(p.grad_ind))
groups = [("b0", [0])]
for name, layers in (("branch", br), ("trunk", tr)):
    for j, l in enumerate(layers):
        groups.append((f"{name}{j}.W", list(range(l.w_off, l.w_off + l.n_out * l.n_in))))
        groups.append((f"{name}{j}.b", list(range(l.b_off, l.b_off + l.n_out))))
nrm = np.linalg.norm(rg)
print(f"noise {noise:g}, C = {C}: |g| {nrm:.4e}; relnorm gram {np.linalg.norm(gg - rg) / nrm:.3e} residual "
      f"{np.linalg.norm(gr - rg) / nrm:.3e} ref_fp32 {np.linalg.norm(g32 - rg) / nrm:.3e}")
print(f"  {'group':12s} {'n':>6s} {'|ref|':>10s} {'gram':>10s} {'residual':>10s} {'ref_fp32':>10s}   (error norms / |g|)")
for gname, fl in groups:
    k = flat_of[np.asarray(fl)]
    k = k[k >= 0]
    if k.size == 0:
        continue
    e = [np.linalg.norm(x[k] - rg[k]) / nrm for x in (gg, gr, g32)]
    print(f"  {gname:12s} {k.size:6d} {np.linalg.norm(rg[k]) / nrm:10.3e} {e[0]:10.3e} {e[1]:10.3e} {e[2]:10.3e}")
