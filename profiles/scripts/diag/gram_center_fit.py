"""Centred vs uncentred Gram form vs the residual form vs the reference's own fp32 closure, against fp64, at fits
1e-1 .. 1e-5 (round 6): the fit-table problem of tests/test_gpu_gram.py::test_gram_precision_vs_fit
(teacher theta, frozen weights at the teacher, data noise), plus a VI-HMC-like case where the centre (the frozen
vector) is NOT the sampled theta (frozen = teacher + mu_noise, theta = teacher). Writes gpurun_out/r06_center_fit.json.
Usage: python gram_center_fit.py [noise ...]"""
import json
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

noises = [float(a) for a in sys.argv[1:]] or [1e-1, 1e-2, 1e-3, 1e-4, 1e-5]
s = DeepONetSpec()
lay = deeponet_layout(s.in_branch, s.width_branch, s.depth_branch, s.in_trunk, s.width_trunk, s.depth_trunk, s.out)
SD = 1e3
R = 3


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / np.linalg.norm(b))


rows = []
for case, mu_noise in (("teacher", 0.0), ("offcentre", 1e-3)):
    for noise in noises:
        p = deeponet_problem(seed=3, noise=noise, mu_noise=mu_noise)
        t0 = p.teacher[p.grad_ind].astype(np.float32)
        rng = np.random.default_rng(31)
        ths = [t0] + [(t0 * (1 + 1e-6 * rng.standard_normal(t0.size))).astype(np.float32) for _ in range(R - 1)]
        eng = DeepONetEngine(s, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, 0.0, SD, "NLL", 1.0,
                             max_chains=R, device="cuda:0")
        eng.option("gram_min_chains", 1)
        eng.option("gram_guard", 0)
        tt = torch.tensor(np.stack(ths), device="cuda:0")
        cols = {"gram_centred": [], "gram_uncentred": [], "residual": [], "ref_fp32": []}
        gc = eng.grad(tt).cpu().numpy()
        assert eng.get_option("gram") & 2
        eng.option("gram_center", 0)
        gu = eng.grad(tt).cpu().numpy()
        _, gr = eng.logp_grad(tt)
        gr = gr.cpu().numpy()
        ref = TorchDeepONetRef(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, 0.0, SD, "NLL", 1.0)
        fit = None
        for i, th in enumerate(ths):
            rl, g64, S = np_logp_grad(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, th, 0.0, SD, "NLL", 1.0)
            cols["gram_centred"].append(rel(gc[i], g64))
            cols["gram_uncentred"].append(rel(gu[i], g64))
            cols["residual"].append(rel(gr[i], g64))
            cols["ref_fp32"].append(rel(ref.logp_grad(th)[1], g64))
            if i == 0:
                y = p.y.astype(np.float64)
                fit = float(((S - y) ** 2).sum() / (y ** 2).sum())
        eng.close()
        med = {k: float(np.median(v)) for k, v in cols.items()}
        row = {"case": case, "noise": noise, "fit_ratio": fit, **{f"{k}_relnorm": v for k, v in cols.items()},
               **{f"{k}_median": v for k, v in med.items()},
               **{f"{k}_over_ref_fp32": med[k] / med["ref_fp32"] for k in ("gram_centred", "gram_uncentred", "residual")}}
        rows.append(row)
        print(f"{case:9s} noise {noise:7.0e} fit {fit:.2e}: " +
              " ".join(f"{k} {med[k]:.2e}" for k in cols) +
              f" | centred/ref {row['gram_centred_over_ref_fp32']:.2f} resid/ref {row['residual_over_ref_fp32']:.2f}",
              flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(rows, open(os.path.join(ROOT, "gpurun_out", "r06_center_fit.json"), "w"), indent=1)
