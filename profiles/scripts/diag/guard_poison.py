"""Which plan buffer does a kernel read past its end? Under VIHMC_GUARD=1 every buffer ends at an unmapped granule;
VIHMC_GUARD_POISON=k fills the bytes behind allocation k's end with 0xFF (NaN). For each k, rebuild the
cfg.sample_data closure of tests/test_gpu_api.py::test_deeponet_sample_data_closure_matches_golden, run its three
calls and report the log-prob errors: the k whose poison shows up names the buffer (VIHMC_GUARD_VERBOSE lists them)."""
import os
import random
import sys
import tempfile

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd"), os.path.join(ROOT, "tests")]
os.environ["VIHMC_GUARD"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402

from goldens import load, spec_of  # noqa: E402
from vihmc import configs  # noqa: E402
from vihmc.data import save_vi_artefacts  # noqa: E402
from vihmc.operator import define_model_log_prob  # noqa: E402

dev = torch.device("cuda", 0)
g = load("deeponet_sampledata")
spec = spec_of(g)
tmp = tempfile.mkdtemp()
save_vi_artefacts(tmp, "g", g["mu"], g["sigma"], g["grad_ind"])
cfg = configs.load("burgers_vi_hmc", prior_file=tmp, prior_uid="g", branch_depth=3, trunk_depth=3, sample_data=True,
                   p=int(g["p"]), prior_var=float(g["prior_var"]))
tr = (torch.from_numpy(g["branch_in"]), torch.from_numpy(g["trunk_in"]), torch.from_numpy(g["y"]))


def run(poison):
    os.environ["VIHMC_GUARD_POISON"] = str(poison)
    f = define_model_log_prob(spec, str(g["loss"]), tr, [torch.tensor(cfg.prior_var)], float(g["tau_out"]), device=dev,
                              cfg=cfg)
    random.seed(int(g["seed"]))
    errs = []
    for t in range(3):
        p = torch.tensor(g[f"theta{t}"], device=dev).requires_grad_()
        lp = float(f(p))
        ref = float(g[f"logp{t}"])
        errs.append(abs(lp - ref) / max(abs(ref), 1.0))
    f._vihmc_engine.close()
    return errs


os.environ["VIHMC_GUARD_VERBOSE"] = "1"
print("no poison:", run(-2), flush=True)
os.environ.pop("VIHMC_GUARD_VERBOSE")
print("all poisoned:", run(-1), flush=True)
for k in range(int(sys.argv[1]) if len(sys.argv) > 1 else 80):
    e = run(k)
    if max(e) > 1e-4 or not np.isfinite(e).all():
        print(f"alloc #{k}: errors {e}", flush=True)
print("done", flush=True)
