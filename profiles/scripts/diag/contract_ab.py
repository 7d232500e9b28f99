"""A/B the side-A contraction kernels (fp32 k_contract_ws vs bf16x6 k_contract_bf) on the Burgers golden
case at several chain counts; prints logp / gradient differences and the worst gradient index."""
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "vi-hmc_amd")
from goldens import deeponet_case  # noqa: E402
from test_gpu_parity import engine_for  # noqa: E402

c = deeponet_case("deeponet_burgers")
for C in [int(a) for a in sys.argv[1:]] or [1, 2, 4, 16]:
    eng = engine_for(c, max_chains=C)
    th = torch.tensor(np.stack([c.thetas[0]] * C), device="cuda:0")
    r = {}
    for on in (0, 1):
        eng.option("contract_bf16x6", on)
        lp, g = eng.logp_grad(th)
        r[on] = (lp.double().cpu().numpy(), g.double().cpu().numpy())
    d = np.abs(r[1][1] - r[0][1])
    i = np.unravel_index(np.argmax(d), d.shape)
    print(f"C={C}: logp {r[0][0][0]:.6f} vs {r[1][0][0]:.6f}; grad max|d| {d.max():.3e} at {i} "
          f"(fp32 {r[0][1][i]:.6e}, bf {r[1][1][i]:.6e}); rel-norm {np.linalg.norm(d) / np.linalg.norm(r[0][1]):.2e}")
