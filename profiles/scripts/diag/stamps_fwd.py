"""Phase stamps of the bf16x6 fused forward (k_fwd_fused_bf) from a -DVIHMC_DIAG=0x10 variant build.

    make -C vi-hmc_amd OUT=$PWD/_ab/fwstamp.so BUILD=$PWD/build/fwstamp EXTRA=-DVIHMC_DIAG=0x10
    VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$PWD/_ab/fwstamp.so python profiles/scripts/diag/stamps_fwd.py --chains 1

Every 8th workgroup (the first 16) of the last forward records per wave and layer: s_memtime after the layer's
barrier [0], after the operand split (compute waves) / the next image's DMA issue (DMA waves) [1], after the layer's
MFMAs, epilogue and h stores are issued [2] (compute), after the wait before the next barrier [3].
"""
import argparse
import ctypes
import os
import sys

os.environ.setdefault("VIHMC_ALLOW_DIAG", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "vi-hmc_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc import _lib  # noqa: E402
from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

WG, NWV, NL = 16, 16, 10


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=1)
    a = ap.parse_args()
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    C = a.chains
    eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0, 0.1,
                         "NLL", 1.0, max_chains=C, device="cuda:0")
    th = torch.tensor(np.tile(prob.mu[prob.grad_ind], (C, 1)), device="cuda:0")
    th += 0.001 * torch.randn_like(th)
    for _ in range(5):
        eng.logp_grad(th)
    torch.cuda.synchronize()
    st = np.zeros((WG, NWV, NL, 4), np.uint64)
    rl = np.zeros((WG, 2, 2), np.uint64)
    f = _lib.lib().vihmc_debug_fwd_stamps
    f.restype = ctypes.c_int
    rc = f(st.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(st.nbytes), rl.ctypes.data_as(ctypes.c_void_p),
           ctypes.c_size_t(rl.nbytes))
    assert rc == 0, rc
    st = st.astype(np.float64)
    rl = rl.astype(np.float64)
    ok = rl[:, 1, 1] > rl[:, 0, 1]
    cyc = rl[ok, 1, 0] - rl[ok, 0, 0]
    us = (rl[ok, 1, 1] - rl[ok, 0, 1]) / 100.0
    print(f"C={C}: workgroups sampled {ok.sum()}, duration {us.mean():.1f} us ({cyc.mean():.0f} cycles), "
          f"shader clock {np.mean(cyc / us) / 1e3:.3f} GHz")
    nw = 4 if C <= 2 else 12
    print("layer | compute: bar->split  split->issued  issued->wait_done | DMA: bar->issued issued->done | period")
    for j in range(NL):
        rows = [g for g in np.nonzero(ok)[0] if st[g, 0, j, 0] > 0]
        if not rows:
            continue
        def m(w0, w1, k0, k1):
            return np.mean([np.mean(st[g, w0:w1, j, k1] - st[g, w0:w1, j, k0]) for g in rows])
        per = [st[g, :nw, j + 1, 0].min() - st[g, :nw, j, 0].min() for g in rows if j + 1 < NL and st[g, 0, j + 1, 0] > 0]
        dma = (m(nw, nw + 4, 0, 1), m(nw, nw + 4, 1, 3)) if C <= 2 else (0.0, 0.0)
        print(f"{j:5d} | {m(0, nw, 0, 1):8.0f} {m(0, nw, 1, 2):8.0f} {m(0, nw, 2, 3):8.0f} | {dma[0]:8.0f} {dma[1]:8.0f} | "
              f"{np.mean(per) if per else float('nan'):8.0f}")
    eng.close()


if __name__ == "__main__":
    main()
