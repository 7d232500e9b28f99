"""Phase stamps of the whole-network backward (k_bwd_chain) from a -DVIHMC_DIAG=0x40 variant build.

    make -C vi-hmc_amd OUT=$PWD/_ab/chstamp.so BUILD=$PWD/build/chstamp EXTRA=-DVIHMC_DIAG=0x40
    VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$PWD/_ab/chstamp.so python profiles/scripts/diag/stamps_chain.py

Every 8th workgroup of a single-chain Burgers evaluation records per wave and layer s_memtime after barrier A,
after A2, when its compute phase is done, after barrier B and when its write phase is done; printed per layer as
the mean cycles of each phase for the dX waves (0-7) and the dW waves (8-11), from the A exit of the layer.
"""
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

WG, MAXL = 16, 12


def main():
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0, 0.1,
                         "NLL", 1.0, max_chains=1, device="cuda:0")
    th = torch.tensor(prob.mu[prob.grad_ind], device="cuda:0")[None]
    for _ in range(5):
        eng.logp_grad(th)
    torch.cuda.synchronize()
    st = np.zeros((WG, 12, MAXL, 5), np.uint64)
    rl = np.zeros((WG, 2, 2), np.uint64)
    f = _lib.lib().vihmc_debug_ch_stamps
    f.restype = ctypes.c_int
    rc = f(st.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(st.nbytes), rl.ctypes.data_as(ctypes.c_void_p),
           ctypes.c_size_t(rl.nbytes))
    assert rc == 0, rc
    st = st.astype(np.float64)
    rl = rl.astype(np.float64)
    ok = rl[:, 1, 1] > rl[:, 0, 1]
    cyc = rl[ok, 1, 0] - rl[ok, 0, 0]
    us = (rl[ok, 1, 1] - rl[ok, 0, 1]) / 100.0
    print(f"workgroups sampled: {ok.sum()}  duration {us.mean():.1f} us  cycles {cyc.mean():.0f}  "
          f"shader clock {np.mean(cyc / us) / 1e3:.3f} GHz")
    first = st[ok][:, :, :, 0][st[ok][:, :, :, 0] > 0].min() if ok.any() else 0
    pro = [st[g, :, 8, 0].min() - rl[g, 0, 0] for g in np.nonzero(ok)[0]]
    print(f"prologue (start -> first A exit of layer 8): {np.mean(pro):.0f} cycles")
    print("layer | role | A->A2  A2->done  done->B  B->end | layer period (A to next A)")
    for j in range(MAXL - 1, -1, -1):
        per, rows = [], {"dX": [], "dW": []}
        for g in np.nonzero(ok)[0]:
            a = st[g, :, j, :]
            if not (a[:, 0] > 0).all():
                continue
            t0 = a[:, 0].min()
            if j > 0 and (st[g, :, j - 1, 0] > 0).all():
                per.append(st[g, :, j - 1, 0].min() - t0)
            for name, ws in (("dX", range(0, 8)), ("dW", range(8, 12))):
                b = a[list(ws)]
                rows[name].append([np.mean(b[:, 1] - b[:, 0]), np.mean(b[:, 2] - b[:, 1]), np.mean(b[:, 3] - b[:, 2]),
                                   np.mean(b[:, 4] - b[:, 3])])
        if not rows["dX"]:
            continue
        for name in ("dX", "dW"):
            m = np.mean(rows[name], axis=0)
            print(f"{j:5d} | {name}   | " + "  ".join(f"{v:7.0f}" for v in m) +
                  (f" | {np.mean(per):.0f}" if per and name == "dX" else ""))


if __name__ == "__main__":
    main()
