"""Phase stamps of the bf16x6 layer backward (k_bwd_bf) from a -DVIHMC_DIAG=0x20 variant build.

    make -C vi-hmc_amd OUT=$PWD/_ab/bbstamp.so BUILD=$PWD/build/bbstamp EXTRA=-DVIHMC_DIAG=0x20
    VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$PWD/_ab/bbstamp.so python profiles/scripts/diag/stamps_bwd.py

Every 16th trunk workgroup of the last launch with a dX part (layer 1) records per wave and 32-row sub-tile
s_memtime at the barrier exit and at the end of each phase of its role (csrc/vihmc_bwd_bf.hip BB_STAMP); printed per
role as cycles from the sub-tile's first barrier exit.
"""
import ctypes
import os
import sys

os.environ.setdefault("VIHMC_ALLOW_DIAG", "1")   # a stamp build is a diagnostic build

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "vi-hmc_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc import _lib  # noqa: E402
from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

WG, SUB, K = 16, 32, 6


def main():
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    C = 16
    eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0, 0.1,
                         "NLL", 1.0, max_chains=C, device="cuda:0")
    th = torch.tensor(np.tile(prob.mu[prob.grad_ind], (C, 1)), device="cuda:0")
    th += 0.001 * torch.randn_like(th)
    for _ in range(5):
        eng.logp_grad(th)
    torch.cuda.synchronize()
    st = np.zeros((WG, 16, SUB, K), np.uint64)
    rl = np.zeros((WG, 2, 2), np.uint64)
    f = _lib.lib().vihmc_debug_bb_stamps
    f.restype = ctypes.c_int
    rc = f(st.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(st.nbytes), rl.ctypes.data_as(ctypes.c_void_p),
           ctypes.c_size_t(rl.nbytes))
    assert rc == 0, rc
    st = st.astype(np.float64)
    rl = rl.astype(np.float64)
    ok = rl[:, 1, 1] > rl[:, 0, 1]
    cyc = rl[ok, 1, 0] - rl[ok, 0, 0]
    us = (rl[ok, 1, 1] - rl[ok, 0, 1]) / 100.0
    print(f"workgroups sampled: {ok.sum()}  duration {us.mean():.1f} us  shader clock {np.mean(cyc / us) / 1e3:.3f} GHz")
    per, pro, ns = [], [], []
    roles = {"dX (waves 0-7)": range(0, 8), "dW (waves 8-11)": range(8, 12), "staging (waves 12-15)": range(12, 16)}
    ph = {k: [[] for _ in range(K)] for k in roles}
    last = {k: [] for k in roles}
    for g in np.nonzero(ok)[0]:
        bar = st[g, :, :, 0]
        nsub = int(np.sum(bar[0] > 0))
        ns.append(nsub)
        pro.append(bar[:, 0].min() - rl[g, 0, 0])
        for i in range(1, nsub - 2):
            t0 = bar[:, i].min()
            per.append(bar[:, i + 1].min() - t0)
            for k, ws in roles.items():
                ends = []
                for w in ws:
                    for q in range(1, K):
                        v = st[g, w, i, q]
                        if v > 0:
                            ph[k][q].append(v - t0)
                            ends.append(v - t0)
                if ends:
                    last[k].append(max(ends))
    print(f"prologue (start -> first barrier exit) {np.mean(pro):7.0f} cycles; sub-tiles per workgroup {np.mean(ns):.1f}; "
          f"total {np.mean(cyc):.0f} cycles; barrier period {np.mean(per):.0f} (p10 {np.percentile(per, 10):.0f}, "
          f"p90 {np.percentile(per, 90):.0f})")
    names = {"dX (waves 0-7)": ["", "MFMAs issued", "epilogue stores", "h stores", "act'", "h loads"],
             "dW (waves 8-11)": ["", "", "MFMAs issued", "", "", ""],
             "staging (waves 12-15)": ["", "split + stores", "loads", "", "", ""]}
    for k in roles:
        print(f"  {k}: last phase end {np.mean(last[k]):.0f} (p90 {np.percentile(last[k], 90):.0f})")
        for q in range(1, K):
            if ph[k][q]:
                print(f"    [{q}] {names[k][q]:16s} {np.mean(ph[k][q]):7.0f} (p10 {np.percentile(ph[k][q], 10):6.0f}, "
                      f"p90 {np.percentile(ph[k][q], 90):6.0f})  from the sub-tile's first barrier exit")


if __name__ == "__main__":
    main()
