"""Phase stamps of k_gram_a's T_b units from a -DVIHMC_DIAG=0x200 variant build.

    make -C vi-hmc_amd OUT=$PWD/_ab/grstamp.so BUILD=$PWD/build/grstamp EXTRA=-DVIHMC_DIAG=0x200
    VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$PWD/_ab/grstamp.so python profiles/scripts/diag/stamps_gram.py --chains 16

Every 16th T_b unit of the last k_gram_a launch records per wave (0-7 compute, 8 the DMA wave) and k block:
s_memtime at the barrier exit [0], after issuing the next block's loads (compute: A rows; DMA wave: the block two
ahead) [1], and after the block's MFMAs are issued (compute) / after the DMA wave's wait for the next block [2].
Per block (median over sampled units and blocks 2..nb-2): the period (barrier exit to barrier exit), the compute
waves' MFMA-issue span, the slack of the first / last compute wave to finish before the next barrier exit, and the
DMA wave's issue and wait times.
"""
import argparse
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

WG, NW, BLK = 32, 9, 48


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=16)
    a = ap.parse_args()
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    C = a.chains
    eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0, 0.1,
                         "NLL", 1.0, max_chains=C, device="cuda:0")
    eng.option("gram_min_chains", 1)
    th = torch.tensor(np.tile(prob.mu[prob.grad_ind], (C, 1)), device="cuda:0")
    th += 0.001 * torch.randn_like(th)
    for _ in range(5):
        eng.grad(th)
    torch.cuda.synchronize()
    assert eng.get_option("gram") & 2
    st = np.zeros((WG, NW, BLK, 3), np.uint64)
    rl = np.zeros((WG, 2, 2), np.uint64)
    f = _lib.lib().vihmc_debug_gram_stamps
    f.restype = ctypes.c_int
    rc = f(st.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(st.nbytes), rl.ctypes.data_as(ctypes.c_void_p),
           ctypes.c_size_t(rl.nbytes))
    assert rc == 0, rc
    st = st.astype(np.float64)
    rl = rl.astype(np.float64)
    ok = rl[:, 1, 1] > rl[:, 0, 1]
    cyc = rl[ok, 1, 0] - rl[ok, 0, 0]
    us = (rl[ok, 1, 1] - rl[ok, 0, 1]) / 100.0
    clk = np.mean(cyc / us)
    print(f"C={C}: T_b units sampled {ok.sum()}, unit duration {us.mean():.1f} us ({cyc.mean():.0f} cycles), "
          f"shader clock {clk / 1e3:.3f} GHz")
    rows = {k: [] for k in ("period", "a_issue", "mfma_issue", "first_done", "last_done", "dma_issue", "dma_wait")}
    nbs = []
    for g in np.nonzero(ok)[0]:
        bar = st[g, :, :, 0]
        nb = int(np.sum(bar[0] > 0))
        nbs.append(nb)
        for i in range(2, nb - 2):
            t0 = bar[:, i].min()
            t1 = bar[:, i + 1].min()
            rows["period"].append(t1 - t0)
            rows["a_issue"].append(np.median(st[g, :8, i, 1] - st[g, :8, i, 0]))
            rows["mfma_issue"].append(np.median(st[g, :8, i, 2] - st[g, :8, i, 1]))
            done = st[g, :8, i, 2]
            rows["first_done"].append(t1 - done.min())
            rows["last_done"].append(t1 - done.max())
            rows["dma_issue"].append(st[g, 8, i, 1] - st[g, 8, i, 0])
            rows["dma_wait"].append(st[g, 8, i, 2] - st[g, 8, i, 1])
    print(f"blocks per unit: {sorted(set(nbs))}")
    for k, v in rows.items():
        v = np.asarray(v)
        print(f"  {k:12s} median {np.median(v):8.0f} cycles  p10 {np.percentile(v, 10):8.0f}  p90 {np.percentile(v, 90):8.0f}")
    # MFMA floor per block: 2 compute waves per SIMD x 84 MFMA x 16 cycles
    print("  MFMA floor per block per SIMD: 2 waves x 84 x 16 = 2688 cycles")
    eng.close()


if __name__ == "__main__":
    main()
