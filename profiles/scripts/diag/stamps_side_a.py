"""Phase stamps of the side-A contraction (k_contract_bf) from a -DVIHMC_DIAG=0x80 variant build.

    make -C vi-hmc_amd OUT=$PWD/_ab/stamp.so BUILD=$PWD/build/stamp EXTRA=-DVIHMC_DIAG=0x80
    VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$PWD/_ab/stamp.so python profiles/scripts/diag/stamps_side_a.py

Every 64th workgroup records, per wave and chunk, s_memtime at the barrier exit and when the chunk's
results exist (S role: G and the likelihood partial; D role: the dZ_t accumulators), plus s_memtime /
s_memrealtime (100 MHz) at its start and end -> the shader clock under load, the barrier period, and how
much of it each role's work fills.
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

WG, CH = 24, 40


def main():
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    C = int(os.environ.get("STAMP_CHAINS", "16"))
    eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0, 0.1,
                         "NLL", 1.0, max_chains=C, device="cuda:0")
    th = torch.tensor(np.tile(prob.mu[prob.grad_ind], (C, 1)), device="cuda:0")
    th += 0.001 * torch.randn_like(th)
    for _ in range(5):
        eng.logp_grad(th)
    torch.cuda.synchronize()
    st = np.zeros((WG, 16, CH, 3), np.uint64)
    rl = np.zeros((WG, 2, 2), np.uint64)
    f = _lib.lib().vihmc_debug_cb_stamps
    f.restype = ctypes.c_int
    rc = f(st.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(st.nbytes), rl.ctypes.data_as(ctypes.c_void_p),
           ctypes.c_size_t(rl.nbytes))
    assert rc == 0, rc
    st = st.astype(np.float64)
    rl = rl.astype(np.float64)
    ok = rl[:, 1, 1] > rl[:, 0, 1]
    cyc = rl[ok, 1, 0] - rl[ok, 0, 0]
    us = (rl[ok, 1, 1] - rl[ok, 0, 1]) / 100.0
    print(f"workgroups sampled: {ok.sum()}  duration {us.mean():.1f} us  shader clock {np.mean(cyc / us) / 1e3:.3f} GHz "
          f"(min {np.min(cyc / us) / 1e3:.3f}, max {np.max(cyc / us) / 1e3:.3f}), cycles {np.mean(cyc):.0f}")
    per, s_work, d_work, skew, s_late, d_late, s_mid, d_mid = [], [], [], [], [], [], [], []
    pro, epi, nchs = [], [], []
    for g in np.nonzero(ok)[0]:
        nch = int((st[g, 8, :, 0] > 0).sum())   # the D role's iterations: the chunks + its trailing one
        pro.append(st[g, :, 0, 0].min() - rl[g, 0, 0])
        epi.append(rl[g, 1, 0] - st[g, :, nch - 1, 0].max())
        nchs.append(nch)
        bar = st[g, :, :nch, 0]
        end = st[g, :, :nch, 1]
        mid = st[g, :, :nch, 2]
        for i in range(1, nch - 1):
            t0 = bar[:, i].min()
            per.append(bar[:, i + 1].min() - t0)
            skew.append(bar[:, i].max() - t0)
            s_work.append(np.mean(end[:8, i] - bar[:8, i]))
            d_work.append(np.mean(end[8:, i] - bar[8:, i]))
            s_late.append(np.max(end[:8, i]) - t0)
            s_mid.append(np.mean(mid[:8, i] - bar[:8, i]))
            d_mid.append(np.mean(mid[8:, i] - bar[8:, i]))
            d_late.append(np.max(end[8:, i]) - t0)
    f = lambda a: f"{np.mean(a):7.0f} (p10 {np.percentile(a, 10):6.0f}, p90 {np.percentile(a, 90):6.0f})"  # noqa: E731
    print(f"chunks per workgroup (D role iterations) {np.mean(nchs):.1f}")
    print(f"  prologue (start -> first barrier exit) {f(pro)}")
    print(f"  epilogue (last barrier exit -> end)     {f(epi)}")
    print("cycles per chunk (shader clock), steady-state chunks:")
    print(f"  barrier period              {f(per)}")
    print(f"  barrier-exit skew            {f(skew)}")
    print(f"  S role work (mean wave)      {f(s_work)}")
    print(f"  D role work (mean wave)      {f(d_work)}")
    print(f"  S role first sub-tile done   {f(s_mid)}")
    print(f"  D role G split done          {f(d_mid)}")
    print(f"  S role last wave done        {f(s_late)}")
    print(f"  D role last wave done        {f(d_late)}")
    g0 = int(np.nonzero(ok)[0][0])
    print("workgroup", g0, "chunk 5, per wave: barrier exit / mid (S: first sub-tile, D: G split) / done, from the first exit")
    t0 = st[g0, :, 5, 0].min()
    for w in range(16):
        print(f"  wave {w:2d} {'S' if w < 8 else 'D'}  {st[g0, w, 5, 0] - t0:6.0f} {st[g0, w, 5, 2] - t0:6.0f} "
              f"{st[g0, w, 5, 1] - t0:6.0f}")
    eng.close()


if __name__ == "__main__":
    main()
