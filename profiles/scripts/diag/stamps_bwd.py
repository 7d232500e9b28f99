"""Phase stamps of the bf16x6 layer backward (k_bwd_bf) from a -DVIHMC_DIAG=0x20 variant build.

    make -C vi-hmc_amd OUT=$PWD/_ab/bbstamp.so BUILD=$PWD/build/bbstamp EXTRA=-DVIHMC_DIAG=0x20
    VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$PWD/_ab/bbstamp.so python profiles/scripts/diag/stamps_bwd.py

Every 16th trunk workgroup of the last launch with a dX part (layer 1) records per wave and 32-row sub-tile:
s_memtime at the barrier exit, after staging the next sub-tile (split + LDS stores + the loads two ahead), and
when its MFMA results exist; waves 0-7 are the dX role, 8-15 the dW role.
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

WG, SUB = 16, 32


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
    st = np.zeros((WG, 16, SUB, 3), np.uint64)
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
    rows = {k: [] for k in ("per", "xs", "xm", "ws", "wm", "xl", "wl")}
    for g in np.nonzero(ok)[0]:
        bar, stg, mm = st[g, :, :, 0], st[g, :, :, 1], st[g, :, :, 2]
        nsub = int(np.sum(bar[0] > 0))
        for i in range(1, nsub - 1):
            t0 = bar[:, i].min()
            rows["per"].append(bar[:, i + 1].min() - t0)
            rows["xs"].append(np.mean(stg[:8, i] - bar[:8, i]))
            rows["ws"].append(np.mean(stg[8:, i] - bar[8:, i]))
            rows["xm"].append(np.mean(mm[:8, i] - bar[:8, i]))
            rows["wm"].append(np.mean(mm[8:, i] - bar[8:, i]))
            rows["xl"].append(np.max(mm[:8, i]) - t0)
            rows["wl"].append(np.max(mm[8:, i]) - t0)
    pro, tail, ns = [], [], []
    for g in np.nonzero(ok)[0]:
        bar = st[g, :, :, 0]
        nsub = int(np.sum(bar[0] > 0))
        ns.append(nsub)
        pro.append(bar[:, 0].min() - rl[g, 0, 0])                      # start -> first barrier exit
        last = st[g, :, nsub - 1, 2].max() if nsub else rl[g, 0, 0]
        tail.append(rl[g, 1, 0] - last)                                   # last sub-tile's work -> workgroup end
    print(f"prologue (start -> first barrier exit) {np.mean(pro):7.0f} cycles; tail (last stamp -> end) "
          f"{np.mean(tail):7.0f}; sub-tiles per workgroup {np.mean(ns):.1f}; total {np.mean(cyc):.0f} cycles")
    f = lambda a: f"{np.mean(a):7.0f} (p10 {np.percentile(a, 10):6.0f}, p90 {np.percentile(a, 90):6.0f})"  # noqa: E731
    print("cycles per 32-row sub-tile (shader clock), steady state:")
    print(f"  barrier period               {f(rows['per'])}")
    print(f"  dX staging done (mean wave)   {f(rows['xs'])}")
    print(f"  dW staging done (mean wave)   {f(rows['ws'])}")
    print(f"  dX MFMAs done (mean wave)     {f(rows['xm'])}")
    print(f"  dW MFMAs done (mean wave)     {f(rows['wm'])}")
    print(f"  dX last wave done             {f(rows['xl'])}")
    print(f"  dW last wave done             {f(rows['wl'])}")
    g0 = int(np.nonzero(ok)[0][0])
    print("workgroup", g0, "sub-tile 5, per wave: barrier exit / staging done / MFMAs done, from the first exit")
    t0 = st[g0, :, 5, 0].min()
    v2 = os.environ.get("VIHMC_BWD_V2", "1") != "0"
    for w in range(16):
        role = ("dX" if w < 8 else "dW" if w < 12 else "stg") if v2 else ("dX" if w < 8 else "dW")
        print(f"  wave {w:2d} {role:3s} SIMD {w % 4}  {st[g0, w, 5, 0] - t0:6.0f} "
              f"{st[g0, w, 5, 1] - t0:6.0f} {st[g0, w, 5, 2] - t0:6.0f}")
    if v2:
        print("k_bwd_bf2 stamps: dX [1] = MFMAs done, [2] = epilogue stored; dW [1] = [2] = MFMAs done; "
              "staging [1] = [2] = next sub-tile staged (the 'staging done' rows above mix roles)")
    eng.close()


if __name__ == "__main__":
    main()
