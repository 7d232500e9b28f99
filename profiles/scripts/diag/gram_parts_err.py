"""Error of each Gram-form intermediate against fp64 (round 5 diagnostic): the fit-table problem (noise, teacher
theta), one chain (46 T_b slabs summed by k_gram_sum, 5 T_t splits in tt_part). From the plan's own buffers
(vihmc_plan_debug_copy): the pre-split images give the exact Zb^ / Zt^ the kernels used; against them, in fp64,
T_b = y Zt^, Gt = Zt^T Zt^, and the T_t accumulator (y^T Zb^ - Zt^ Gb), and the dZ each gives.
Usage: python gram_parts_err.py [noise]"""
import os
import sys
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

noise = float(sys.argv[1]) if len(sys.argv) > 1 else 1e-2
C = int(sys.argv[2]) if len(sys.argv) > 2 else 1
s = DeepONetSpec()
p = deeponet_problem(seed=3, noise=noise, mu_noise=0.0)
th = p.teacher[p.grad_ind].astype(np.float32)
eng = DeepONetEngine(s, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, 0.0, 1e3, "NLL", 1.0,
                     max_chains=C, device="cuda:0")
eng.option("gram_min_chains", 1)
eng.option("gram_guard", 0)
eng.grad(torch.tensor(np.stack([th] * C), device="cuda:0"))
assert eng.get_option("gram") & 2
N, P = p.N, p.P
BLK, PL, PITCH = 22528, 7168, 224


def image(name, rows):
    raw = eng.debug_buffer(name)
    nb = (rows + 31) // 32
    raw = raw[:raw.size // C]                            # chain 0
    out = np.zeros((nb * 32, 112))
    for pl in range(3):
        for b in range(nb):
            seg = raw[b * BLK + pl * PL: b * BLK + (pl + 1) * PL].view(np.uint16).reshape(32, 112)
            out[b * 32:(b + 1) * 32] += (seg.astype(np.uint32) << 16).view(np.float32)
    return out[:rows, :101]


Zb = image("bimg", N)
Zt = image("timg", P)
y = p.y.astype(np.float64)
Tb, Gt, Gb, Tt = y @ Zt, Zt.T @ Zt, Zb.T @ Zb, y.T @ Zb
acc_ex = Tt - Zt @ Gb
dzb_ex = Zb @ Gt - Tb


def tiles(raw, groups, ngroup_rows):
    """[groups][8 waves][14 tiles][256] (lane l, r: row 4(l >> 4) + r of the tile, column l & 15) -> rows x 112"""
    a = raw.reshape(groups, 8, 2, 7, 16, 4, 4)          # g, w, rt, t, lane(lg, lr)... lane = 16 lg + lr
    a = raw.reshape(groups, 8, 2, 7, 4, 16, 4)          # g, w, rt, t, lg, lr, r
    out = a.transpose(0, 1, 2, 4, 6, 3, 5).reshape(groups * 8 * 2 * 16, 7 * 16)  # rows (g w rt lg r), cols (t lr)
    return out[:ngroup_rows]


NG, PT = (N + 255) // 256, (P + 255) // 256
tbs = eng.debug_buffer("gram_tb_sum")
if tbs is not None:
    tbs = tbs[:tbs.size // C]
    tb_eng = tiles(tbs.view(np.float32)[:NG * 8 * 14 * 256].astype(np.float64), NG, N)[:, :101]
else:
    tbp = eng.debug_buffer("gram_tb")
    tbp = tbp[:tbp.size // C].view(np.float32).astype(np.float64)
    S = tbp.size // (NG * 8 * 14 * 256)
    tb_eng = sum(tiles(tbp[s_ * NG * 8 * 14 * 256:(s_ + 1) * NG * 8 * 14 * 256], NG, N) for s_ in range(S))[:, :101]
gt_eng = eng.debug_buffer("gram_gt").view(np.float32)[:112 * 112].reshape(112, 112)[:101, :101].astype(np.float64)
tt = eng.debug_buffer("gram_tt")
acc_eng = None
if tt is not None and tt.size:
    tt = tt[:tt.size // C].view(np.float32).astype(np.float64)
    SB = tt.size // (PT * 8 * 14 * 256)
    tt = tt.reshape(PT, SB, 8 * 14 * 256)
    acc_eng = sum(tiles(tt[:, sb].reshape(-1), PT, P) for sb in range(SB))[:, :101]
st = eng.debug_buffer("gram_stats")
st = st[:st.size // C].view(np.float64)
db_eng = st[1:2 * PT * 8:2].sum()                       # sum over (pt, wave) slots of d ll / d b0 (= -gscale acc)


def rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


print(f"noise {noise:g}: fit {((Zb @ Zt.T - y) ** 2).sum() / (y ** 2).sum():.3e}")
print(f"  T_b  = y Zt^        rel err {rel(tb_eng, Tb):.3e}   |T_b| / |dZb| = {np.linalg.norm(Tb) / np.linalg.norm(dzb_ex):.1f}")
print(f"  Gt   = Zt^T Zt^     rel err {rel(gt_eng, Gt):.3e}")
print(f"  dZb from T_b err    rel err {rel(Zb @ Gt - tb_eng, dzb_ex):.3e}")
print(f"  dZb from Gt err     rel err {rel(Zb @ gt_eng - Tb, dzb_ex):.3e}")
if acc_eng is not None:
    print(f"  T_t acc = y^T Zb^ - Zt^ Gb  rel err {rel(acc_eng, acc_ex):.3e}   |y^T Zb^| / |acc| = "
          f"{np.linalg.norm(Tt) / np.linalg.norm(acc_ex):.1f}")
print(f"  d ll / d b0: engine slots {db_eng:.6e} exact {acc_ex[:, 100].sum():.6e} (gscale = -1: d ll / d b0 = sum acc)"
      f" -> abs err {abs(db_eng - acc_ex[:, 100].sum()):.3e}")

# ---- gradient error of each intermediate's error, through an fp64 backward (the oracle's activations)
from oracle.deeponet_ref import deeponet_layout, np_forward, trunk_feats_np  # noqa: E402
lay = deeponet_layout(s.in_branch, s.width_branch, s.depth_branch, s.in_trunk, s.width_trunk, s.depth_trunk, s.out)
flat = p.mu.astype(np.float64).copy()
flat[p.grad_ind] = th
_, hs = np_forward(lay, flat, p.branch_in, trunk_feats_np(p.trunk_in))


def backward(dzb, dzt):
    br, tr, D = lay
    g = np.zeros(D)
    for name, layers, dz in (("b", br, dzb[:, :100]), ("t", tr, dzt[:, :100])):
        h, gg = hs[name], dz
        for j in range(len(layers) - 1, -1, -1):
            l = layers[j]
            d = gg if not l.act else gg * (1 - h[j + 1] ** 2)
            g[l.w_off:l.w_off + l.n_out * l.n_in] = (d.T @ h[j]).reshape(-1)
            g[l.b_off:l.b_off + l.n_out] = d.sum(0)
            if j > 0:
                gg = d @ flat[l.w_off:l.w_off + l.n_out * l.n_in].reshape(l.n_out, l.n_in)
    return g[p.grad_ind]


dzt_ex = -acc_ex                                          # gscale = -1: dZt = -gscale acc... (sign: dZt = acc * 1)
dzt_ex = acc_ex
g_ex = backward(dzb_ex, dzt_ex)
nrm = np.linalg.norm(g_ex)
gt32 = Gt.astype(np.float32).astype(np.float64)
gb32 = Gb.astype(np.float32).astype(np.float64)
terms = {"T_b (engine slabs)": (Zb @ Gt - tb_eng, dzt_ex),
         "Gt rounded to fp32 (exact)": (Zb @ gt32 - Tb, dzt_ex),
         "Gt (engine)": (Zb @ gt_eng - Tb, dzt_ex),
         "Gb rounded to fp32 (exact)": (dzb_ex, Tt - Zt @ gb32)}
if acc_eng is not None:
    terms["T_t acc (engine)"] = (dzb_ex, acc_eng)
for k, (a, b) in terms.items():
    print(f"  grad err from {k:28s} {np.linalg.norm(backward(a, b) - g_ex) / nrm:.3e}")
