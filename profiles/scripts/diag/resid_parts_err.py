"""Where the residual form's gradient error sits (round 6 diagnostic): the fit-table problem
(teacher theta, data noise), every layer output of the engine's forward (vihmc_plan_debug_copy act_b / act_t) and of
the reference's own fp32 closure, both against fp64. Prints, per fit:
  * per layer: rms relative error of h and its mean signed error in units of ulp(|h|) (a coherent bias adds up in the
    contraction's sums over 10.2 M points, a random error does not);
  * the gradient error of the whole evaluation, and of the forward alone (an fp64 contraction + backward fed with the
    engine's / the reference's fp32 activations), split by parameter group (b0, each layer's W and b).
Usage: python resid_parts_err.py [noise ...]"""
import os
import sys
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd"), os.path.join(ROOT, "tests")]
import json  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from oracle.deeponet_ref import TorchDeepONetRef, deeponet_layout, np_forward, trunk_feats_np  # noqa: E402
from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

noises = [float(a) for a in sys.argv[1:]] or [1e-2, 1e-3]
s = DeepONetSpec()
lay = deeponet_layout(s.in_branch, s.width_branch, s.depth_branch, s.in_trunk, s.width_trunk, s.depth_trunk, s.out)
br, tr, D = lay
SD = 1e3
R = 3


def backward64(flat, hs, y, idx, dz=None):
    """fp64 contraction + backward from the given layer outputs (the kernel spec of oracle.np_logp_grad); dz = the
    contraction's outputs {"b": dZ_b, "t": dZ_t} to start the backward from instead."""
    S = hs["b"][-1] @ hs["t"][-1].T + flat[0]
    G = -(S - y)
    g = np.zeros(D)
    g[0] = G.sum()
    if dz is None:
        dz = {"b": G @ hs["t"][-1], "t": G.T @ hs["b"][-1]}
    for name, layers in (("b", br), ("t", tr)):
        gg, h = dz[name], hs[name]
        for j in range(len(layers) - 1, -1, -1):
            l = layers[j]
            d = gg if not l.act else gg * (1 - h[j + 1] ** 2)
            g[l.w_off:l.w_off + l.n_out * l.n_in] = (d.T @ h[j]).reshape(-1)
            g[l.b_off:l.b_off + l.n_out] = d.sum(0)
            if j > 0:
                gg = d @ flat[l.w_off:l.w_off + l.n_out * l.n_in].reshape(l.n_out, l.n_in)
    return g[idx] - flat[idx] / (SD * SD)


def groups(idx):
    """parameter group of every sampled index: b0, then (net, layer, W|b)"""
    lab = np.empty(len(idx), dtype=object)
    for k, d in enumerate(idx):
        if d == 0:
            lab[k] = "b0"
            continue
        for name, layers in (("b", br), ("t", tr)):
            for j, l in enumerate(layers):
                if l.w_off <= d < l.w_off + l.n_out * l.n_in:
                    lab[k] = f"{name}{j}W"
                elif l.b_off <= d < l.b_off + l.n_out:
                    lab[k] = f"{name}{j}b"
    return lab


def torch_hs(ref, th):
    """the reference closure's fp32 layer outputs (its F.linear / tanh in its order)"""
    with torch.no_grad():
        flat = ref.mu.clone()
        flat[ref.idx] = torch.as_tensor(th)
        w = ref._views(flat)
        nb = len(ref.br)
        xb = ref.x1.reshape(-1, ref.br[0].n_in)
        hb = [xb.double().numpy()]
        for i in range(nb):
            xb = F.linear(xb, *w[i])
            if i < nb - 1:
                xb = torch.tanh(xb)
            hb.append(xb.double().numpy())
        X2 = ref.x2
        x_bc = torch.stack([torch.sin(2 * np.pi * X2[:, :, 1]), torch.sin(4 * np.pi * X2[:, :, 1]),
                            torch.cos(2 * np.pi * X2[:, :, 1]), torch.cos(4 * np.pi * X2[:, :, 1])], dim=2)
        xt = torch.cat([X2[:, :, 0].unsqueeze(dim=2), x_bc], dim=2)[0]
        ht = [xt.double().numpy()]
        for i in range(len(ref.tr)):
            xt = F.linear(xt, *w[nb + i])
            if i < len(ref.tr) - 1:
                xt = torch.tanh(xt)
            ht.append(xt.double().numpy())
    return {"b": hb, "t": ht}


def ulp32(x):
    a = np.abs(x).astype(np.float32)
    return np.spacing(np.maximum(a, np.float32(1e-30))).astype(np.float64)


rows = []
for noise in noises:
    p = deeponet_problem(seed=3, noise=noise, mu_noise=0.0)
    idx = p.grad_ind
    t0 = p.teacher[idx].astype(np.float32)
    rng = np.random.default_rng(31)
    ths = [t0] + [(t0 * (1 + 1e-6 * rng.standard_normal(t0.size))).astype(np.float32) for _ in range(R - 1)]
    eng = DeepONetEngine(s, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, idx, 0.0, SD, "NLL", 1.0,
                         max_chains=R, device="cuda:0")
    eng.option("debug_dz", 1)
    tt = torch.tensor(np.stack(ths), device="cuda:0")
    # the centred Gram form's gradient and contraction outputs first (gradient-only; the activations are then
    # overwritten by the residual-form evaluation below, whose act_b / act_t are read)
    eng.option("gram_min_chains", 1)
    eng.option("gram_guard", 0)
    gg = eng.grad(tt).cpu().numpy().astype(np.float64)
    assert eng.get_option("gram") & 2
    dzg = (eng.debug_buffer("dzb_snap").view(np.float32), eng.debug_buffer("dzt_snap").view(np.float32))
    _, ge = eng.logp_grad(tt)
    ge = ge.cpu().numpy().astype(np.float64)
    dzr = (eng.debug_buffer("dzb_snap").view(np.float32), eng.debug_buffer("dzt_snap").view(np.float32))
    ab = eng.debug_buffer("act_b").view(np.float32)
    at = eng.debug_buffer("act_t").view(np.float32)
    csb, cst = ab.size // R, at.size // R
    ref = TorchDeepONetRef(lay, p.branch_in, p.trunk_in, p.y, p.mu, idx, 0.0, SD, "NLL", 1.0)
    feats = trunk_feats_np(p.trunk_in)
    y = p.y.astype(np.float64)
    lab = groups(idx)
    glist = sorted(set(lab))
    acc = {}
    for i, th in enumerate(ths):
        flat = p.mu.astype(np.float64).copy()
        flat[idx] = th
        _, h64 = np_forward(lay, flat, p.branch_in, feats)
        g64 = backward64(flat, h64, y, idx)
        he = {"b": [h64["b"][0]], "t": [h64["t"][0]]}
        for name, layers, raw, cs, rows_ in (("b", br, ab, csb, p.N), ("t", tr, at, cst, p.P)):
            off = i * cs
            for j, l in enumerate(layers):
                he[name].append(raw[off + j * rows_ * 100: off + (j + 1) * rows_ * 100].reshape(rows_, 100)[:, :l.n_out]
                                .astype(np.float64))
        hr = torch_hs(ref, th)
        _, gr = ref.logp_grad(th)
        gr = gr.astype(np.float64)
        g_fe = backward64(flat, he, y, idx)
        g_fr = backward64(flat, hr, y, idx)

        def dz_of(snap):
            cb, ct = snap[0].size // R, snap[1].size // R
            return {"b": snap[0][i * cb: i * cb + p.N * 100].reshape(p.N, 100).astype(np.float64),
                    "t": snap[1][i * ct: i * ct + p.P * 100].reshape(p.P, 100).astype(np.float64)}
        # the engine's forward AND contraction, the rest (layer backward) in fp64
        g_fc = backward64(flat, he, y, idx, dz_of(dzr))
        g_fcg = backward64(flat, he, y, idx, dz_of(dzg))
        nrm = np.linalg.norm(g64)
        res = {"engine": ge[i], "ref_fp32": gr, "engine_fwd_only": g_fe, "ref_fwd_only": g_fr,
               "engine_fwd_contract": g_fc, "engine_gram": gg[i], "engine_gram_fwd_contract": g_fcg}
        for k, g in res.items():
            acc.setdefault(k, []).append(float(np.linalg.norm(g - g64) / nrm))
            for gname in glist:
                m = lab == gname
                acc.setdefault(f"{k}:{gname}", []).append(float(np.linalg.norm((g - g64)[m]) / nrm))
        if i == 0:
            for name in ("b", "t"):
                for j in range(1, len(he[name])):
                    ex = h64[name][j]
                    for who, hh in (("engine", he[name][j]), ("ref", hr[name][j])):
                        e = hh - ex
                        acc.setdefault(f"h_{who}_{name}{j}_rms", []).append(
                            float(np.sqrt((e ** 2).mean() / (ex ** 2).mean())))
                        acc.setdefault(f"h_{who}_{name}{j}_bias_ulp", []).append(float((e / ulp32(ex)).mean()))
            S64 = h64["b"][-1] @ h64["t"][-1].T + flat[0]
            acc["fit"] = [float(((S64 - y) ** 2).sum() / (y ** 2).sum())]
    eng.close()
    row = {"noise": noise, **{k: (float(np.median(v)) if len(v) > 1 else v[0]) for k, v in acc.items()}}
    rows.append(row)
    print(f"noise {noise:g}  fit {row['fit']:.3e}")
    for k in ("engine", "ref_fp32", "engine_fwd_only", "ref_fwd_only", "engine_fwd_contract", "engine_gram",
              "engine_gram_fwd_contract"):
        print(f"  grad rel err {k:18s} {row[k]:.3e}   by group: " +
              " ".join(f"{gname}={row[k + ':' + gname]:.1e}" for gname in glist
                       if row[k + ':' + gname] > 0.05 * row[k]))
    for name in ("b", "t"):
        for j in range(1, 10):
            kk = f"{name}{j}"
            if f"h_engine_{kk}_rms" in row:
                print(f"  h {kk}: engine rms {row[f'h_engine_{kk}_rms']:.2e} bias {row[f'h_engine_{kk}_bias_ulp']:+.3f} ulp"
                      f" | ref rms {row[f'h_ref_{kk}_rms']:.2e} bias {row[f'h_ref_{kk}_bias_ulp']:+.3f} ulp")
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(rows, open(os.path.join(ROOT, "gpurun_out", "resid_parts.json"), "w"), indent=1)
