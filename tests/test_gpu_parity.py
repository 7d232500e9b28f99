"""HIP path vs oracle / reference goldens, through the C-ABI (libvihmc.so via vihmc.engine).

Tolerances: every error is recorded and checked by tests/parity.py against a bound per (test, quantity) set
from the errors measured on the MI355X (about 4x the largest over the test's cases; profiles/r03_parity_errors.json).
"""
import numpy as np
import pytest
import torch

import parity
from goldens import BNN_CASES, DEEPONET_CASES, bnn_case, deeponet_case, load, spec_of
from oracle.deeponet_ref import deeponet_layout, np_logp_grad

pytestmark = pytest.mark.gpu


def rel_norm(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def engine_for(c, max_chains=4, device="cuda:0"):
    from vihmc.engine import DeepONetEngine, trunk_features
    p = c.prob
    return DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu,
                          c.prior_sd, c.loss, c.tau_out, max_chains=max_chains, device=device)


def check_logp(lp, ref, note=""):
    parity.check("logp_rel", abs(lp - ref) / max(abs(ref), 1.0), note)


def check_grad(g, ref, note=""):
    g = np.asarray(g, np.float64)
    ref = np.asarray(ref, np.float64)
    parity.check("grad_relnorm", rel_norm(g, ref), note)
    parity.check("grad_elem", np.abs(g - ref).max() / np.abs(ref).max(), note)


def check_grad_sub(g, sub, gs, ref_norm, note=""):
    """full-shape goldens: a 4,096-entry subsample of the gradient and the norm of the whole gradient"""
    g = np.asarray(g, np.float64)
    gs = np.asarray(gs, np.float64)
    parity.check("grad_elem", np.abs(g[sub] - gs).max() / np.abs(gs).max(), note)
    parity.check("grad_norm_rel", abs(np.linalg.norm(g) - ref_norm) / ref_norm, note)


def check_pred(out, pred, note=""):
    out = np.asarray(out, np.float64)
    pred = np.asarray(pred, np.float64)
    parity.check("pred_elem", np.abs(out - pred).max() / np.abs(pred).max(), note)


@pytest.mark.parametrize("name", DEEPONET_CASES + ["deeponet_burgers"])
def test_deeponet_engine_matches_golden(name, cuda_device):
    c = deeponet_case(name)
    eng = engine_for(c, max_chains=len(c.thetas))
    th = torch.tensor(np.stack(c.thetas), device=cuda_device)
    lp, g = eng.logp_grad(th)
    lp, g = lp.cpu().numpy(), g.cpu().numpy()
    for t in range(len(c.thetas)):
        check_logp(float(lp[t]), float(c.g[f"logp{t}"]), f"{name} theta{t}")
        if f"grad{t}" in c.g:
            check_grad(g[t], c.g[f"grad{t}"], f"{name} theta{t}")
        else:
            check_grad_sub(g[t], c.g["grad_subsample"], c.g[f"grad{t}_sub"], float(c.g[f"grad{t}_norm"]),
                           f"{name} theta{t}")
        if f"pred{t}" in c.g:
            lpf, out = eng.forward(th[t:t + 1])
            check_pred(out[0].cpu().numpy(), c.g[f"pred{t}"], f"{name} theta{t}")
            check_logp(float(lpf[0]), float(c.g[f"logp{t}"]), f"{name} forward theta{t}")


@pytest.mark.parametrize("C,fwd_bf16x6,contract_bf16x6,bwd_bf16x6", [(1, 1, 1, 1), (4, 1, 1, 1), (16, 1, 1, 1),
                                                                    (16, 0, 0, 0), (16, 1, 0, 1), (3, 0, 1, 0)])
def test_deeponet_burgers_every_launch_geometry(C, fwd_bf16x6, contract_bf16x6, bwd_bf16x6, cuda_device):
    """Burgers shape at the chain counts that select different launch geometries (fused forward 4- vs
    12-wave workgroups, fp32 or bf16x6 hidden-layer products, contraction q-splits, backward row chunks):
    every chain (replicated golden thetas) must match the reference closure's golden."""
    c = deeponet_case("deeponet_burgers")
    eng = engine_for(c, max_chains=C)
    eng.option("fwd_bf16x6", fwd_bf16x6)
    eng.option("contract_bf16x6", contract_bf16x6)
    eng.option("bwd_bf16x6", bwd_bf16x6)
    n = len(c.thetas)
    th = torch.tensor(np.stack([c.thetas[i % n] for i in range(C)]), device=cuda_device)
    lp, g = eng.logp_grad(th)
    lp, g = lp.cpu().numpy(), g.cpu().numpy()
    sub = c.g["grad_subsample"]
    for i in range(C):
        t = i % n
        note = f"C={C} forms={fwd_bf16x6}{contract_bf16x6}{bwd_bf16x6} chain {i}"
        check_logp(float(lp[i]), float(c.g[f"logp{t}"]), note)
        check_grad_sub(g[i], sub, c.g[f"grad{t}_sub"], float(c.g[f"grad{t}_norm"]), note)


@pytest.mark.parametrize("name", ["deeponet_burgers", "deeponet_refshape"])
def test_single_chain_kernels_bitwise_equal_batched_kernels(name, cuda_device):
    """Single-chain plans run the backward of both nets in one launch (k_bwd_chain: deltas kept in LDS, W^T from
    the scatter-kept transposed images); it must equal the nine per-layer k_bwd_bf2 launches bit for bit, and
    match the golden."""
    c = deeponet_case(name)
    eng = engine_for(c, max_chains=1)
    res = {}
    for fs, bc in ((1, 1), (0, 0)):
        eng.option("bwd_chain", bc)
        out = []
        for th in c.thetas:
            lp, g = eng.logp_grad(torch.tensor(th, device=cuda_device)[None])
            out.append((lp.cpu(), g.cpu()))
        assert eng.get_option("bwd_chain") == (3 if bc else 0)
        res[(fs, bc)] = out
    for key in ((0, 0),):
        for (la, ga), (lb, gb) in zip(res[(1, 1)], res[key]):
            assert torch.equal(la, lb) and torch.equal(ga, gb), key
    sub = c.g["grad_subsample"]
    for t, (lp, g) in enumerate(res[(1, 1)]):
        check_logp(float(lp[0]), float(c.g[f"logp{t}"]), f"{name} theta{t}")
        check_grad_sub(g[0].numpy(), sub, c.g[f"grad{t}_sub"], float(c.g[f"grad{t}_norm"]), f"{name} theta{t}")


def test_bf16x6_paths_match_fp32_mfma_paths(cuda_device):
    """Burgers shape, 16 perturbed chains: the bf16x6 forward, contraction and layer backward (exact 3-way
    bf16 split, six products, fp32 accumulation) against the fp32-MFMA kernels on the same inputs. Both are fp32-level
    computations, so they agree far inside the golden tolerance: logp to 2e-6 relative, the gradient to
    2e-5 of its norm (measured r01: see the printed values)."""
    c = deeponet_case("deeponet_burgers")
    rng = np.random.default_rng(5)
    C = 16
    base = c.thetas[0]
    th = torch.tensor(np.stack([base + 0.01 * rng.standard_normal(base.size).astype(np.float32) for _ in range(C)]),
                      device=cuda_device)
    eng = engine_for(c, max_chains=C)
    res = {}
    for on in (0, 1):
        for key in ("fwd_bf16x6", "contract_bf16x6", "bwd_bf16x6"):
            eng.option(key, on)
        lp, g = eng.logp_grad(th)
        res[on] = (lp.double().cpu().numpy(), g.double().cpu().numpy())
    dlp = np.abs(res[1][0] - res[0][0]) / np.abs(res[0][0])
    dg = np.linalg.norm(res[1][1] - res[0][1], axis=1) / np.linalg.norm(res[0][1], axis=1)
    print(f"bf16x6 vs fp32 MFMA: logp rel max {dlp.max():.2e}, grad rel-norm max {dg.max():.2e}")
    parity.check("logp_rel", dlp.max(), "bf16x6 vs fp32-MFMA forms, 16 chains")
    parity.check("grad_relnorm", dg.max(), "bf16x6 vs fp32-MFMA forms, 16 chains")


def test_forward_without_weight_images_matches(cuda_device):
    """Plan option fwd_wimg = 0: the hidden layers run the fp32-MFMA fused forward (the bf16x6 one needs the
    pre-split images for its f32 k tail) -- same evaluation to fp32-level agreement."""
    c = deeponet_case("deeponet_burgers")
    rng = np.random.default_rng(11)
    C = 4
    base = c.thetas[0]
    th = torch.tensor(np.stack([base + 0.01 * rng.standard_normal(base.size).astype(np.float32) for _ in range(C)]),
                      device=cuda_device)
    res = []
    for on in (1, 0):
        eng = engine_for(c, max_chains=C)
        eng.option("fwd_wimg", on)
        lp, g = eng.logp_grad(th)
        res.append((lp.double().cpu().numpy(), g.double().cpu().numpy()))
        eng.close()
    dlp = np.abs(res[1][0] - res[0][0]) / np.abs(res[0][0])
    dg = np.linalg.norm(res[1][1] - res[0][1], axis=1) / np.linalg.norm(res[0][1], axis=1)
    parity.check("logp_rel", dlp.max(), "fwd_wimg 0 vs 1")
    parity.check("grad_relnorm", dg.max(), "fwd_wimg 0 vs 1")


@pytest.mark.parametrize("C", [1, 16])
def test_input_layer_in_forward_launch_bitwise(C, cuda_device):
    """Plan option fwd_in0 (default 1): the input layers of both nets run inside the bf16x6 forward's launch
    (FusedNet::x) == the separate row-dot launch (fwd_in0 = 0), bit for bit: log-prob, gradient (both contraction
    forms: a gradient-only call runs the Gram form from 4 chains) and the activations the backward reads."""
    c = deeponet_case("deeponet_burgers")
    rng = np.random.default_rng(12)
    base = c.thetas[0]
    seq = [torch.tensor(np.stack([base + 0.01 * rng.standard_normal(base.size).astype(np.float32) for _ in range(C)]),
                        device=cuda_device) for _ in range(2)]
    res = []
    for on in (1, 0):
        eng = engine_for(c, max_chains=C)
        eng.option("fwd_in0", on)
        assert eng.get_option("fwd_in0") == on
        out = []
        for th in seq:
            lp, g = eng.logp_grad(th)
            out += [lp.cpu(), g.cpu(), torch.from_numpy(eng.debug_buffer("act_b").copy()),
                    torch.from_numpy(eng.debug_buffer("act_t").copy())]
            out.append(eng.grad(th).cpu())
        res.append(out)
        eng.close()
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_weight_images_kept_by_scatter_bitwise(cuda_device):
    """Weight images split once per plan and kept current by the scatter (default) == split from the packed weights
    every evaluation (plan option img_scatter = 0), bit for bit, over a sequence of different thetas per chain and across a
    single-chain sensitivity call (which scatters chain 0 too)."""
    c = deeponet_case("deeponet_burgers")
    rng = np.random.default_rng(5)
    C = 3
    base = c.thetas[0]
    seq = [torch.tensor(np.stack([base + 0.01 * rng.standard_normal(base.size).astype(np.float32) for _ in range(C)]),
                        device=cuda_device) for _ in range(3)]
    res = []
    for on in (1, 0):
        eng = engine_for(c, max_chains=C)
        eng.option("img_scatter", on)
        assert eng.get_option("img_scatter") == on
        out = []
        for i, th in enumerate(seq):
            if i == 1:
                N, P = np.asarray(c.prob.y).shape[-2:]
                eng.sensitivity(th[2], pts=np.random.default_rng(1).integers(0, P, (N, 4)).astype(np.int32))
            lp, g = eng.logp_grad(th)
            out.append((lp.cpu(), g.cpu()))
        res.append(out)
        eng.close()
    for (la, ga), (lb, gb) in zip(*res):
        assert torch.equal(la, lb) and torch.equal(ga, gb)


@pytest.mark.parametrize("name", ["deeponet_small", "deeponet_odd_full"])
def test_deeponet_engine_vs_fp64_oracle_many_chains(name, cuda_device):
    """C chains with independent thetas in one launch == each chain against the fp64 oracle."""
    c = deeponet_case(name)
    rng = np.random.default_rng(42)
    C = 7
    base = c.thetas[0]
    thetas = np.stack([base + 0.03 * rng.standard_normal(base.size).astype(np.float32) for _ in range(C)])
    eng = engine_for(c, max_chains=C)
    lp, g = eng.logp_grad(torch.tensor(thetas, device=cuda_device))
    lay = deeponet_layout(c.spec.in_branch, c.spec.width_branch, c.spec.depth_branch, c.spec.in_trunk,
                          c.spec.width_trunk, c.spec.depth_trunk, c.spec.out)
    p = c.prob
    for i in range(C):
        rl, rg, _ = np_logp_grad(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, thetas[i], c.prior_mu,
                                 c.prior_sd, c.loss, c.tau_out, full=c.full)
        check_logp(float(lp[i]), rl, f"{name} chain {i} vs fp64 oracle")
        check_grad(g[i].cpu().numpy(), rg, f"{name} chain {i} vs fp64 oracle")
    # a smaller C on the same plan only touches the first C chains and agrees bit for bit
    lp2, g2 = eng.logp_grad(torch.tensor(thetas[:3], device=cuda_device))
    assert torch.equal(lp2, lp[:3]) and torch.equal(g2, g[:3])


def test_deeponet_engine_deterministic(cuda_device):
    c = deeponet_case("deeponet_refshape")
    eng = engine_for(c, max_chains=2)
    th = torch.tensor(np.stack(c.thetas), device=cuda_device)
    a = eng.logp_grad(th)
    b = eng.logp_grad(th)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert torch.equal(eng.logp(th), a[0])


@pytest.mark.parametrize("kind", ["deeponet", "bnn"])
def test_graph_replay_bitwise_equal_to_direct_launches(kind, cuda_device):
    """vihmc_graph_enable: the captured-graph evaluation (plan-owned buffers, copy in / out) returns
    exactly the direct-launch results, for every chain count it has captured, and across replays."""
    if kind == "deeponet":
        c = deeponet_case("deeponet_refshape")
        eng = engine_for(c, max_chains=4)
    else:
        from vihmc.engine import MLPEngine
        c = bnn_case("bnn_vi_hmc")
        eng = MLPEngine(c.spec, c.data["x_train"], c.data["y_train"], c.g["mu"], c.idx, c.prior_mu, c.prior_sd,
                        c.loss, c.tau_out, max_chains=4, device=cuda_device)
    base = torch.tensor(np.stack(c.thetas), device=cuda_device)
    for C in (1, 2, 4):
        th = base[torch.arange(C, device=cuda_device) % base.shape[0]].clone()
        th[1:] += 1e-3 * torch.arange(1, C, device=cuda_device, dtype=th.dtype)[:, None]
        eng.graph(False)
        ref = eng.logp_grad(th)
        eng.graph(True)
        for _ in range(2):
            got = eng.logp_grad(th)
            assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    eng.graph(False)


def test_deeponet_split_shards_engine(cuda_device):
    from vihmc.engine import DeepONetEngine, trunk_features
    g = load("deeponet_split")
    spec = spec_of(g)
    th = torch.tensor(g["theta"], device=cuda_device)[None]
    for m in range(2):
        sl = slice(4 * m, 4 * (m + 1))
        eng = DeepONetEngine(spec, g["branch_in"][sl], trunk_features(g["trunk_in"]), g["y"][sl], g["theta"],
                             np.arange(spec.n_params), 0.0, float(np.sqrt(g["prior_var"])), str(g["loss"]),
                             float(g["tau_out"]), prior_scale=2.0, device=cuda_device)
        lp, gr = eng.logp_grad(th)
        check_logp(float(lp[0]), float(g[f"logp_shard{m}"]), f"shard {m}")
        check_grad(gr[0].cpu().numpy(), g[f"grad_shard{m}"], f"shard {m}")


def test_deeponet_nonfinite_is_not_an_error(cuda_device):
    c = deeponet_case("deeponet_small")
    eng = engine_for(c, max_chains=2)
    th = np.stack(c.thetas)
    th[1, 3] = np.nan
    lp, g = eng.logp_grad(torch.tensor(th, device=cuda_device))
    lp = lp.cpu().numpy()
    check_logp(float(lp[0]), float(c.g["logp0"]))
    assert not np.isfinite(lp[1])


def test_plan_option_rejects_unknown_key(cuda_device):
    c = deeponet_case("deeponet_small")
    eng = engine_for(c, max_chains=1)
    with pytest.raises(RuntimeError, match="unknown plan option"):
        eng.option("no_such_option", 1)


def test_engine_rejects_bad_shapes(cuda_device):
    c = deeponet_case("deeponet_small")
    eng = engine_for(c, max_chains=2)
    with pytest.raises(ValueError):
        eng.logp_grad(torch.zeros(3, eng.K, device=cuda_device))
    with pytest.raises(ValueError):
        eng.logp_grad(torch.zeros(1, eng.K + 1, device=cuda_device))


@pytest.mark.parametrize("name", BNN_CASES)
def test_bnn_engine_matches_golden(name, cuda_device):
    from vihmc.engine import MLPEngine
    c = bnn_case(name)
    g = c.g
    eng = MLPEngine(c.spec, c.data["x_train"], c.data["y_train"], g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                    c.tau_out, max_chains=2, device=cuda_device)
    th = torch.tensor(np.stack(c.thetas), device=cuda_device)
    lp, gr = eng.logp_grad(th)
    for t in range(2):
        check_logp(float(lp[t]), float(g[f"logp{t}"]), f"{name} theta{t}")
        check_grad(gr[t].cpu().numpy(), g[f"grad{t}"], f"{name} theta{t}")
    val = MLPEngine(c.spec, c.data["x_val"], c.data["y_val"], g["mu"], c.idx, c.prior_mu, c.prior_sd, c.loss,
                    c.tau_out, max_chains=2, device=cuda_device)
    lpv, pred = val.forward(th)
    for t in range(2):
        check_logp(float(lpv[t]), float(g[f"val_logp{t}"]), f"{name} validation theta{t}")
        check_pred(pred[t].cpu().numpy(), g[f"val_pred{t}"], f"{name} validation theta{t}")


def test_split_shards_small_rows_on_concurrent_streams(cuda_device):
    """Round-1 record (profiles/README.md): a variant that built side B's pre-split trunk image on a second
    stream faulted in the N = 4-per-shard split test. The shipped kernels take the caller's stream; here the
    two shard engines (N = 4 rows: below one 32-row chunk and one 256-row side-B owner tile) run on two torch
    streams at once, interleaved over many evaluations, and every result must equal the single-stream one
    bit for bit -- no fault, no cross-talk between plans on concurrent streams."""
    from vihmc.engine import DeepONetEngine, trunk_features
    g = load("deeponet_split")
    spec = spec_of(g)
    th = torch.tensor(g["theta"], device=cuda_device)[None].repeat(3, 1)
    th[1:] += 1e-3 * torch.arange(1, 3, device=cuda_device, dtype=th.dtype)[:, None]
    engs = [DeepONetEngine(spec, g["branch_in"][4 * m:4 * m + 4], trunk_features(g["trunk_in"]), g["y"][4 * m:4 * m + 4],
                           g["theta"], np.arange(spec.n_params), 0.0, float(np.sqrt(g["prior_var"])), str(g["loss"]),
                           float(g["tau_out"]), prior_scale=2.0, max_chains=3, device=cuda_device) for m in range(2)]
    ref = [e.logp_grad(th) for e in engs]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=cuda_device) for _ in range(2)]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    outs = [[], []]
    for _ in range(20):
        for m in range(2):
            with torch.cuda.stream(streams[m]):
                outs[m].append(engs[m].logp_grad(th))
    torch.cuda.synchronize()
    for m in range(2):
        for lp, gr in outs[m]:
            assert torch.equal(lp, ref[m][0]) and torch.equal(gr, ref[m][1])
        check_logp(float(ref[m][0][0]), float(g[f"logp_shard{m}"]))
