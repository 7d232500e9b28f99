#!/usr/bin/env python3
"""DeepONet VI-HMC benchmark on MI355X: leapfrog-steps/s (+ grad-evals/s, optional ESS/s).

Workload (BASELINE.json config 5, per-GPU share): Burgers-shaped synthetic data (N=1000 functions,
P=10,201 space-time points, branch 101->100x8->100, trunk 5->100x8->100, D=172,401), K=17,240
sensitive parameters, L=7, eps=1e-4, 16 independent chains per GPU (weak scaling: 128 chains on 8
GPUs), log-posterior + gradient on the HIP engine. One bench "step" = one HMC iteration of every
local chain (momentum draw, L leapfrog steps, Metropolis accept), all device-resident.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Prints one JSON line on rank 0 (contract in the task statement / DESIGN.md §Measurement).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vi-hmc_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "leapfrog-steps/sec/GPU (grad evals/sec) + ESS/sec, DeepONet VI-HMC"
FP32_PEAK_TFLOPS = 157.3        # MI355X_MICROARCH.md: dense fp32 (vector = MFMA rate)
BF16_PEAK_TFLOPS = 2516.6       # MI355X_MICROARCH.md "~2.5 PF dense": 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz
BF16X6_PRODUCTS = 6             # fp32 operand = 3 exact bf16 planes; the 6 products of order <= 2 are kept
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 240 HMC iterations at ~9 ms: a timed region of >= 2 s (MI355X_MICROARCH.md DVFS item 6: the clock under load
    # settles over seconds; a 0.18-s region was shorter than the box spread it was meant to resolve)
    ap.add_argument("--steps", type=int, default=240)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--chains-per-gpu", type=int, default=16)
    ap.add_argument("--L", type=int, default=7)
    ap.add_argument("--step-size", type=float, default=1e-4)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--ess-steps", type=int, default=100,
                    help="HMC iterations of a separately timed phase after the timed region whose samples give "
                         "ESS/s (Geyer initial monotone sequence; 0 = skip)")
    ap.add_argument("--no-gather", dest="gather", action="store_false",
                    help="skip the RCCL all-gather of the sample pool after the timed region (N > 1)")
    ap.add_argument("--cpu-procs", type=int, default=14,
                    help="one-thread CPU processes of the multi-chain CPU throughput baseline (0 = skip); the GPU "
                         "box's CPU share is 16 cores, and a ROCm torch import counts against its limit of 16 "
                         "processes per GPU (this one included)")
    ap.add_argument("--no-side-legs", dest="side_legs", action="store_false",
                    help="skip the single-chain (configs 2 and 4) and BNN (configs 2-3) legs reported beside the line")
    return ap.parse_args()


def cpu_baseline(prob, L, step_size, seconds):
    """The reference's log-prob (oracle restatement with the reference's torch ops, fp32 CPU) inside the
    scalar hamiltorch loop, 1 chain, all host threads, bounded to ~`seconds` of work."""
    sys.path.insert(0, ROOT)
    from oracle.deeponet_ref import TorchDeepONetRef, deeponet_layout
    from oracle import hamiltorch_ref as HR
    ref = TorchDeepONetRef(deeponet_layout(), prob.branch_in, prob.trunk_in, prob.y, prob.mu, prob.grad_ind, 0.0, 0.1,
                           "NLL", 1.0)
    th = torch.tensor(prob.mu[prob.grad_ind])
    g = torch.Generator().manual_seed(0)
    n = 0
    t0 = time.perf_counter()
    while True:
        out = HR.sample(ref.log_prob, th, 1, L, step_size, generator=g)
        th = out[-1]
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), cpu)
    except OSError:
        pass
    return {"value": L * n / dt, "unit": "leapfrog-steps/s", "cores": torch.get_num_threads(), "kind": "port",
            "cpu_model": cpu,
            "sample": f"1 chain x {n} HMC samples (L={L}; hamiltorch: L+1 grad + 2 value evals each) in {dt:.1f} s, "
                      f"oracle/deeponet_ref.TorchDeepONetRef (reference torch ops) + oracle/hamiltorch_ref.sample, "
                      f"torch {torch.__version__} CPU, {torch.get_num_threads()} threads"}


def cpu_baseline_bnn(seconds, L=196, eps=5e-4):
    """BNN VI-HMC (configs 2-3) on the CPU: the reference closure's torch ops (oracle/bnn_ref.TorchBNNRef: width
    [10, 10] tanh, 20 shipped points, NLL variance 0.0025, prior N(0, 1) per tensor) in the scalar hamiltorch loop,
    the same K = 90 sampled indices as leg_bnn, 1 chain, 1 thread (the tiny ops run fastest on one thread: SURVEY
    §6), bounded to ~`seconds`."""
    sys.path.insert(0, ROOT)
    from oracle import hamiltorch_ref as HR
    from oracle.bnn_ref import TorchBNNRef, mlp_layout
    from vihmc.data import bnn_data, bnn_init
    from vihmc.layout import MLPSpec
    spec = MLPSpec()
    x, y, _, _ = bnn_data()
    mu = bnn_init(spec, seed=0)
    idx = np.sort(np.random.default_rng(11).choice(spec.n_params, 90, replace=False))
    ref = TorchBNNRef(mlp_layout(), x, y, mu, idx, prior_list=[1.0] * 6, loss="NLL", tau_out=0.0025)
    th = torch.tensor(mu[idx])
    g = torch.Generator().manual_seed(0)
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    n = 0
    t0 = time.perf_counter()
    try:
        while True:
            th = HR.sample(ref.log_prob, th, 1, L, eps, generator=g)[-1]
            n += 1
            if time.perf_counter() - t0 >= seconds:
                break
    finally:
        torch.set_num_threads(nt)
    dt = time.perf_counter() - t0
    return {"value": L * n / dt, "unit": "leapfrog-steps/s (1 chain)", "cores": 1, "kind": "port",
            "sample": f"1 chain x {n} HMC samples (L={L}, eps={eps}; hamiltorch: L+1 grad + 2 value evals each) in "
                      f"{dt:.1f} s, oracle/bnn_ref.TorchBNNRef (the reference's torch ops) + "
                      f"oracle/hamiltorch_ref.sample, torch {torch.__version__} CPU, 1 thread"}


def cpu_throughput(procs, seconds, L, step_size):
    """One process per core at one thread, one chain each: oracle/cpu_throughput.py."""
    sys.path.insert(0, ROOT)
    from oracle.cpu_throughput import run_parallel
    r = run_parallel(procs, seconds, L, step_size)
    return {"value": r["value"], "unit": "leapfrog-steps/s", "cores": procs, "kind": "port",
            "sample": f"{procs} processes x 1 thread x 1 chain, {r['samples']} HMC samples in <= {r['seconds_max']:.1f} s "
                      f"(L={L}, hamiltorch loop + the reference torch ops, oracle/cpu_throughput.py)"}


# ------------------------------------------------------------------------------------------------
# kernel classes (include/vihmc.h VIHMC_T_*) priced on the roofline
# ------------------------------------------------------------------------------------------------
KCLASS = {0: ("contract_a", "k_contract_bf", "side-A contraction: S = Z_b Z_t^T + b, Gaussian NLL, G, dZ_trunk"),
          1: ("contract_b", "k_contract_bf_b", "side-B contraction: dZ_branch = G Z_trunk"),
          2: ("bwd", "k_bwd_bf2", "layer backward (dX and dW of both MLPs), one launch per layer"),
          3: ("fwd", "k_fwd_fused_bf", "fused forward of both MLPs (layers 1..8; with plan option fwd_in0 also the "
                                       "input layers, on the f32 MFMA)"),
          6: ("gram", "k_gram_a + k_gram_b",
              "Gram-form gradient-only contraction of the inner leapfrog steps: y Zt^, y^T Zb^, Gram terms, dZ "
              "epilogues (one HIP-event pair around both launches)")}
T_EVAL = 4
CAL_STEPS = 2          # untimed HMC iterations with every kernel class under HIP events


def mfma_peak(bf16x6: int) -> float:
    # bf16x6: each fp32 product costs 6 bf16 MFMA products, so the fp32-equivalent ceiling is the bf16 dense peak
    # / 6 (= 419.4 TFLOP/s); the fp32 MFMA form is priced against the fp32 peak
    return BF16_PEAK_TFLOPS / BF16X6_PRODUCTS if bf16x6 else FP32_PEAK_TFLOPS


def class_flops(eng, spec, prob):
    """Algorithmic FLOP per chain of each timing class (the input layers count with the forward when its launch runs
    them: plan option fwd_in0)."""
    fl = spec.flops_by_kernel(prob.N, prob.P)
    fl["gram"] = spec.flops_gram(prob.N, prob.P, centred=bool(eng.get_option("gram_center")))
    if eng.get_option("fwd_in0"):
        fl["fwd"] += fl["input"]
    return fl


def class_table(eng, spec, prob, C, evals):
    """Per-class HIP-event times recorded over `evals` evaluations -> per-launch roofline numbers."""
    fl = class_flops(eng, spec, prob)
    forms = {"contract_a": eng.get_option("contract_bf16x6"), "contract_b": eng.get_option("contract_bf16x6"),
             "bwd": eng.get_option("bwd_bf16x6"), "fwd": eng.get_option("fwd_bf16x6"), "gram": 1}
    ev_ms, ev_n = eng.timing_class(T_EVAL)
    eval_ms = ev_ms / max(ev_n, 1)
    out = {}
    for cls, (key, kname, what) in KCLASS.items():
        ms, n = eng.timing_class(cls)
        if n == 0:
            continue
        per_eval = n / evals
        # per launch: classes that do not run in every evaluation (side A / B on the end points only, the Gram form
        # on the inner steps) launch once in the evaluations that run them
        flops = C * fl[key] / max(per_eval, 1.0)
        avg = ms / n
        ach = flops / (avg / 1e3) / 1e12
        pk = mfma_peak(forms[key])
        out[key] = {"kernel": kname, "what": what, "avg_launch_ms": avg, "launches_per_eval": per_eval,
                    "flops_per_launch": flops, "achieved": ach, "peak": pk, "frac": ach / pk,
                    "share_of_eval": ms / max(ev_ms, 1e-12)}
    total = C * spec.flops_per_grad_eval(prob.N, prob.P)
    ach = total / (eval_ms / 1e3) / 1e12
    out["eval"] = {"kernel": "whole evaluation (all launches, scatter -> gather)", "avg_ms": eval_ms,
                   "flops": total, "achieved": ach, "peak": mfma_peak(1), "frac": ach / mfma_peak(1)}
    return out


def load_traffic(kname, C):
    """PMC-measured HBM bytes per launch of `kname` at this chain count (profiles/traffic.json, written by
    profiles/traffic_from_pmc.py from separate FETCH_SIZE / WRITE_SIZE passes of this bench), or None."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        tj = json.load(f)
    if tj.get("chains_per_gpu") != C:
        return None, None
    total = 0.0
    for kn in kname.split(" + "):                      # a class of several kernels: the sum over its launches
        k = tj.get("kernels", {}).get(kn.split(" ")[0])
        if k is None:
            return None, None
        total += k["hbm_bytes_per_launch"]
    return total, tj.get("source")


EV_STEPS = 3            # one-chain legs: HMC iterations with HIP-event timing after the timed ones
DOM_EVERY = 4           # the main timed region: the dominant class's HIP events on every 4th evaluation


def _timed_steps(runner, warm, steps):
    for _ in range(warm):
        runner.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        runner.step()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def leg_deeponet_c1(prob, spec, dev, L, eps, steps=20):
    """The VI-HMC DeepONet config at ONE chain per GPU (single-chain latency)."""
    from vihmc.engine import DeepONetEngine, trunk_features
    from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner
    eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0,
                         0.1, "NLL", 1.0, max_chains=1, device=dev)
    ev = EngineEvaluator(eng)
    th0 = torch.tensor(prob.mu[prob.grad_ind], device=dev)[None]
    r = HMCRunner(ev, th0, steps + 3 + EV_STEPS, L, eps, rng=ChainRNG(1, eng.K, dev, seeds=[1000]))
    dt = _timed_steps(r, 3, steps)
    # the evaluation time from HIP events over a few further steps: at one chain the event records' idle gaps (~12 us
    # per evaluation) are a measurable share, so they stay out of the throughput's timed steps
    eng.timing(T_EVAL, True)
    _timed_steps(r, 0, EV_STEPS)
    ms, n = eng.timing_class(T_EVAL)
    ev_ms = ms / max(n, 1)
    fl = spec.flops_per_grad_eval(prob.N, prob.P)
    eng.timing(-1, False)
    eng.close()
    return {"workload": "DeepONet VI-HMC Burgers (config 5 network / data), 1 chain per GPU", "chains": 1,
            "leapfrog_steps_per_s": steps * L / dt, "ms_per_eval": ev_ms, "ms_per_hmc_step": dt / steps * 1e3,
            "eval_tflops_algorithmic": fl / (ev_ms / 1e3) / 1e12, "frac_of_bf16x6_ceiling": fl / (ev_ms / 1e3) / 1e12 /
            mfma_peak(1)}


def leg_good_fit(spec, dev, L, eps, C=16, steps=20):
    """The posterior the reference actually samples: frozen weights at a network that fits the data
    to the noise -- deeponet_problem(noise=1e-3, mu_noise=0), sum r^2 / sum y^2 ~ 1.5e-3 at mu, the reference's
    trained VI mean (main_VI_HMC_burgers.py:63-65,278-283) -- 16 chains started at mu, the bench's L / eps. Reports the
    throughput and which contraction form the inner steps ran (the centred Gram form's fit guard compares sum r^2 with
    sum y~^2, y~ = y - the output at mu)."""
    from vihmc.data import deeponet_problem
    from vihmc.engine import DeepONetEngine, trunk_features
    from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner
    prob = deeponet_problem(seed=0, noise=1e-3, mu_noise=0.0)
    eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0,
                         0.1, "NLL", 1.0, max_chains=C, device=dev)
    ev = EngineEvaluator(eng)
    th0 = torch.tensor(prob.mu[prob.grad_ind], device=dev).repeat(C, 1)
    r = HMCRunner(ev, th0, steps + 3, L, eps, rng=ChainRNG(C, eng.K, dev, seeds=[3000 + c for c in range(C)]))
    for _ in range(3):
        r.step()
    eng.option("gram_evals", 0)
    dt = _timed_steps(r, 0, steps)
    n_calls, n_gram = eng.get_option("grad_evals"), eng.get_option("gram_evals")
    n_chain_gram = eng.get_option("gram_chain_evals")
    res = r.result()
    lp = res.logp_trace[:, -1].double()
    y = prob.y.astype(np.float64)
    fit_mu = float(1e-3 ** 2 * y.size / (y ** 2).sum())   # at mu the residual is the data noise (std 1e-3)
    out = {"workload": "DeepONet VI-HMC Burgers at a good fit: deeponet_problem(noise=1e-3, mu_noise=0), frozen "
                       f"weights = the data's generator, {C} chains from mu, L = {L}, eps = {eps}",
           "chains": C, "leapfrog_steps_per_s": C * L * steps / dt, "ms_per_hmc_step": dt / steps * 1e3,
           "gram_eval_fraction": n_gram / max(n_calls, 1),
           "gram_chain_eval_fraction": n_chain_gram / max(n_calls * C, 1),
           "gram_center": eng.get_option("gram_center"), "gram_guard": eng.get_option("gram_guard"),
           "fit_ratio_at_mu_approx": fit_mu,
           "accept_rate": float(res.accepted[:, 3:].float().mean()),
           "final_logp_mean": float(lp.mean())}
    eng.close()
    return out


def sustained_leg(runner, eng, dev, C, L, world, target_s=2.0, ms_per_step=None):
    """when the driver's --steps give a timed region shorter than ~2 s, the same plan's chains
    continue (a fresh runner from their current states, no sample storage) for >= target_s more, with their own
    per-XCD shader clocks; the headline value / steps stay exactly as asked."""
    from vihmc.engine import ShaderClock
    from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner
    from vihmc.dist import max_over_ranks
    n = max(10, int(np.ceil(target_s / max(ms_per_step / 1e3, 1e-4))))
    idx = (runner.counts - 1).clamp(min=0)
    theta = runner.samples[torch.arange(C, device=dev), idx].clone()
    r2 = HMCRunner(EngineEvaluator(eng), theta, n, L, runner.eps_host[0], burn=0, store=False,
                   rng=ChainRNG(C, eng.K, dev, seeds=[5000 + c for c in range(C)]))
    clock = ShaderClock(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    clock.start()
    for _ in range(n):
        r2.step()
    clock.stop()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    T = max_over_ranks(time.perf_counter() - t0, dev)
    clk = clock.summary()
    return {"sustained_leapfrog_steps_per_s": world * C * L * n / T, "sustained_steps": n, "sustained_s": T,
            "sustained_ms_per_step": T / n * 1e3, "sustained_sclk_mhz": clk["mean_mhz"],
            "sustained_sclk_mhz_by_xcd": {str(k): round(v, 1) for k, v in clk["mhz_by_xcd"].items()},
            "sustained_sclk_spread": clk["spread"],
            "sustained_basis": "the timed region was shorter than 2 s: the same chains continued for >= 2 s under the "
                               "same runner settings (timed like the headline: sync + barrier, max over ranks)"}


def leg_split_c1(spec, dev, L, eps, steps=10):
    """Config 4: full-parameter DeepONet HMC, Burgers, 2 data shards of N/2, Integrator.SPLITTING, 1 chain."""
    from vihmc.data import deeponet_problem
    from vihmc.engine import DeepONetEngine, trunk_features
    from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner, Integrator
    prob = deeponet_problem(seed=0, k=None)
    half = prob.N // 2
    tf = trunk_features(prob.trunk_in)
    engs = [DeepONetEngine(spec, prob.branch_in[m * half:(m + 1) * half], tf, prob.y[m * half:(m + 1) * half],
                           prob.mu, prob.grad_ind, 0.0, 0.1, "NLL", 1.0, prior_scale=2.0, max_chains=1, device=dev)
            for m in range(2)]
    evs = [EngineEvaluator(e) for e in engs]
    th0 = torch.tensor(prob.mu, device=dev)[None]
    r = HMCRunner(evs, th0, steps + 2 + EV_STEPS, L, eps, integrator=Integrator.SPLITTING,
                  rng=ChainRNG(1, spec.n_params, dev, seeds=[1000]))
    for _ in range(2):
        r.step()
    for e in evs:
        e.n_grad = e.n_value = 0
    dt = _timed_steps(r, 0, steps)
    n_grad = sum(e.n_grad for e in evs)
    for e in engs:                                   # evaluation times over further steps (see leg_deeponet_c1)
        e.timing(T_EVAL, True)
    _timed_steps(r, 0, EV_STEPS)
    ms = sum(e.timing_class(T_EVAL)[0] for e in engs)
    n = sum(e.timing_class(T_EVAL)[1] for e in engs)
    out = {"workload": "config 4: full-parameter DeepONet HMC (D = 172,401), Burgers, 2 shards of N/2 = 500, "
                       "Integrator.SPLITTING, 1 chain", "chains": 1, "leapfrog_steps_per_s": steps * L / dt,
           "half_shard_grad_evals_per_s": n_grad / dt, "ms_per_half_shard_eval": ms / max(n, 1),
           "ms_per_hmc_step": dt / steps * 1e3,
           "note": "a leapfrog step = 2M = 4 half-shard gradient evaluations (3 with the end-point gradient reused)"}
    for e in engs:
        e.close()
    return out


def leg_bnn(dev, C, steps=10, L=196, eps=5e-4, fast=True):
    """BNN VI-HMC (Neural_network/VI_HMC, configs 2 and 3): width [10, 10] tanh, 20 shipped training points,
    NLL variance 0.0025, prior N(0, 1), K = 90 sensitive parameters of D = 141 (seeded), L = 196, eps = 5e-4."""
    from vihmc.data import bnn_data, bnn_init
    from vihmc.engine import MLPEngine, prior_per_tensor
    from vihmc.layout import MLPSpec
    from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner
    spec = MLPSpec()
    x, y, _, _ = bnn_data()
    mu = bnn_init(spec, seed=0)
    D = spec.n_params
    idx = np.sort(np.random.default_rng(11).choice(D, 90, replace=False))
    K = idx.size
    eng = MLPEngine(spec, x, y, mu, idx, 0.0, prior_per_tensor(spec.tensor_sizes, K, [1.0] * 6), "NLL", 0.0025,
                    max_chains=C, device=dev)
    if not fast:
        eng.option("mlp_fast", 0)                           # the generic LDS kernels (A/B)
    ev = EngineEvaluator(eng)
    th0 = torch.tensor(mu[idx], device=dev)[None].repeat(C, 1)
    r = HMCRunner(ev, th0, steps + 2, L, eps, rng=ChainRNG(C, K, dev, seeds=[1000 + c for c in range(C)]))
    eng.timing(eng.T_MLP, True)
    dt = _timed_steps(r, 2, steps)
    ms, n = eng.timing_class(eng.T_MLP)
    eng.timing(-1, False)
    avg = ms / max(n, 1)                                   # in-kernel ms per leapfrog step (L counted per launch)
    # one k_mlp_traj launch per HMC iteration runs the whole trajectory; algorithmic bytes per launch: theta, p,
    # g in and out per chain, x / y / frozen weights / index map once
    byts = C * 6 * 4 * K + 2 * 4 * x.size + 4 * D + 4 * K
    lf = C * L * steps / dt
    kern = "k_mlp_traj_bnn" if eng.get_option("mlp_fast") else "k_mlp_traj"
    eng.close()
    return {"workload": f"BNN VI-HMC (configs 2-3), {C} chain(s) per GPU, L = {L}", "chains": C,
            "leapfrog_steps_per_s": lf, "us_per_leapfrog_step": 1e6 * dt / (L * steps),
            "kernel_us_per_leapfrog_step": avg * 1e3,
            "kernel_share_of_wall": avg * L * steps / 1e3 / dt,
            "algorithmic_bytes_per_launch": byts,
            "hbm_frac": byts / (avg * L / 1e3) / 1e9 / HBM_PEAK_GBS,
            "kernel": kern,
            "note": "latency-bound: one trajectory launch per HMC iteration (one wave per chain, theta / p / g and the "
                    "per-row activations in registers); the HBM fraction is from algorithmic bytes"}


def ess_phase(args, ev, runner, K, dev, chains, world):
    """ESS/s: continue every chain for `ess_steps` HMC iterations (fresh per-chain seeds 2000 + c), timed
    like the main region (barrier + sync, max over ranks); Geyer ESS of the log-prob trace and of every
    sensitive coordinate over those samples, summed over all chains of the job."""
    from vihmc.diagnostics import ess
    from vihmc.samplers import ChainRNG, HMCRunner
    C = len(chains)
    idx = (runner.counts - 1).clamp(min=0)
    theta = runner.samples[torch.arange(C, device=dev), idx].clone()
    r2 = HMCRunner(ev, theta, args.ess_steps, args.L, args.step_size, burn=0,
                   rng=ChainRNG(C, K, dev, seeds=[2000 + c for c in chains]))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.ess_steps):
        r2.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    res = r2.result()
    n = int(res.counts.min())
    e_lp = ess(res.logp_trace.double()).sum().reshape(1)
    e_coord = ess(res.samples[:, 1:n].double().transpose(1, 2)).sum(0)           # [K], summed over chains
    if world > 1:
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
        dist.all_reduce(e_lp)
        dist.all_reduce(e_coord)
    w = float(wall.item())
    return {"ess_steps": args.ess_steps, "ess_wall_s": w, "ess_logp": float(e_lp.item()),
            "ess_min": float(e_coord.min().item()), "ess_median": float(e_coord.median().item()),
            "ess_logp_per_s": float(e_lp.item()) / w, "ess_min_per_s": float(e_coord.min().item()) / w,
            "ess_median_per_s": float(e_coord.median().item()) / w,
            "ess_note": "whole job; Geyer IMSE over post-timing samples, summed over chains; "
                        "eps=1e-4 trajectories are short, so coordinate ESS is low"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one process per GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from vihmc.data import deeponet_problem
    from vihmc.dist import gather_ragged_pool, max_over_ranks
    from vihmc.engine import DeepONetEngine, ShaderClock, trunk_features
    from vihmc.layout import DeepONetSpec
    from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner

    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    C = args.chains_per_gpu
    eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0,
                         0.1, "NLL", 1.0, max_chains=C, device=dev)
    chains = list(range(rank * C, (rank + 1) * C))
    theta0 = torch.tensor(prob.mu[prob.grad_ind], device=dev).repeat(C, 1)
    ev = EngineEvaluator(eng)
    n_total = args.warmup + CAL_STEPS + args.steps
    runner = HMCRunner(ev, theta0, n_total, args.L, args.step_size, burn=0,
                       rng=ChainRNG(C, eng.K, dev, seeds=[1000 + c for c in chains]))
    for _ in range(args.warmup):
        runner.step()
    torch.cuda.synchronize()
    # calibration (untimed): every kernel class and the whole evaluation under HIP events for a few steps,
    # to find the kernel class with the largest share of the evaluation -- the one the roofline prices
    cal_steps = CAL_STEPS
    eng.timing(-1, True)
    for _ in range(cal_steps):
        runner.step()
    torch.cuda.synchronize()
    cal = class_table(eng, spec, prob, C, cal_steps * args.L)
    eng.timing(-1, False)
    dom_cls = max(KCLASS, key=lambda k: cal.get(KCLASS[k][0], {}).get("share_of_eval", -1.0))
    ev.n_grad = 0
    eng.option("gram_evals", 0)                     # reset the plan's evaluation counters (both forms)
    clock = ShaderClock(dev)
    # the dominant class under HIP events on every DOM_EVERY-th evaluation of the timed region (each event record
    # leaves a few-us idle gap before the next launch: instrumentation, not workload)
    eng.option("timing_every", DOM_EVERY)
    eng.timing(dom_cls, True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    clock.start()
    for _ in range(args.steps):
        runner.step()
    clock.stop()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    k_ms, k_n = eng.timing_class(dom_cls)
    eng.timing(-1, False)
    eng.option("timing_every", 1)
    grad_evals = ev.n_grad
    n_calls, n_gram = eng.get_option("grad_evals"), eng.get_option("gram_evals")
    clk = clock.summary()
    sclk = clk["mhz_by_xcd"]
    T = max_over_ranks(t1 - t0, dev)

    extra = {}
    if args.gather and world > 1:
        # ragged-safe: a chain that hit a LogProbError stores fewer samples, so ranks may differ in length
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        pool, _ = gather_ragged_pool(runner.samples, runner.counts)
        torch.cuda.synchronize()
        extra["allgather_ms"] = (time.perf_counter() - g0) * 1e3
        extra["allgather_bytes"] = pool.numel() * 4
    res = runner.result()
    acc_rate = float(res.accepted[:, args.warmup + cal_steps:].float().mean())
    if T < 2.0:
        extra.update(sustained_leg(runner, eng, dev, C, args.L, world, ms_per_step=T / args.steps * 1e3))
    if args.ess_steps > 0:
        extra.update(ess_phase(args, ev, runner, eng.K, dev, chains, world))
    side = {}
    if world == 1 and args.side_legs:
        side["deeponet_1_chain"] = leg_deeponet_c1(prob, spec, dev, args.L, args.step_size)
        side["deeponet_good_fit_16_chains"] = leg_good_fit(spec, dev, args.L, args.step_size, C=C)
        side["config4_split_1_chain"] = leg_split_c1(spec, dev, args.L, args.step_size)
        side["bnn_config2_1_chain"] = leg_bnn(dev, 1)
        side["bnn_config3_8_chains"] = leg_bnn(dev, 8)

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    leapfrog = world * C * args.L * args.steps
    value = leapfrog / T
    key, kname, what = KCLASS[dom_cls]
    fl = class_flops(eng, spec, prob)
    per_eval = cal[key]["launches_per_eval"]
    flops_launch = C * fl[key] / max(per_eval, 1.0)
    avg_s = (k_ms / max(k_n, 1)) / 1e3
    achieved = flops_launch / avg_s / 1e12 if k_n else None
    evals_per_s = world * grad_evals / T
    gram_frac = n_gram / max(n_calls, 1)
    fl_res = spec.flops_per_grad_eval(prob.N, prob.P)
    fl_gram = fl_res - fl["contract_a"] - fl["contract_b"] + fl["gram"]
    flops_performed = (1.0 - gram_frac) * fl_res + gram_frac * fl_gram
    form_key = {"contract_a": "contract_bf16x6", "contract_b": "contract_bf16x6", "bwd": "bwd_bf16x6",
                "fwd": "fwd_bf16x6", "gram": "contract_bf16x6"}[key]
    bf = eng.get_option(form_key)
    peak = mfma_peak(bf)
    traffic, tsrc = load_traffic(kname, C)
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "leapfrog-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": T / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "mfma_form": {k: eng.get_option(k) for k in ("fwd_bf16x6", "contract_bf16x6", "bwd_bf16x6")},
        "data": "synthetic (Burgers shapes, seeded teacher DeepONet; the .mat is not shipped)",
        "config": {"workload": "DeepONet VI-HMC Burgers, config 5 per-GPU share", "N": prob.N, "P": prob.P,
                   "D": spec.n_params, "K": prob.K, "chains_per_gpu": C, "global_chains": world * C, "L": args.L,
                   "step_size": args.step_size, "parallelism": f"chain-sharded x{world}, no data-path collective"},
        "grad_evals_per_s": evals_per_s,
        "hamiltorch_equiv_grad_evals_per_s": world * C * (args.L + 1) * args.steps / T,
        "eval_tflops_algorithmic": evals_per_s * spec.flops_per_grad_eval(prob.N, prob.P) / 1e12,
        "eval_flops_basis": "the reference's residual-form FLOPs per gradient evaluation (the inner leapfrog steps run the "
                            "Gram form, which does fewer: layout.flops_gram)",
        "eval_tflops_performed": evals_per_s * flops_performed / 1e12,
        "eval_flops_performed_basis": "FLOPs of the forms that ran: residual-form evaluations at "
                                      "flops_per_grad_eval, Gram-form evaluations with the contraction at flops_gram",
        "gram_eval_fraction": gram_frac,
        "gram_eval_fraction_basis": f"{n_gram} of {n_calls} gradient-evaluation calls in the timed region ran the "
                                    "Gram form (plan counters grad_evals / gram_evals)",
        "timed_region_s": T,
        "sclk_mhz": clk["mean_mhz"],
        "sclk_mhz_by_xcd": {str(k): round(v, 1) for k, v in sclk.items()},
        "sclk_spread": clk["spread"],
        "sclk_cus_per_xcd": {str(k): v for k, v in clk["cus_per_xcd"].items()},
        "sclk_rejected_above_2400": clk["rejected_above_max"],
        "sclk_basis": "average shader clock over the timed region per CU from that CU's own two stamps: d s_memtime / "
                      "d s_memrealtime x 100 MHz (vihmc_clock_stamp before and after the region, 256 one-wave "
                      "workgroups paired by XCD / CU; MI355X_MICROARCH.md DVFS item 6); per XCD the median over its "
                      "CUs; readings above the 2,400-MHz maximum rejected and listed; spread = (max - min) / mean "
                      "over the XCD medians",
        "roofline_frac_at_sclk": ((achieved / (peak * clk["mean_mhz"] / 2400.0))
                                  if (achieved and clk["mean_mhz"] and clk["spread"] is not None
                                      and clk["spread"] <= 0.10) else None),
        "roofline_frac_at_sclk_basis": "the roofline fraction against the peak scaled to the measured clock; reported "
                                       "only when the per-XCD spread is <= 10 %",
        "accept_rate": acc_rate,
        "roofline": {"kernel": f"{kname}: {what}", "selected_as": "largest share of the evaluation's GPU time "
                     f"({cal[key]['share_of_eval']:.3f}, HIP-event calibration before the timed region)",
                     "bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "frac": (achieved / peak) if achieved else None, "traffic": traffic,
                     "peak_basis": ("fp32-equivalent: bf16 dense MFMA peak 2516.6 / 6 bf16 products per fp32 product"
                                    if bf else "fp32 MFMA dense peak"),
                     "achieved_vs_fp32_mfma_peak": (achieved / FP32_PEAK_TFLOPS) if achieved else None,
                     "traffic_unit": "HBM bytes/launch (PMC FETCH_SIZE x2 + WRITE_SIZE, separate rocprofv3 passes; "
                                     f"profiles/traffic.json: {tsrc})",
                     "avg_launch_ms": avg_s * 1e3, "launches": k_n, "launches_per_eval": per_eval,
                     "flops_per_launch": flops_launch},
        "roofline_all": cal,
    }
    line.update(extra)
    if side:
        line["side_legs"] = side
    if world == 1 and args.cpu_seconds > 0 and "bnn_config2_1_chain" in side:
        bc = cpu_baseline_bnn(min(args.cpu_seconds, 10.0))
        side["bnn_cpu_baseline"] = bc
        side["bnn_config2_1_chain"]["speedup_vs_cpu"] = side["bnn_config2_1_chain"]["leapfrog_steps_per_s"] / bc["value"]
        side["bnn_config3_8_chains"]["speedup_per_chain_vs_cpu"] = \
            side["bnn_config3_8_chains"]["leapfrog_steps_per_s"] / 8 / bc["value"]
    if world == 1 and args.cpu_seconds > 0:
        cb = cpu_baseline(prob, args.L, args.step_size, args.cpu_seconds)
        line["cpu_baseline"] = cb
        line["speedup_vs_cpu"] = value / cb["value"]
        line["speedup_per_chain_vs_cpu"] = value / C / cb["value"]
        if args.cpu_procs > 0:
            mp = cpu_throughput(args.cpu_procs, args.cpu_seconds, args.L, args.step_size)
            line["cpu_baseline_throughput"] = mp
            line["speedup_vs_cpu_throughput"] = value / mp["value"]
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
