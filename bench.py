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
    ap.add_argument("--steps", type=int, default=20)
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
    from vihmc.engine import DeepONetEngine, trunk_features
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
    n_total = args.warmup + args.steps
    runner = HMCRunner(ev, theta0, n_total, args.L, args.step_size, burn=0,
                       rng=ChainRNG(C, eng.K, dev, seeds=[1000 + c for c in chains]))
    for _ in range(args.warmup):
        runner.step()
    torch.cuda.synchronize()
    ev.n_grad = 0
    eng.timing(0, True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    k_ms, k_n = eng.timing_read()
    eng.timing(0, False)
    grad_evals = ev.n_grad
    T = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(T, op=dist.ReduceOp.MAX)
    T = float(T.item())

    extra = {}
    if args.gather and world > 1:
        local_pool = runner.samples[:, :int(runner.counts.min())].contiguous()
        pool = torch.empty((world,) + tuple(local_pool.shape), device=dev)
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        dist.all_gather_into_tensor(pool, local_pool)
        torch.cuda.synchronize()
        extra["allgather_ms"] = (time.perf_counter() - g0) * 1e3
        extra["allgather_bytes"] = pool.numel() * 4
    res = runner.result()
    acc_rate = float(res.accepted[:, args.warmup:].float().mean())
    if args.ess_steps > 0:
        extra.update(ess_phase(args, ev, runner, eng.K, dev, chains, world))

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    leapfrog = world * C * args.L * args.steps
    value = leapfrog / T
    flops_contract = C * 4.0 * prob.N * prob.P * spec.out            # S + dZ_trunk, algorithmic, per launch
    avg_s = (k_ms / max(k_n, 1)) / 1e3
    achieved = flops_contract / avg_s / 1e12 if k_n else None
    evals_per_s = world * grad_evals / T
    bf = eng.get_option("contract_bf16x6")
    # bf16x6: each fp32 product costs 6 bf16 MFMA products, so the fp32-equivalent ceiling of the kernel is
    # the bf16 dense peak / 6 (= 419.4 TFLOP/s); the fp32 MFMA path is priced against the fp32 peak
    peak = BF16_PEAK_TFLOPS / BF16X6_PRODUCTS if bf else FP32_PEAK_TFLOPS
    kname = ("k_contract_bf: side-A contraction on the bf16 MFMA, bf16x6 fp32 emulation" if bf else
             "k_contract_ws: side-A contraction on the fp32 MFMA")
    traffic = None
    tpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "traffic_contract.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
        if tj.get("chains_per_gpu") == C and tj.get("contract_bf16x6", 0) == bf:
            traffic = tj["hbm_bytes_per_launch"]     # PMC-measured bytes per side-A launch (same config)
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
        "accept_rate": acc_rate,
        "roofline": {"kernel": kname + " (branch x trunk S, Gaussian NLL, G, dZ_trunk)",
                     "bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "frac": (achieved / peak) if achieved else None, "traffic": traffic,
                     "peak_basis": ("fp32-equivalent: bf16 dense MFMA peak 2516.6 / 6 bf16 products per fp32 product"
                                    if bf else "fp32 MFMA dense peak"),
                     "achieved_vs_fp32_mfma_peak": (achieved / FP32_PEAK_TFLOPS) if achieved else None,
                     "traffic_unit": "bytes/launch (HBM, PMC FETCH_SIZE x2 + WRITE_SIZE; profiles/traffic_contract.json)",
                     "avg_launch_ms": avg_s * 1e3, "launches": k_n,
                     "flops_per_launch": flops_contract},
    }
    line.update(extra)
    if world == 1 and args.cpu_seconds > 0:
        line["cpu_baseline"] = cpu_baseline(prob, args.L, args.step_size, args.cpu_seconds)
        line["speedup_vs_cpu"] = value / line["cpu_baseline"]["value"]
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
