"""Probe: 16 chains per GPU as G independent chain groups (one plan + one HMCRunner per group), each group on its own
HIP stream, stepped round-robin, so one group's kernels fill the launch tails and gaps of the other's. Reports
leapfrog-steps/s per G (same workload as bench.py: Burgers shapes, K = 17,240, L = 7, eps = 1e-4).

    python profiles/scripts/probes/probe_groups.py --groups 1 2 4 --steps 20
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "vi-hmc_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--chains", type=int, default=16)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    from vihmc.data import deeponet_problem
    from vihmc.engine import DeepONetEngine, trunk_features
    from vihmc.layout import DeepONetSpec
    from vihmc.samplers import ChainRNG, EngineEvaluator, HMCRunner
    dev = torch.device("cuda", 0)
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    tf = trunk_features(prob.trunk_in)
    th = torch.tensor(prob.mu[prob.grad_ind], device=dev)
    for rep in range(a.reps):
        for G in a.groups:
            cg = a.chains // G
            engs = [DeepONetEngine(spec, prob.branch_in, tf, prob.y, prob.mu, prob.grad_ind, 0.0, 0.1, "NLL", 1.0,
                                   max_chains=cg, device=dev) for _ in range(G)]
            streams = [torch.cuda.Stream(dev) for _ in range(G)] if G > 1 else [torch.cuda.current_stream(dev)]
            runners = []
            for g in range(G):
                with torch.cuda.stream(streams[g]):
                    runners.append(HMCRunner(EngineEvaluator(engs[g]), th[None].repeat(cg, 1), a.warmup + a.steps,
                                             7, 1e-4, rng=ChainRNG(cg, engs[g].K, dev,
                                                                   seeds=[1000 + g * cg + c for c in range(cg)])))
            for _ in range(a.warmup):
                for g in range(G):
                    with torch.cuda.stream(streams[g]):
                        runners[g].step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                for g in range(G):
                    with torch.cuda.stream(streams[g]):
                        runners[g].step()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(f"rep {rep} G={G} ({cg} chains each): {a.chains * 7 * a.steps / dt:.0f} leapfrog-steps/s, "
                  f"{dt / a.steps * 1e3:.3f} ms per HMC step", flush=True)
            for e in engs:
                e.close()
            del runners


if __name__ == "__main__":
    main()
