"""Time one batched DeepONet log-prob+grad evaluation (Burgers shapes) on the GPU.

    python profiles/scripts/probes/probe_eval.py --chains 16 --iters 10
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "vi-hmc_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.engine import DeepONetEngine, trunk_features  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, nargs="+", default=[1, 16])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--no-timing", action="store_true", help="leave the HIP-event kernel timing off (graph path)")
    ap.add_argument("--host", action="store_true",
                    help="also time the PCIe-inclusive path: theta from pinned host memory, logp + grad copied back")
    args = ap.parse_args()
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    eng = DeepONetEngine(spec, prob.branch_in, trunk_features(prob.trunk_in), prob.y, prob.mu, prob.grad_ind, 0.0, 0.1,
                         "NLL", 1.0, max_chains=max(args.chains), device="cuda:0")
    print(f"plan device bytes: {eng.device_bytes / 1e6:.1f} MB", flush=True)
    fl = spec.flops_per_grad_eval(prob.N, prob.P)
    for C in args.chains:
        th = torch.tensor(np.tile(prob.mu[prob.grad_ind], (C, 1)), device="cuda:0")
        th += 0.001 * torch.randn_like(th)
        for _ in range(3):
            eng.logp_grad(th)
        torch.cuda.synchronize()
        if not args.no_timing:
            eng.timing(0, True)
        t0 = time.perf_counter()
        for _ in range(args.iters):
            lp, g = eng.logp_grad(th)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.iters
        kms, n = (0.0, 0) if args.no_timing else eng.timing_read()
        eng.timing(0, False)
        print(f"C={C:3d}  {dt * 1e3:8.3f} ms/eval  {C / dt:9.1f} grad-evals/s  "
              f"{fl * C / dt / 1e12:6.2f} TFLOP/s algorithmic  contractA {kms / max(n, 1):.3f} ms  "
              f"logp0={lp[0].item():.4f}", flush=True)
        if args.host:
            th_h = th.cpu().pin_memory()
            lp_h = torch.empty(C, pin_memory=True)
            g_h = torch.empty(th.shape, pin_memory=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                lp, g = eng.logp_grad(th_h.to("cuda:0", non_blocking=True))
                lp_h.copy_(lp, non_blocking=True)
                g_h.copy_(g, non_blocking=True)
            torch.cuda.synchronize()
            dth = (time.perf_counter() - t0) / args.iters
            print(f"C={C:3d}  host in/out (PCIe-inclusive): {dth * 1e3:8.3f} ms/eval  {C / dth:9.1f} grad-evals/s  "
                  f"({2 * th.numel() * 4 / 1e6:.2f} MB per eval over PCIe)", flush=True)


if __name__ == "__main__":
    main()
