#!/usr/bin/env python3
"""BNN leapfrog-step timing (configs 2-3 network, bench.leg_bnn) at 1 and 8 chains per GPU, for A/B of the MLP
kernels: the register-resident kernels (default) and the generic LDS kernels (--generic, plan option mlp_fast = 0).
One line per chain count."""
import argparse
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vi-hmc_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--generic", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for C in (1, 8):
        r = bench.leg_bnn(dev, C, steps=args.steps, fast=not args.generic)
        print(f"{args.tag} C={C} us/leapfrog-step {r['us_per_leapfrog_step']:.2f} kernel {r['kernel_us_per_leapfrog_step']:.2f}"
              f" leapfrog-steps/s {r['leapfrog_steps_per_s']:.0f}", flush=True)


if __name__ == "__main__":
    main()
