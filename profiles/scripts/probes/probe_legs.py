"""The bench's one-chain legs only (VI-HMC DeepONet at one chain, config 4's splitting HMC), for A/B runs of two
builds (VIHMC_LIB selects the library).

    python profiles/scripts/probes/probe_legs.py --reps 2
"""
import argparse
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    for _ in range(a.reps):
        c1 = bench.leg_deeponet_c1(prob, spec, dev, 7, 1e-4)
        c4 = bench.leg_split_c1(spec, dev, 7, 1e-4)
        print(json.dumps({"c1_lf_per_s": c1.get("leapfrog_steps_per_s"), "c1_eval_ms": c1.get("ms_per_eval"),
                          "c4_lf_per_s": c4.get("leapfrog_steps_per_s"),
                          "c4_half_eval_ms": c4.get("ms_per_half_shard_eval")}), flush=True)


if __name__ == "__main__":
    main()
