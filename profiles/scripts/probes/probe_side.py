"""Config 4's split HMC leg with the end-point value evaluation on a side stream (HMCRunner.side_value) on and off,
alternating: python profiles/scripts/probes/probe_side.py [reps]. Ran against the side-stream change that was measured
and not kept (profiles/r05s2_side_stream_ab.txt); on the current tree both arms run the same code."""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402
from vihmc.samplers import HMCRunner  # noqa: E402

spec = DeepONetSpec()
dev = torch.device("cuda", 0)
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    for on in (False, True):
        HMCRunner.side_value = on
        a = bench.leg_split_c1(spec, dev, 7, 1e-4)
        print(json.dumps({"side_value": on, "c4_lf_per_s": round(a["leapfrog_steps_per_s"], 1),
                          "ms_per_hmc_step": round(a["ms_per_hmc_step"], 4)}), flush=True)
