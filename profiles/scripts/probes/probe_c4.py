"""Config 4's split HMC leg alone (bench.leg_split_c1), for a kernel trace: python profiles/scripts/probes/probe_c4.py"""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

a = bench.leg_split_c1(DeepONetSpec(), torch.device("cuda", 0), 7, 1e-4)
print(json.dumps({k: v for k, v in a.items() if k != "note"}))
