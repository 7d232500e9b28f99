"""bench.py's one-chain side legs alone (config 4's split HMC and the one-chain VI-HMC DeepONet), repeated:
python profiles/scripts/diag/legs_c1.py [reps]"""
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vi-hmc_amd"))

import bench  # noqa: E402
if os.environ.get("SAMPLERS_FILE"):          # A/B of the sampler module (e.g. a previous revision)
    import importlib.util
    import vihmc
    sp = importlib.util.spec_from_file_location("vihmc.samplers", os.environ["SAMPLERS_FILE"])
    mod = importlib.util.module_from_spec(sp)
    sys.modules["vihmc.samplers"] = mod
    sp.loader.exec_module(mod)
    vihmc.samplers = mod
from vihmc.data import deeponet_problem  # noqa: E402
from vihmc.layout import DeepONetSpec  # noqa: E402

spec = DeepONetSpec()
prob = deeponet_problem(seed=0)
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    a = bench.leg_split_c1(spec, "cuda:0", 7, 1e-4)
    b = bench.leg_deeponet_c1(prob, spec, "cuda:0", 7, 1e-4)
    print(json.dumps({"config4_leapfrog_steps_per_s": round(a["leapfrog_steps_per_s"], 1),
                      "config4_ms_per_half_shard_eval": round(a["ms_per_half_shard_eval"], 4),
                      "c1_leapfrog_steps_per_s": round(b["leapfrog_steps_per_s"], 1),
                      "c1_ms_per_eval": round(b["ms_per_eval"], 4)}), flush=True)
