"""The multi-GPU path on RCCL: the driver launches `bench.py` / the entry scripts as
`python -m torch.distributed.run --nproc-per-node N` with the ``nccl`` backend. On the one-GPU test box this runs
that launch form at N = 1 (tests/dist_nccl_child.py): RCCL initialises on the device, the batched HIP sampler
samples the rank's chain block, and a real all-gather + all-reduce move the pool. The gathered pool must equal
this process's own run of the same chains bit for bit (chain seeds do not depend on the world size; the gloo
world-size-2 test in tests/test_dist.py covers the block partition and multi-rank padding)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from goldens import deeponet_case

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_nccl_launch_form_pool_equals_single_process(tmp_path, cuda_device):
    from vihmc.dist import chain_seeds
    from vihmc.engine import DeepONetEngine, trunk_features
    from vihmc.samplers import ChainRNG, EngineEvaluator, run_chains
    out = str(tmp_path / "pool.pt")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(HERE, "dist_nccl_child.py"), "--out", out,
           "--chains", "2"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    got = torch.load(out, weights_only=True)
    assert got["backend"] == "nccl"
    c = deeponet_case("deeponet_small")
    p = c.prob
    eng = DeepONetEngine(c.spec, p.branch_in, trunk_features(p.trunk_in), p.y, p.mu, p.grad_ind, c.prior_mu,
                         c.prior_sd, c.loss, c.tau_out, max_chains=2, device=cuda_device)
    th0 = torch.tensor(np.asarray(c.thetas[0]))
    ref = run_chains(EngineEvaluator(eng), th0[None].repeat(2, 1), 6, 7, 2e-3,
                     rng=ChainRNG(2, th0.numel(), cuda_device, seeds=chain_seeds(range(2))))
    assert torch.equal(got["pool"], ref.stacked().cpu())
    assert float(got["acc"][0]) == float(ref.accepted.sum())
