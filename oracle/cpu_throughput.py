"""ORACLE (test / CPU-baseline infrastructure only) -- multi-chain CPU throughput of the reference path.

SURVEY.md §8d asks for the CPU reference timed two ways on the GPU box's host: all cores on one chain
(bench.py's in-process leg) and one process per core at one thread each for multi-chain throughput (this
file). ``run_parallel`` starts ``procs`` child processes of this script (plain subprocesses, no fork of a
GPU-initialised interpreter); each runs ONE chain of the reference log-prob (TorchDeepONetRef: the
reference's torch ops, fp32) inside the scalar hamiltorch loop (oracle/hamiltorch_ref.py, L+1 gradient and
2 value evaluations per sample) with ``torch.set_num_threads(1)`` until ``seconds`` have passed, and
prints its leapfrog steps and wall time. The pool's throughput is the sum of the per-process rates.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def worker(chain: int, seconds: float, L: int, eps: float) -> dict:
    import torch
    torch.set_num_threads(1)
    sys.path[:0] = [ROOT, os.path.join(ROOT, "vi-hmc_amd")]
    from oracle import hamiltorch_ref as HR
    from oracle.deeponet_ref import TorchDeepONetRef, deeponet_layout
    from vihmc.data import deeponet_problem
    prob = deeponet_problem(seed=0)
    ref = TorchDeepONetRef(deeponet_layout(), prob.branch_in, prob.trunk_in, prob.y, prob.mu, prob.grad_ind, 0.0, 0.1,
                           "NLL", 1.0)
    th = torch.tensor(prob.mu[prob.grad_ind])
    g = torch.Generator().manual_seed(1000 + chain)
    n = 0
    t0 = time.perf_counter()
    while True:
        th = HR.sample(ref.log_prob, th, 1, L, eps, generator=g)[-1]
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"chain": chain, "samples": n, "leapfrog": n * L, "seconds": dt}


def run_parallel(procs: int, seconds: float, L: int = 7, eps: float = 1e-4) -> dict:
    # the workers never touch the GPU, but a ROCm torch import still counts against the GPU box's
    # per-GPU process limit (16 with the parent): keep procs <= 14 there
    env = dict(os.environ, OMP_NUM_THREADS="1", MKL_NUM_THREADS="1", HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="",
               CUDA_VISIBLE_DEVICES="")
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), str(c), str(seconds), str(L), str(eps)],
                           stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, env=env, cwd=ROOT)
          for c in range(procs)]
    res = []
    for p in ps:
        out, _ = p.communicate(timeout=seconds * 4 + 300)
        if p.returncode != 0:
            raise RuntimeError(f"cpu throughput worker failed (rc {p.returncode})")
        res.append(json.loads(out.decode().strip().splitlines()[-1]))
    rate = sum(r["leapfrog"] / r["seconds"] for r in res)
    return {"value": rate, "procs": procs, "samples": sum(r["samples"] for r in res),
            "seconds_max": max(r["seconds"] for r in res)}


if __name__ == "__main__":
    c, sec, L, eps = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4])
    print(json.dumps(worker(c, sec, L, eps)), flush=True)
