"""The reference's entry scripts, rebuilt on the engine, run end to end on the GPU at reduced sizes (each as
one child process of the test, run one at a time): Operator_network/VI_HMC/main_VI_HMC_burgers.py (sampling,
then cfg.evaluate on a saved run), post_process_burgers.py (fnames.txt pooling), Operator_network/HMC/
main_HMC_splitting.py (config 4), NUTS_DeepOnets.py, Neural_network/HMC/main_regression_hmc.py (config 1,
then its validate mode) and Neural_network/VI_HMC/main_VI_HMC.py (configs 2-3)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
SCRIPTS = os.path.join(ROOT, "vi-hmc_amd", "scripts")


def run(script, args, cwd):
    r = subprocess.run([sys.executable, os.path.join(SCRIPTS, script)] + args, cwd=cwd, capture_output=True, text=True,
                       timeout=240)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stderr[-4000:]
    return r.stdout


def test_vi_hmc_burgers_sample_evaluate_and_pool(tmp_path):
    out = str(tmp_path / "samples") + "/"
    so = run("main_VI_HMC_burgers.py", ["--num-samples", "6", "--chains", "2", "--n-train", "12", "--out-dir", out],
             tmp_path)
    assert "Expected MSE" in so and "posterior-predictive mean" in so
    uids = open(os.path.join(out, "fnames.txt")).read().split()
    assert len(uids) == 2
    for u in uids:
        s = np.load(os.path.join(out, f"hmc_params_{u}.npy"))
        assert s.shape[1] == 17240 and s.shape[0] >= 2
    so = run("main_VI_HMC_burgers.py", ["--evaluate", uids[0], "--burn", "1", "--n-train", "12", "--out-dir", out],
             tmp_path)
    assert "Evaluating" in so and "Expected MSE" in so
    so = run("post_process_burgers.py", ["--out-dir", out, "--burn", "1", "--n-train", "12"], tmp_path)
    assert "Mean Relative L2 error" in so and "pooled 2 runs" in so


def test_hmc_splitting_config4_script(tmp_path):
    so = run("main_HMC_splitting.py", ["--num-samples", "3", "--n-train", "8", "--out-dir", str(tmp_path)], tmp_path)
    assert "Number of splits:  2" in so and "Expected MSE" in so
    f = [x for x in os.listdir(tmp_path) if x.startswith("hmc_params_")]
    assert len(f) == 1 and np.load(tmp_path / f[0]).shape[1] == 172401


def _full_prior(d, D=172401, seed=3):
    """means_flattened / stds_flattened as the reference's full-parameter scripts read them (no uid)."""
    import torch
    rs = np.random.default_rng(seed)
    os.makedirs(d, exist_ok=True)
    torch.save(torch.from_numpy((0.05 * rs.standard_normal(D)).astype(np.float32)), os.path.join(d, "means_flattened"))
    torch.save(torch.from_numpy((0.01 + 0.02 * rs.random(D)).astype(np.float32)), os.path.join(d, "stds_flattened"))
    return d


def test_hmc_splitting_and_nuts_load_prior(tmp_path):
    """cfg.load_prior / cfg.init_prior on the full-parameter scripts: {prior_file}/means_flattened and
    stds_flattened, no uid and no gradient indices (main_HMC_splitting.py:343-344, NUTS_DeepOnets.py:270-271)."""
    pf = _full_prior(str(tmp_path / "prior"))
    so = run("main_HMC_splitting.py", ["--num-samples", "3", "--n-train", "8", "--out-dir", str(tmp_path / "s"),
                                       "--prior-file", pf], tmp_path)
    assert "Number of splits:  2" in so and "Expected MSE" in so
    so = run("NUTS_DeepOnets.py", ["--num-samples", "4", "--burn", "2", "--out-dir", str(tmp_path / "n"),
                                   "--prior-file", pf], tmp_path)
    assert "final step sizes" in so and "Expected MSE" in so


def test_nuts_deeponets_script(tmp_path):
    so = run("NUTS_DeepOnets.py", ["--num-samples", "5", "--burn", "2", "--out-dir", str(tmp_path)], tmp_path)
    assert "final step sizes" in so and "Expected MSE" in so


def test_regression_hmc_script_and_validate(tmp_path):
    so = run("main_regression_hmc.py", ["--num-samples", "6", "--L", "30", "--out-dir", str(tmp_path)], tmp_path)
    assert "Expected MSE" in so
    f = [x for x in os.listdir(tmp_path) if x.startswith("hmc_params_")]
    assert len(f) == 1 and np.load(tmp_path / f[0]).shape[1] == 141
    dt = f[0][len("hmc_params_"):-len(".npy")]
    so = run("main_regression_hmc.py", ["--num-samples", "6", "--test", dt, "--out-dir", str(tmp_path)], tmp_path)
    assert "Expected validation log probability" in so


def test_bnn_vi_hmc_script(tmp_path):
    so = run("main_VI_HMC.py", ["--num-samples", "8", "--chains", "3"], tmp_path)
    assert "acceptance rate per chain" in so and "Expected MSE" in so
