"""CPU-baseline check (test infrastructure, runs only where /root/reference exists, i.e. the build
container): times one DeepONet VI-HMC log-prob + gradient of the reference's own closure
(Operator_network/VI_HMC/main_VI_HMC_burgers.py:27-178, imported read-only with the hamiltorch stub of
tests/golden/make_golden.py) against the oracle restatement that bench.py times on the GPU box
(oracle/deeponet_ref.TorchDeepONetRef), same inputs, same thread count (SURVEY §8d asks for both).

    python oracle/time_reference_cpu.py [threads]
"""
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "vi-hmc_amd"))

import torch  # noqa: E402


def bench(fn, th, n=5):
    for _ in range(2):
        p = th.clone().requires_grad_()
        torch.autograd.grad(fn(p).sum(), p)
    t0 = time.perf_counter()
    for _ in range(n):
        p = th.clone().requires_grad_()
        torch.autograd.grad(fn(p).sum(), p)
    return (time.perf_counter() - t0) / n


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.set_num_threads(threads)
    import tempfile
    import make_golden as MG
    from oracle.deeponet_ref import TorchDeepONetRef, deeponet_layout
    from vihmc.data import deeponet_problem, save_vi_artefacts
    from vihmc.layout import DeepONetSpec

    spec = DeepONetSpec()
    prob = deeponet_problem(seed=0)
    MG.stub_hamiltorch()
    M = MG.import_ref("Operator_network/VI_HMC", "main_VI_HMC_burgers")
    cfg = M.cfg
    tmp = tempfile.mkdtemp()
    cfg.branch_depth, cfg.trunk_depth, cfg.activation = spec.depth_branch, spec.depth_trunk, spec.activation
    cfg.load_prior, cfg.sample_data = False, False
    cfg.prior_file, cfg.prior_uid = tmp, "timing"
    save_vi_artefacts(tmp, "timing", prob.mu, prob.sigma, prob.grad_ind)
    net = M.DeepONet(spec.width_branch, spec.width_trunk, spec.in_branch, spec.in_trunk, spec.depth_branch,
                     spec.depth_trunk, spec.activation, spec.output_neurons)
    tr = (torch.from_numpy(prob.branch_in), torch.from_numpy(prob.trunk_in), torch.from_numpy(prob.y))
    fn_ref = M.define_model_log_prob(net, cfg.loss, tr, [torch.tensor(cfg.prior_var)], cfg.tau_out, device="cpu")
    ref = TorchDeepONetRef(deeponet_layout(), prob.branch_in, prob.trunk_in, prob.y, prob.mu, prob.grad_ind, 0.0,
                           float(cfg.prior_var) ** 0.5, cfg.loss, float(cfg.tau_out))
    th = torch.tensor(prob.mu[prob.grad_ind])
    t_ref = bench(fn_ref, th)
    t_port = bench(ref.log_prob, th)
    print(f"threads={threads}  reference closure {t_ref:.3f} s/grad-eval   oracle restatement {t_port:.3f} s/grad-eval"
          f"   ratio {t_ref / t_port:.2f}")


if __name__ == "__main__":
    main()
