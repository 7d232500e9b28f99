"""Neural_network/VI_HMC/config.py:11-39 (BNN VI-HMC; BASELINE configs 2-3)."""
import numpy as np

N_tr = 20
N_val = 300
width = 2 * [10]
act = "tanh"
depth = len(width) - 1
bias = True

step_size = 5e-4
num_samples = 100
burn = num_samples // 5
prior_var = 1.0
post_var = 0.2501 ** 2
L = int(np.pi * post_var / (2 * step_size))          # 196
loss = "NLL"
tau_out = 5e-2 ** 2
num_chains = 10

out_dir = "samples_large_network/try/"
load_prior = False
load_std = False
prior_file = "VI/checkpoints/Sensitivity"
prior_uid = "synthetic"
init_prior = False
test = False
test_dtstring = ""

seed = 0
reuse_endpoint_grad = True
