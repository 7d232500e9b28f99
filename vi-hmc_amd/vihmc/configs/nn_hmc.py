"""Neural_network/HMC/config.py:12-38 (plain HMC on all 141 BNN parameters; BASELINE config 1)."""
import numpy as np

N_tr = 20
N_val = 300
width = 2 * [10]
act = "tanh"
depth = len(width) - 1
bias = True

tau = 1.
step_size = 1e-4
num_samples = 1000
post_var = 0.2024 ** 2
L = int(np.pi * post_var / (2 * step_size))          # 643
tau_out = 1 / 5e-2 ** 2
burn = num_samples // 5
num_chains = 1

out_dir = "samples"
test = False
test_dtstring = ""
seed = 0
