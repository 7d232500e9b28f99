"""Operator_network/HMC/config.py (full-parameter DeepONet HMC with dual-averaging adaptation,
NUTS_DeepOnets.py)."""
import numpy as np

width_branch = 100
width_trunk = 100
branch_depth = 9
trunk_depth = 9
in_branch = 101
in_trunk = 5
output_neurons = 100
activation = "tanh"

step_size = 1e-4
num_samples = 10
burn = num_samples // 10
load_prior = False
prior_file = "Saved_models/"
prior_uid = ""
init_prior = False
prior_var = 0.1 ** 2
post_var = 0.0214 ** 2
L = int(np.pi * post_var / (2 * step_size))          # 7

dataset = "Burgers"
sample_data = False
p = 10201
N_train = 10
N_valid = 10

loss = "NLL"
tau_out = 1.0 ** 2
out_dir = "Experiments/"

# build additions
num_chains = 1
seed = 0
reuse_endpoint_grad = True
