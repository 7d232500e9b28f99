"""Operator_network/HMC/config_splitting.py (full-parameter DeepONet HMC, split over 2 data shards)."""
import numpy as np

width_branch = 100
width_trunk = 100
branch_depth = 9
trunk_depth = 9
in_branch = 101
in_trunk = 5
output_neurons = 100
activation = "tanh"

dataset = "Burgers"
sample_data = False
p = 10201
N_train = 1000
N_valid = 1000

is_nuts = False
step_size = 1e-4
num_samples = 1001
burn = num_samples // 2
load_prior = False
load_std = False
init_prior = False
prior_file = "Saved_models/Burgers"
prior_uid = "020125162111"
prior_var = 0.1 ** 2
post_var = 0.0214 ** 2
L = int(np.pi * post_var / (2 * step_size))
split = True
num_splits = 2
loss = "NLL"
tau_out = 1.0 ** 2
out_dir = "samples/Burgers/"
evaluate = False
eval_uid = "01"

num_chains = 1
seed = 0
reuse_endpoint_grad = True
