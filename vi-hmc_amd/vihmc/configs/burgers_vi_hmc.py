"""Operator_network/VI_HMC/config.py:11-56 (DeepONet VI-HMC on Burgers; BASELINE config 5)."""
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

step_size = 1e-4
num_samples = 1000
burn = 100
load_prior = False
load_std = False
prior_file = "VI/Saved_models/Burgers"
prior_uid = "synthetic"
init_prior = False
sample_prior = True
prior_var = 0.1 ** 2
post_var = 0.0214 ** 2
L = int(np.pi * post_var / (2 * step_size))          # 7

loss = "NLL"
tau_out = 1.0 ** 2
evaluate = False
eval_dt_string = ""
out_dir = "samples/Burgers/"

# build additions
num_chains = 16            # total chains (sharded over ranks)
seed = 0                   # chain c uses seed + 1000 + c
sensitive_k = 17240        # size of the synthetic sensitive set when artefacts are generated
reuse_endpoint_grad = True
