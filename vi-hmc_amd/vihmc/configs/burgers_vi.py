"""Operator_network/VI/config.py:10-53 (Bayesian DeepONet BBB training on Burgers) + config_sens.py:10-37
(sensitivity step)."""
# Training params
batch_size = 128
epochs = 10
lr_start = 1e-3
lr_patience = 500
n_save = int(epochs / 10)

# Network params
width_branch = 100
width_trunk = 100
branch_depth = 9
trunk_depth = 9
in_branch = 101
in_trunk = 5
output_neurons = 100
activation = "tanh"

# Data params
dataset = "Burgers"
p = 10201
N_train = 1000
N_valid = 1000

# Learning params
priors = {
    "prior_mu": 0,
    "prior_sigma": 0.1,
    "posterior_mu_initial": (0, 0.1),
    "posterior_rho_initial": (-5, 0.1),
}
num_ens = 5
beta_type = 1.0

# Noise params
learn_noise = False
noise_type = 0
noise_neuron = 0
noise_param = 1.0 ** 2

# sensitivity step (config_sens.py)
sens_p = 100                 # trunk points per validation function
importance_threshold = 0.90

# build additions
seed = 0
save_loc = "VI/Saved_models/Burgers"
uid = "synthetic"
