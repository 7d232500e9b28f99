"""vihmc -- MI355X-native VI-HMC log-posterior/gradient engine and hamiltorch-compatible sampler."""
from .layout import DeepONetSpec, MLPSpec  # noqa: F401

__version__ = "0.1.0"
