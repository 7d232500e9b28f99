"""Config modules with the reference's names and values (module attributes read as ``cfg.X``), plus
the build's additions: num_chains, seed, chains_per_gpu, reuse_endpoint_grad, synthetic data."""
import copy
import importlib
import types


def load(name: str, **overrides) -> types.SimpleNamespace:
    """A mutable copy of config module ``name`` with overrides applied."""
    mod = importlib.import_module(f"{__name__}.{name}")
    ns = types.SimpleNamespace(**{k: copy.deepcopy(v) for k, v in vars(mod).items()
                                  if not k.startswith("_") and not isinstance(v, types.ModuleType)})
    for k, v in overrides.items():
        setattr(ns, k, v)
    return ns
