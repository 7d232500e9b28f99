"""Flat-parameter layout tables for the two model families on the VI-HMC hot path.

The reference keeps every network as one flat fp32 vector in ``named_parameters`` order and
views it per tensor with ``util.unflatten`` (Operator_network/VI_HMC/util.py:141-152,
Neural_network/VI_HMC/util.py:121-136).  The order is fixed by module construction:

* DeepONet (Operator_network/VI_HMC/model.py:11-35): scalar output bias ``b`` first (model.py:26),
  then the branch ``nn.Sequential`` (model.py:42-51), then the trunk (model.py:53-62); every
  ``nn.Linear`` contributes ``weight[out,in]`` (row-major) then ``bias[out]``.
* BNN MLP (Neural_network/VI_HMC/main_VI_HMC.py:297-334): ``Linear(1,w0)``, ``depth`` hidden
  ``Linear(w_i,w_{i+1})`` and ``Linear(w_last,1,bias=bias_on)``.

The tables here are what the HIP plan uploads: one row per linear layer with the weight and bias
offsets into the flat vector, the fan-in/fan-out and whether an activation follows.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

ACT_IDENTITY = 0
ACT_TANH = 1
ACT_RELU = 2
ACT_SINE = 3

_ACT_CODES = {"tanh": ACT_TANH, "relu": ACT_RELU, "sine": ACT_SINE, "identity": ACT_IDENTITY}


def act_code(name: str) -> int:
    try:
        return _ACT_CODES[name]
    except KeyError:
        raise ValueError("activation should be relu, sine or tanh") from None


@dataclass(frozen=True)
class Linear:
    w_off: int          # offset of weight[n_out, n_in] in the flat vector
    b_off: int          # offset of bias[n_out], -1 when the layer has no bias
    n_out: int
    n_in: int
    act: int            # activation applied after this layer (ACT_IDENTITY for the last)


@dataclass(frozen=True)
class DeepONetSpec:
    """Shape of ``DeepONet(width_branch, width_trunk, in_branch, in_trunk, depth_branch, depth_trunk,
    activation, output_neurons)`` (Operator_network/VI_HMC/model.py:11-35).  ``impose_bc`` selects the
    trunk feature map ``[t, sin2πx, sin4πx, cos2πx, cos4πx]`` (my_make_func.py:33-36,63-65)."""
    width_branch: int = 100
    width_trunk: int = 100
    in_branch: int = 101
    in_trunk: int = 5
    depth_branch: int = 9
    depth_trunk: int = 9
    activation: str = "tanh"
    output_neurons: Optional[int] = None
    impose_bc: bool = True

    @property
    def out(self) -> int:
        return self.width_branch if self.output_neurons is None else self.output_neurons

    def _mlp(self, off: int, n_in: int, width: int, depth: int) -> (List[Linear], int):
        act = act_code(self.activation)
        dims = [n_in] + [width] * (depth - 1) + [self.out]
        layers = []
        for i in range(depth):
            fi, fo = dims[i], dims[i + 1]
            layers.append(Linear(off, off + fo * fi, fo, fi, act if i < depth - 1 else ACT_IDENTITY))
            off += fo * fi + fo
        return layers, off

    @property
    def branch(self) -> List[Linear]:
        return self._mlp(1, self.in_branch, self.width_branch, self.depth_branch)[0]

    @property
    def trunk(self) -> List[Linear]:
        _, off = self._mlp(1, self.in_branch, self.width_branch, self.depth_branch)
        return self._mlp(off, self.in_trunk, self.width_trunk, self.depth_trunk)[0]

    @property
    def n_params(self) -> int:
        _, off = self._mlp(1, self.in_branch, self.width_branch, self.depth_branch)
        return self._mlp(off, self.in_trunk, self.width_trunk, self.depth_trunk)[1]

    def flops_per_grad_eval(self, n: int, p: int) -> float:
        """Algorithmic FLOP of one log-prob + gradient evaluation for one chain (2 per MAC):
        forward MLPs + branch×trunk contraction, backward = 2× each GEMM (dX and dW, no dX for the
        input layer) + 2× the contraction (dZ_b, dZ_t)."""
        fwd = bwd = 0.0
        for rows, layers in ((n, self.branch), (p, self.trunk)):
            for i, l in enumerate(layers):
                g = 2.0 * rows * l.n_in * l.n_out
                fwd += g
                bwd += g if i == 0 else 2 * g
        c = 2.0 * n * p * self.out
        return fwd + c + bwd + 2 * c

    def flops_by_kernel(self, n: int, p: int) -> dict:
        """Algorithmic FLOP per chain of each kernel class of one gradient evaluation (include/vihmc.h
        VIHMC_T_*): input layers (row-dot), hidden + last layers (fused forward), contraction side A
        (S = Z_b Z_t^T and dZ_t = G^T Z_b), side B (dZ_b = G Z_t), layer backward (dW every layer, dX all but
        the input layer). They sum to flops_per_grad_eval."""
        d = {"input": 0.0, "fwd": 0.0, "bwd": 0.0}
        for rows, layers in ((n, self.branch), (p, self.trunk)):
            for i, l in enumerate(layers):
                g = 2.0 * rows * l.n_in * l.n_out
                d["input" if i == 0 else "fwd"] += g
                d["bwd"] += g if i == 0 else 2 * g
        c = 2.0 * n * p * self.out
        d["contract_a"] = 2 * c
        d["contract_b"] = c
        return d

    def flops_gram(self, n: int, p: int, centred: bool = True) -> float:
        """Algorithmic FLOP per chain of the Gram-form gradient-only contraction (vihmc_gram.hip, the inner
        leapfrog evaluations), which replaces side A + side B there: y Zt^ and y^T Zb^ (2 N P (W+1) each) and the
        (N + P) (W+1)^2 Gram / correction products (Zt^T Zt^, Zb^T Zb^, Zt^ Gb, Zb^ Gt), augmented width W + 1.
        Centred (plan option gram_center, round 6): also Ht = dT^T Zt^, Hb = dB^T Zb^ and the second correction of
        each side (B0 Ht, T0 Hb)."""
        wa = self.out + 1
        return 4.0 * n * p * wa + (8.0 if centred else 4.0) * (n + p) * wa * wa


@dataclass(frozen=True)
class MLPSpec:
    """BNN regression net ``get_model`` (Neural_network/VI_HMC/main_VI_HMC.py:297-334) evaluated by
    ``Functional_Net.functional_model`` (Neural_network/VI_HMC/my_make_func.py:52-73)."""
    width: tuple = (10, 10)
    act: str = "tanh"
    bias: bool = True
    in_dim: int = 1
    out_dim: int = 1

    @property
    def layers(self) -> List[Linear]:
        dims = [self.in_dim] + list(self.width) + [self.out_dim]
        act = act_code(self.act)
        out, off = [], 0
        for i in range(len(dims) - 1):
            fi, fo = dims[i], dims[i + 1]
            last = i == len(dims) - 2
            has_b = (not last) or self.bias
            out.append(Linear(off, off + fo * fi if has_b else -1, fo, fi, ACT_IDENTITY if last else act))
            off += fo * fi + (fo if has_b else 0)
        return out

    @property
    def tensor_sizes(self) -> List[int]:
        """``[p.nelement() for p in model.parameters()]`` (main_VI_HMC.py:367-369)."""
        sizes = []
        for l in self.layers:
            sizes.append(l.n_out * l.n_in)
            if l.b_off >= 0:
                sizes.append(l.n_out)
        return sizes

    @property
    def n_params(self) -> int:
        return sum(self.tensor_sizes)
