"""LRP rule descriptors with zennit 0.5.1 names and constructor signatures.

Semantics (reference name maps ``constants.py:27-51``):
  Epsilon(ε)   R_in = x ⊙ Jᵀ_W(R / stab_ε(z))
  Gamma(γ, ε)  W± = W + γ·W.clamp(min/max=0) (bias likewise); positive/negative output split;
               den± = f(x+; W±, b±) + f(x-; W∓, 0) (zennit 0.5.1 zero_bias on the x- terms)
  WSquare(ε)   R_in = Jᵀ_{W²}(R / stab_ε(conv(1; W², b²)))
  Flat(ε)      as WSquare with W -> 1, b -> 0
  Pass()       R_in = R_out (activation layers only)
  ZPlus(ε)     z = f(x+; W+, b+) + f(x-; W-, 0);  R_in = x+ ⊙ Jᵀ_{W+} g + x- ⊙ Jᵀ_{W-} g,
               g = R / stab_ε(z)   (conv layers; runs on the Gamma kernels with these sets)
  AlphaBeta(α, β, ε)  positive set (x+, W+, b+) + (x-, W-, 0), negative set (x+, W-, b-) + (x-, W+, 0),
               one denominator per set; R_in = α·pos − β·neg (HIP engine: convs with a non-negative
               input; elsewhere compiling the composite raises ``EngineError``)
  Norm(ε)      ≡ Epsilon(ε) on conv/dense layers
A ``Hook`` subclass with its own ``backward`` (not a descriptor) runs on the autograd slow path
(``engine/hooks.py``).
"""
from __future__ import annotations

from .core import BasicHook, Stabilizer


class Epsilon(BasicHook):
    kind = "epsilon"

    def __init__(self, epsilon=1e-6, zero_params=None):
        super().__init__(zero_params)
        self.epsilon = Stabilizer.ensure(epsilon).epsilon


class Gamma(BasicHook):
    kind = "gamma"

    def __init__(self, gamma=0.25, stabilizer=1e-6, zero_params=None):
        super().__init__(zero_params)
        self.gamma = float(gamma)
        self.stabilizer = Stabilizer.ensure(stabilizer).epsilon


class WSquare(BasicHook):
    kind = "wsquare"

    def __init__(self, stabilizer=1e-6, zero_params=None):
        super().__init__(zero_params)
        self.stabilizer = Stabilizer.ensure(stabilizer).epsilon


class Flat(BasicHook):
    kind = "flat"

    def __init__(self, stabilizer=1e-6, zero_params=None):
        super().__init__(zero_params)
        self.stabilizer = Stabilizer.ensure(stabilizer).epsilon


class Pass(BasicHook):
    kind = "pass"

    def __init__(self):
        super().__init__()


class ZPlus(BasicHook):
    kind = "zplus"

    def __init__(self, stabilizer=1e-6, zero_params=None):
        super().__init__(zero_params)
        self.stabilizer = Stabilizer.ensure(stabilizer).epsilon


class AlphaBeta(BasicHook):
    kind = "alphabeta"

    def __init__(self, alpha=2.0, beta=1.0, stabilizer=1e-6, zero_params=None):
        # zennit 0.5.1 refuses these configurations (conservation needs alpha - beta = 1)
        if alpha < 0 or beta < 0:
            raise ValueError("Both alpha and beta parameters must be non-negative!")
        if (alpha - beta) != 1.0:
            raise ValueError("The difference of parameters alpha - beta must equal 1!")
        super().__init__(zero_params)
        self.alpha, self.beta = float(alpha), float(beta)
        self.stabilizer = Stabilizer.ensure(stabilizer).epsilon


class Norm(BasicHook):
    kind = "norm"

    def __init__(self, stabilizer=1e-6):
        super().__init__()
        self.stabilizer = Stabilizer.ensure(stabilizer).epsilon
