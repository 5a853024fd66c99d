"""Core descriptor types (zennit.core equivalents)."""
from __future__ import annotations

from typing import Iterable, Optional


class Stabilizer:
    """zennit ``Stabilizer``: t -> t + eps * (sign(t) + [t == 0]) (clip/norm_scale unsupported)."""

    def __init__(self, epsilon: float = 1e-6, clip: bool = False, norm_scale: bool = False, dim=None):
        if clip or norm_scale or dim is not None:
            raise NotImplementedError("Stabilizer(clip/norm_scale/dim) is not supported by the HIP engine")
        self.epsilon = float(epsilon)

    @classmethod
    def ensure(cls, value) -> "Stabilizer":
        if isinstance(value, Stabilizer):
            return value
        if isinstance(value, (int, float)):
            return cls(epsilon=float(value))
        raise NotImplementedError("only float stabilizers are supported by the HIP engine")


def _zero_params(zero_params) -> tuple:
    if zero_params is None:
        return ()
    if isinstance(zero_params, str):
        return (zero_params,)
    return tuple(zero_params)


class Hook:
    """Base of all rules (zennit.core.Hook).  The HIP plan executes the hooks it knows (the rule
    descriptors and ``SubspaceHook``); a subclass that overrides ``backward`` runs on the
    autograd slow path (``engine/hooks.py``), called as zennit calls it."""

    def __init__(self) -> None:
        self.stored_tensors = {}

    def backward(self, module, grad_input, grad_output):
        return grad_input

    def copy(self) -> "Hook":
        return self.__class__()

    def register(self, module):   # zennit API surface; nothing is attached here
        return None

    def remove(self) -> None:
        return None


class BasicHook(Hook):
    """Descriptor of a modified-gradient rule (zennit.core.BasicHook)."""

    kind: str = "basic"

    def __init__(self, zero_params=None) -> None:
        super().__init__()
        self.zero_params = _zero_params(zero_params)

    def copy(self) -> "BasicHook":
        import copy
        return copy.copy(self)

    def __repr__(self) -> str:
        fields = {k: v for k, v in self.__dict__.items() if k not in ("stored_tensors",)}
        return f"{type(self).__name__}({fields})"
