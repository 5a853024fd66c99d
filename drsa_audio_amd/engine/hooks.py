"""Slow path for composites that map a module to a ``Hook`` subclass with its own ``backward``
("``Hook`` subclasses with a custom ``backward`` must still work via a slow
path (autograd hook fallback)"; reference hook contract: cxai/xai/explain/attribute.py:12-67,
``backward(module, grad_input, grad_output) -> tuple`` replacing the module's input gradient).

A user-written hook is arbitrary Python on torch tensors, so no compiled plan can execute it.
``HookedAutograd`` therefore runs the model's own forward on the GPU under autograd, with every
mapped module hooked the way zennit attaches its hooks (forward hook storing the input, full
backward hook replacing the input gradient):

* a custom hook: its ``backward`` is called as is;
* the built-in rule descriptors (Epsilon, Gamma, WSquare, Flat, ZPlus, AlphaBeta, Norm, Pass):
  the modified-gradient arithmetic of zennit 0.5.1's BasicHook for that rule, on the stored
  input (the same arithmetic the HIP plan fuses into its kernels);
* unmapped modules: the plain gradient.

The heatmap split / sum / sort of ``subspace_heatmaps`` still runs on the HIP kernel
(``drsa_amd_heatmap_sort``).  Composites without custom hooks never come here (``get_engine``
compiles the HIP plan for them), and this path, like the plan, refuses host tensors.
"""
from __future__ import annotations

import copy
import weakref
from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _capi
from ..zennit.canonizers import SequentialMergeBatchNorm
from ..zennit.core import Hook


def _is_subspace_hook(rule) -> bool:
    t = type(rule)
    return t.__name__ == "SubspaceHook" and t.__module__.endswith("xai.explain.attribute")


def is_custom_hook(rule) -> bool:
    """A rule object the HIP plan cannot compile: a Hook (or duck-typed hook) whose class
    defines its own ``backward``, other than the built-in descriptors and ``SubspaceHook``."""
    if rule is None or _is_subspace_hook(rule):
        return False
    bw = getattr(type(rule), "backward", None)
    return callable(bw) and bw is not Hook.backward


def has_custom_hooks(rules: Dict[str, object]) -> bool:
    return any(is_custom_hook(r) for r in rules.values())


def _stab(t: torch.Tensor, eps: float) -> torch.Tensor:
    # zennit Stabilizer: t + eps * (sign(t) + [t == 0])
    return t + eps * ((t >= 0).to(t.dtype) * 2 - 1)


def _aff(m: nn.Module, x, w, b):
    if isinstance(m, nn.Conv2d):
        return F.conv2d(x, w, b, m.stride, m.padding, m.dilation, m.groups)
    return F.linear(x, w, b)


def _grad(fn, xs, gs):
    """sum_i  x_i (.) J^T_{fn_i}(g_i), every fn_i evaluated at its own x_i (zennit reducer)."""
    ins = [x.detach().requires_grad_(True) for x in xs]
    with torch.enable_grad():
        outs = [f(i) for f, i in zip(fn, ins)]
    grads = torch.autograd.grad(outs, ins, gs)
    return [i.detach() * g for i, g in zip(ins, grads)]


def rule_relevance(rule, m: nn.Module, x: torch.Tensor, R: torch.Tensor) -> torch.Tensor:
    """R_in of a built-in rule descriptor on module ``m`` with input ``x`` and output relevance R."""
    kind = rule.kind
    if kind == "pass":
        return R
    zp = getattr(rule, "zero_params", ())
    if not isinstance(m, (nn.Conv2d, nn.Linear)):
        if kind not in ("epsilon", "norm"):
            raise NotImplementedError(f"{type(rule).__name__} needs a Conv2d/Linear module (got {type(m).__name__})")
        eps = rule.epsilon if kind == "epsilon" else rule.stabilizer
        # m.forward, not m(...): the module carries this path's hooks, and calling it would
        # re-enter its own backward hook
        with torch.no_grad():
            z = m.forward(x)
        return _grad([m.forward], [x], [R / _stab(z, eps)])[0]
    w = m.weight.detach()
    b = None if m.bias is None or "bias" in zp else m.bias.detach()
    if "weight" in zp:
        w = torch.zeros_like(w)
    mod = lambda p, f: None if p is None else f(p)
    with torch.no_grad():
        if kind in ("epsilon", "norm"):
            eps = rule.epsilon if kind == "epsilon" else rule.stabilizer
            g = R / _stab(_aff(m, x, w, b), eps)
            return _grad([lambda t: _aff(m, t, w, b)], [x], [g])[0]
        if kind in ("wsquare", "flat"):
            if kind == "wsquare":
                w2, b2 = w * w, mod(b, lambda t: t * t)
            else:
                w2, b2 = torch.ones_like(w), mod(b, torch.zeros_like)
            one = torch.ones_like(x)
            g = R / _stab(_aff(m, one, w2, b2), rule.stabilizer)
            ins = one.requires_grad_(True)
            with torch.enable_grad():
                out = _aff(m, ins, w2, b2)
            return torch.autograd.grad(out, ins, g)[0]
        xp, xn = x.clamp(min=0), x.clamp(max=0)
        if kind == "gamma":
            gam = rule.gamma
            wp, wn = w + gam * w.clamp(min=0), w + gam * w.clamp(max=0)
            bp, bn = mod(b, lambda t: t + gam * t.clamp(min=0)), mod(b, lambda t: t + gam * t.clamp(max=0))
            z = _aff(m, x, w, b)
            b0 = mod(b, torch.zeros_like)     # zennit 0.5.1: the x- terms carry no bias (zero_bias)
            den_p = _aff(m, xp, wp, bp) + _aff(m, xn, wn, b0)
            den_n = _aff(m, xp, wn, bn) + _aff(m, xn, wp, b0)
            gp = R * (z > 0) / _stab(den_p, rule.stabilizer)
            gn = R * (z < 0) / _stab(den_n, rule.stabilizer)
            fs = [lambda t: _aff(m, t, wp, bp), lambda t: _aff(m, t, wn, b0),
                  lambda t: _aff(m, t, wn, bn), lambda t: _aff(m, t, wp, b0)]
            return sum(_grad(fs, [xp, xn, xp, xn], [gp, gp, gn, gn]))
        wp, wn = w.clamp(min=0), w.clamp(max=0)
        bp, bn, b0 = mod(b, lambda t: t.clamp(min=0)), mod(b, lambda t: t.clamp(max=0)), mod(b, torch.zeros_like)
        if kind == "zplus":
            g = R / _stab(_aff(m, xp, wp, bp) + _aff(m, xn, wn, b0), rule.stabilizer)
            return sum(_grad([lambda t: _aff(m, t, wp, bp), lambda t: _aff(m, t, wn, b0)], [xp, xn], [g, g]))
        if kind == "alphabeta":
            gp = R / _stab(_aff(m, xp, wp, bp) + _aff(m, xn, wn, b0), rule.stabilizer)
            gn = R / _stab(_aff(m, xp, wn, bn) + _aff(m, xn, wp, b0), rule.stabilizer)
            pos = _grad([lambda t: _aff(m, t, wp, bp), lambda t: _aff(m, t, wn, b0)], [xp, xn], [gp, gp])
            neg = _grad([lambda t: _aff(m, t, wn, bn), lambda t: _aff(m, t, wp, b0)], [xp, xn], [gn, gn])
            return rule.alpha * (pos[0] + pos[1]) - rule.beta * (neg[0] + neg[1])
    raise NotImplementedError(f"rule {type(rule).__name__} is not supported")


def _merge_bn(model: nn.Module) -> nn.Module:
    """Private copy with every BatchNorm that follows a Conv2d/Linear folded into it (zennit
    SequentialMergeBatchNorm); the folded BatchNorm becomes the identity."""
    model = copy.deepcopy(model)
    for seq in model.modules():
        if not isinstance(seq, nn.Sequential):
            continue
        names = list(seq._modules.keys())
        for a, bnm in zip(names, names[1:]):
            prev, bn = seq._modules[a], seq._modules[bnm]
            if isinstance(prev, (nn.Conv2d, nn.Linear)) and isinstance(bn, (nn.BatchNorm1d, nn.BatchNorm2d)):
                w, b = SequentialMergeBatchNorm.fold(prev.weight.data, None if prev.bias is None else prev.bias.data, bn)
                prev.weight.data = w
                if prev.bias is None:
                    prev.bias = nn.Parameter(b)
                else:
                    prev.bias.data = b
                seq._modules[bnm] = nn.Identity()
    return model


class HookedAutograd:
    """Engine-compatible object (``forward`` / ``backward`` / ``subspace_heatmaps``) for
    composites with custom hooks; see the module docstring."""

    def __init__(self, model: nn.Module, composite):
        p0 = next(model.parameters())
        if p0.device.type != "cuda":
            raise _capi.DrsaAmdError("the LRP engine runs on the GPU only; move the model to a HIP device")
        _capi.load()
        self.device = p0.device
        self.rules = composite.rules(model) if composite is not None else {}
        merge = any(isinstance(c, SequentialMergeBatchNorm) for c in getattr(composite, "canonizers", []))
        # the BN-merged private copy, or a weak reference to the user's model (the engine cache
        # holds no strong reference to the model, engine/__init__.py)
        self._net = _merge_bn(model) if merge else None
        self._model_ref = weakref.ref(model)
        self._x = None
        self._out = None

    @property
    def net(self) -> nn.Module:
        return self._net if self._net is not None else self._model_ref()

    def _hooks(self):
        handles, store = [], {}
        mods = dict(self.net.named_modules())
        for name, rule in self.rules.items():
            m = mods.get(name)
            if m is None:
                continue

            def fwd(mod, inp, out, name=name):
                store[name] = inp[0].detach()

            def bwd(mod, grad_input, grad_output, name=name, rule=rule):
                if is_custom_hook(rule) or _is_subspace_hook(rule):
                    res = rule.backward(mod, grad_input, grad_output)
                    return tuple(res) if res is not None else None
                R_in = rule_relevance(rule, mod, store[name], grad_output[0])
                return tuple(R_in if (g is not None and g.shape == R_in.shape) else g for g in grad_input)

            handles.append(m.register_forward_hook(fwd))
            handles.append(m.register_full_backward_hook(bwd))
        return handles

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.device.type != "cuda":
            raise _capi.DrsaAmdError("input must be a GPU tensor")
        self._remove()   # a forward without its backward must not leave its hooks attached
        self._x = x.detach().to(self.device, torch.float32).requires_grad_(True)
        self._handles = self._hooks()
        try:
            with torch.enable_grad():
                self._out = self.net(self._x)
        except Exception:
            self._remove()
            raise
        return self._out.detach()

    def _remove(self):
        for h in getattr(self, "_handles", []):
            h.remove()
        self._handles = []

    def backward(self, seed: Optional[torch.Tensor] = None, cls: Optional[torch.Tensor] = None,
                 one_hot: bool = False) -> torch.Tensor:
        if self._out is None:
            raise RuntimeError("backward() before forward()")
        try:
            if seed is None:
                out = self._out.detach()
                mask = torch.zeros_like(out)
                mask[torch.arange(out.size(0), device=out.device), cls.long()] = 1
                seed = mask if one_hot else out * mask
            R, = torch.autograd.grad(self._out, self._x, seed.to(self._out))
        finally:
            self._remove()
            self._out = None
        return R.detach()

    @torch.no_grad()
    def subspace_heatmaps(self, x: torch.Tensor, class_idx=None, cls: Optional[torch.Tensor] = None,
                          one_hot: bool = False, standard: str = "clone") -> dict:
        """The reference's clone semantics literally (explainer.py:92-104): K+1 copies of every
        sample through the hooked model, then split / sum / sort on the HIP kernel.  The standard
        heatmap is always clone 0 here (``standard`` is accepted for the engine's signature: a
        user hook need not be linear in the relevance, so the sum form is not used)."""
        K = next((r.num_concepts for r in self.rules.values() if _is_subspace_hook(r) or
                  hasattr(r, "num_concepts")), None)
        if K is None:
            raise ValueError("subspace heatmaps need a SubspaceHook in the composite")
        B = x.size(0)
        if cls is None:
            cls = torch.full((B,), int(class_idx), dtype=torch.int32, device=self.device)
        xr = x.repeat_interleave(K + 1, dim=0)
        self.forward(xr)
        hm = self.backward(cls=cls.repeat_interleave(K + 1), one_hot=one_hot).contiguous()
        H, W = hm.shape[-2:]
        out = {
            "standard_heatmaps": torch.empty(B, 1, H, W, device=self.device),
            "standard_relevance": torch.empty(B, device=self.device),
            "subspace_heatmaps": torch.empty(B, K, H, W, device=self.device),
            "subspace_relevances": torch.empty(B, K, device=self.device),
            "mask": torch.empty(B, K, dtype=torch.int64, device=self.device),
        }
        _capi.call("drsa_amd_heatmap_sort", hm.data_ptr(), B, K, H * W, 0, out["standard_heatmaps"].data_ptr(),
                   out["standard_relevance"].data_ptr(), out["subspace_heatmaps"].data_ptr(),
                   out["subspace_relevances"].data_ptr(), out["mask"].data_ptr(), _capi.stream_ptr(self.device))
        return out

    def release(self) -> None:
        self._remove()
        self._x = self._out = None
