"""ORACLE — test infrastructure only. CPU (PyTorch fp32) restatement of the LRP path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module; the product (``drsa_audio_amd``) never does.

What it restates
----------------
* ``compute_relevances`` / ``lrp_output_modifier``  — reference ``cxai/xai/explain/attribute.py:70-160``
* ``SubspaceHook.backward``                         — reference ``cxai/xai/explain/attribute.py:42-60``
* ``HeatmapGenerator.generate_subspace_heatmaps`` +
  ``sort_subspaces``                                — reference ``cxai/xai/explain/explainer.py:68-176``
* ``get_class_composite`` (ε on (inv)projection)   — reference ``cxai/xai/explain/explainer.py:179-203``
* zennit 0.5.1 rules ``Epsilon/Gamma/WSquare/Flat/Pass`` (third-party, pinned in
  ``requirements.txt:23``, NOT present in the container) — restated from zennit's
  published rule definitions; see SURVEY.md Appendix A.  **Parity vs zennit itself is
  unpinned** (no zennit, no reference tests); the rule arithmetic is pinned only by
  the theory known-answer tests in ``tests/test_oracle_lrp.py``.

Rule arithmetic (z = f(x; W, b), Jᵀ_W g = input-gradient of f with weights W):
  stab_ε(t)  = t + ε·(sign(t) + [t == 0])
  Epsilon    : R_in = x ⊙ Jᵀ_W( R / stab_ε(z) )
  Gamma(γ)   : W± = W + γ·W.clamp(min/max=0) (bias likewise);
               z0 = f(x⁺;W⁺,b⁺), z1 = f(x⁻;W⁻,b⁻), z2 = f(x⁺;W⁻,b⁻), z3 = f(x⁻;W⁺,b⁺)
               g₊ = R·[z>0]/stab(z0+z1),  g₋ = R·[z<0]/stab(z2+z3)
               R_in = x⁺⊙Jᵀ_{W⁺}g₊ + x⁻⊙Jᵀ_{W⁻}g₊ + x⁺⊙Jᵀ_{W⁻}g₋ + x⁻⊙Jᵀ_{W⁺}g₋
  WSquare    : R_in = Jᵀ_{W²}( R / stab(f(1; W², b²)) )            (no x⊙)
  Flat       : as WSquare with W → 1, b → 0
  Pass       : R_in = R
Layers without a rule use their plain gradient (ReLU, MaxPool [first max], Dropout
(eval), BatchNorm (eval), flatten), exactly like zennit's Gradient attributor.

Two execution modes share that arithmetic:
* ``mode="analytic"`` — each rule evaluated with explicit conv/conv-transpose calls.
* ``mode="zennit"``   — each rule evaluated the way zennit's BasicHook does it
  (modified forwards + ``torch.autograd.grad``), and the heatmap generator replicates
  the batch K+1 times like ``explainer.py:92``.  This is the representative CPU
  baseline that ``bench.py`` times; tests check both modes agree.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

# ----------------------------------------------------------------------------
# rule specs (plain tuples so the oracle does not depend on the product's classes)
#   ("epsilon", eps) | ("gamma", gamma, eps) | ("wsquare", eps) | ("flat", eps)
#   ("pass",) | ("subspace", K)
# ----------------------------------------------------------------------------
RuleSpec = Tuple


def stabilize(t: torch.Tensor, eps: float) -> torch.Tensor:
    """zennit ``Stabilizer`` (clip=False, norm_scale=False): t + ε·(sign(t) + [t == 0])."""
    return t + ((t == 0.0).to(t) + t.sign()) * eps


@dataclass
class Layer:
    name: str
    module: nn.Module
    kind: str          # conv | linear | relu | maxpool | dropout | bn2d | bn1d | flatten | proj | filter | invproj


def _kind(m: nn.Module) -> str:
    cname = type(m).__name__
    if isinstance(m, nn.Conv2d):
        return "conv"
    if isinstance(m, nn.Linear):
        return "linear"
    if isinstance(m, nn.ReLU):
        return "relu"
    if isinstance(m, nn.MaxPool2d):
        return "maxpool"
    if isinstance(m, nn.Dropout):
        return "dropout"
    if isinstance(m, nn.BatchNorm2d):
        return "bn2d"
    if isinstance(m, nn.BatchNorm1d):
        return "bn1d"
    if cname == "Projection":
        return "proj"
    if cname == "SubspaceFilter":
        return "filter"
    if cname == "InvProjection":
        return "invproj"
    raise TypeError(f"oracle: unsupported module {cname}")


def sequential_layers(model: nn.Module) -> List[Layer]:
    """features.* -> flatten -> classifier.* (the reference's model contract)."""
    out: List[Layer] = []
    for n, m in model.features.named_children():
        out.append(Layer(f"features.{n}", m, _kind(m)))
    out.append(Layer("flatten", nn.Identity(), "flatten"))
    for n, m in model.classifier.named_children():
        out.append(Layer(f"classifier.{n}", m, _kind(m)))
    return out


def _layer_fwd(L: Layer, x: torch.Tensor) -> torch.Tensor:
    m = L.module
    if L.kind == "flatten":
        return x.reshape(x.size(0), -1)
    if L.kind == "dropout":
        return x
    return m(x)


# ----------------------------------------------------------------------------
# Jacobian-transpose products for the parametrised layers
# ----------------------------------------------------------------------------
def _pad(m: nn.Conv2d):
    if isinstance(m.padding, str):   # 'same' (odd kernels, stride 1)
        return tuple((k - 1) // 2 for k in m.kernel_size)
    return m.padding


def _conv(m: nn.Conv2d, x, w, b):
    return F.conv2d(x, w, b, stride=m.stride, padding=_pad(m), dilation=m.dilation, groups=m.groups)


def _conv_jt(m: nn.Conv2d, x_shape, w, g):
    return torch.nn.grad.conv2d_input(x_shape, w, g, stride=m.stride, padding=_pad(m),
                                      dilation=m.dilation, groups=m.groups)


def _aff(L: Layer, x, w, b):
    if L.kind == "conv":
        return _conv(L.module, x, w, b)
    return F.linear(x, w, b)


def _aff_jt(L: Layer, x_shape, w, g):
    if L.kind == "conv":
        return _conv_jt(L.module, x_shape, w, g)
    return g @ w


def _params(m):
    return m.weight.detach(), (m.bias.detach() if m.bias is not None else None)


def _mod(p, fn):
    return None if p is None else fn(p)


# ----------------------------------------------------------------------------
# analytic rules
# ----------------------------------------------------------------------------
def rule_backward_analytic(L: Layer, rule: RuleSpec, x: torch.Tensor, z: torch.Tensor,
                           R: torch.Tensor) -> torch.Tensor:
    kind = rule[0]
    if kind == "pass":
        return R
    if L.kind in ("proj", "invproj"):
        # only Epsilon is meaningful here (explainer.py:200,202); generic via autograd
        if kind != "epsilon":
            raise ValueError("oracle: only Epsilon on (inv)projection")
        xx = x.detach().requires_grad_(True)
        with torch.enable_grad():
            zz = L.module(xx)
            g, = torch.autograd.grad(zz, xx, R / stabilize(zz.detach(), rule[1]))
        return x * g
    w, b = _params(L.module)
    if kind == "epsilon":
        g = R / stabilize(z, rule[1])
        return x * _aff_jt(L, x.shape, w, g)
    if kind == "gamma":
        gam, eps = rule[1], rule[2]
        wp = w + gam * w.clamp(min=0)
        wn = w + gam * w.clamp(max=0)
        bp = _mod(b, lambda t: t + gam * t.clamp(min=0))
        bn = _mod(b, lambda t: t + gam * t.clamp(max=0))
        xp, xn = x.clamp(min=0), x.clamp(max=0)
        z0 = _aff(L, xp, wp, bp)
        z1 = _aff(L, xn, wn, bn)
        z2 = _aff(L, xp, wn, bn)
        z3 = _aff(L, xn, wp, bp)
        gpos = R * (z > 0) / stabilize(z0 + z1, eps)
        gneg = R * (z < 0) / stabilize(z2 + z3, eps)
        return (xp * _aff_jt(L, x.shape, wp, gpos) + xn * _aff_jt(L, x.shape, wn, gpos)
                + xp * _aff_jt(L, x.shape, wn, gneg) + xn * _aff_jt(L, x.shape, wp, gneg))
    if kind in ("wsquare", "flat"):
        eps = rule[1]
        if kind == "wsquare":
            w2, b2 = w * w, _mod(b, lambda t: t * t)
        else:
            w2, b2 = torch.ones_like(w), _mod(b, torch.zeros_like)
        den = _aff(L, torch.ones_like(x), w2, b2)
        return _aff_jt(L, x.shape, w2, R / stabilize(den, eps))
    raise ValueError(f"oracle: unknown rule {rule}")


# ----------------------------------------------------------------------------
# zennit-structured rules (modified forwards + autograd.grad), for the CPU baseline
# ----------------------------------------------------------------------------
def rule_backward_zennit(L: Layer, rule: RuleSpec, x: torch.Tensor, z: torch.Tensor,
                         R: torch.Tensor) -> torch.Tensor:
    kind = rule[0]
    if kind == "pass" or L.kind in ("proj", "invproj"):
        return rule_backward_analytic(L, rule, x, z, R)
    w, b = _params(L.module)

    def run(inputs, params):
        ins = [i.detach().requires_grad_(True) for i in inputs]
        with torch.enable_grad():
            outs = [_aff(L, i, pw, pb) for i, (pw, pb) in zip(ins, params)]
        return ins, outs

    if kind == "epsilon":
        ins, outs = run([x], [(w, b)])
        g, = torch.autograd.grad(outs, ins, [R / stabilize(outs[0].detach(), rule[1])])
        return ins[0].detach() * g
    if kind == "gamma":
        gam, eps = rule[1], rule[2]
        wp = w + gam * w.clamp(min=0)
        wn = w + gam * w.clamp(max=0)
        bp = _mod(b, lambda t: t + gam * t.clamp(min=0))
        bn = _mod(b, lambda t: t + gam * t.clamp(max=0))
        inputs = [x.clamp(min=0), x.clamp(max=0), x.clamp(min=0), x.clamp(max=0), x]
        params = [(wp, bp), (wn, bn), (wn, bn), (wp, bp), (w, b)]
        ins, outs = run(inputs, params)
        o = [t.detach() for t in outs]
        gpos = R * (o[4] > 0) / stabilize(o[0] + o[1], eps)
        gneg = R * (o[4] < 0) / stabilize(o[2] + o[3], eps)
        grads = torch.autograd.grad(outs[:4], ins[:4], [gpos, gpos, gneg, gneg])
        return sum(i.detach() * g for i, g in zip(ins[:4], grads))
    if kind in ("wsquare", "flat"):
        eps = rule[1]
        if kind == "wsquare":
            w2, b2 = w * w, _mod(b, lambda t: t * t)
        else:
            w2, b2 = torch.ones_like(w), _mod(b, torch.zeros_like)
        ins, outs = run([torch.ones_like(x)], [(w2, b2)])
        g, = torch.autograd.grad(outs, ins, [R / stabilize(outs[0].detach(), eps)])
        return g
    raise ValueError(f"oracle: unknown rule {rule}")


# ----------------------------------------------------------------------------
# plain-gradient layers
# ----------------------------------------------------------------------------
def _plain_backward(L: Layer, x: torch.Tensor, z: torch.Tensor, R: torch.Tensor, aux) -> torch.Tensor:
    if L.kind == "relu":
        return torch.where(z > 0, R, torch.zeros_like(R))
    if L.kind == "maxpool":
        m = L.module
        return F.max_unpool2d(R, aux, m.kernel_size, m.stride, m.padding, output_size=x.shape[-2:])
    if L.kind in ("dropout",):
        return R
    if L.kind == "flatten":
        return R.reshape(x.shape)
    if L.kind in ("bn2d", "bn1d", "conv", "linear", "proj", "invproj"):
        xx = x.detach().requires_grad_(True)
        with torch.enable_grad():
            zz = _layer_fwd(L, xx)
            g, = torch.autograd.grad(zz, xx, R)
        return g
    if L.kind == "filter":
        return R
    raise TypeError(L.kind)


def subspace_mask(R: torch.Tensor, K: int) -> torch.Tensor:
    """SubspaceHook.backward (attribute.py:53-60): clone 0 unmasked, clone k keeps block k-1."""
    b, n, c, dk = R.shape
    Rv = R.reshape(-1, K + 1, n, c, dk).clone()
    Rv[:, 1:] *= torch.eye(K, dtype=R.dtype)[None, :, None, :, None]
    return Rv.reshape(b, n, c, dk)


# ----------------------------------------------------------------------------
# forward + modified backward
# ----------------------------------------------------------------------------
def output_seed(logits: torch.Tensor, class_idx=None, num_classes=None,
                one_hot_encoded: bool = False) -> torch.Tensor:
    """lrp_output_modifier (attribute.py:111-160), evaluated on detached logits."""
    if class_idx is not None:
        mask = torch.zeros_like(logits)
        mask[..., class_idx] = 1
    elif num_classes is not None:
        mask = torch.repeat_interleave(torch.eye(num_classes).to(logits),
                                       logits.size(0) // num_classes, dim=0)
    else:
        raise ValueError("Provide either class_idx to attribute or num_classes")
    return mask if one_hot_encoded else logits * mask


@torch.no_grad()
def lrp(model: nn.Module, rules: Dict[str, RuleSpec], x: torch.Tensor, class_idx=None,
        num_classes=None, one_hot_encoded=False, mode: str = "analytic",
        capture: Optional[str] = None):
    """Returns (logits, R_input[, (act, rel) at layer ``capture``])."""
    layers = sequential_layers(model)
    acts: List[Tuple[torch.Tensor, torch.Tensor, object]] = []
    h = x.detach().to(torch.float32)
    for L in layers:
        aux = None
        if L.kind == "maxpool":
            m = L.module
            out, aux = F.max_pool2d(h, m.kernel_size, m.stride, m.padding, m.dilation,
                                    m.ceil_mode, return_indices=True)
        else:
            out = _layer_fwd(L, h)
        acts.append((h, out, aux))
        h = out
    logits = h
    R = output_seed(logits, class_idx, num_classes, one_hot_encoded)
    rb = rule_backward_zennit if mode == "zennit" else rule_backward_analytic
    captured = None
    for L, (xin, zout, aux) in zip(reversed(layers), reversed(acts)):
        if capture is not None and L.name == capture:
            captured = (zout.clone(), R.clone())
        rule = rules.get(L.name)
        if rule is not None and rule[0] == "subspace":
            R = subspace_mask(R, rule[1])
        elif rule is not None:
            R = rb(L, rule, xin, zout, R)
        else:
            R = _plain_backward(L, xin, zout, R, aux)
    if capture is not None:
        return logits, R, captured
    return logits, R


def class_composite_rules(name_map: Dict[str, RuleSpec], K: int) -> Dict[str, RuleSpec]:
    """get_class_composite (explainer.py:198-203): ε(1e-6) on (inv)projection + subspace mask."""
    r = dict(name_map)
    r["features.invprojection"] = ("epsilon", 1e-6)
    r["features.subspacefilter"] = ("subspace", K)
    r["features.projection"] = ("epsilon", 1e-6)
    return r


def sort_subspaces(sub: np.ndarray):
    """explainer.py:151-176 with batch dims kept (defect D7: B=1 must not squeeze)."""
    rel = sub.sum(axis=(-2, -1)).reshape(sub.shape[0], sub.shape[1])
    mask = np.argsort(rel, axis=-1)[..., ::-1]
    ar = np.arange(sub.shape[0])[:, None]
    return sub[ar, mask], rel[ar, mask], mask


@torch.no_grad()
def subspace_heatmaps(proj_model: nn.Module, name_map: Dict[str, RuleSpec], K: int,
                      x: torch.Tensor, class_idx: int, one_hot_encoded=False,
                      mode: str = "analytic") -> Dict[str, np.ndarray]:
    """HeatmapGenerator.generate_subspace_heatmaps (explainer.py:87-123) on the CPU."""
    rules = class_composite_rules(name_map, K)
    xr = x.repeat_interleave(K + 1, dim=0)
    _, R = lrp(proj_model, rules, xr, class_idx=class_idx, one_hot_encoded=one_hot_encoded, mode=mode)
    H, W = R.shape[-2:]
    hm = R.reshape(-1, K + 1, H, W).numpy()
    std, sub = hm[:, 0:1], hm[:, 1:]
    sub_s, rel_s, mask = sort_subspaces(sub)
    return {
        "standard_heatmaps": std,
        "standard_relevance": std.sum(axis=(-2, -1)).flatten(),
        "subspace_heatmaps": sub_s,
        "subspace_relevances": rel_s,
        "mask": mask,
    }


def compute_subspace_relevances(act, ctx, U, n_concepts=4):
    """explainer.py:206-242."""
    act = act if act.dim() == 3 else act.unsqueeze(0)
    ctx = ctx if ctx.dim() == 3 else ctx.unsqueeze(0)
    b = act.size(0)
    dk = U.size(0) // n_concepts
    x = (act @ U) * (ctx @ U)
    x = x.transpose(-2, -1).contiguous().view(b, n_concepts, -1, dk)
    return x.sum(-1).sum(-1)
