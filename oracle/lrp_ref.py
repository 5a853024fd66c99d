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
               z0 = f(x⁺;W⁺,b⁺), z1 = f(x⁻;W⁻,0), z2 = f(x⁺;W⁻,b⁻), z3 = f(x⁻;W⁺,0)
               (zennit 0.5.1 zeroes the bias of the x⁻ terms' GammaMod with zero_bias(), as
               for ZPlus / AlphaBeta: each denominator holds the bias once)
               g₊ = R·[z>0]/stab(z0+z1),  g₋ = R·[z<0]/stab(z2+z3)
               R_in = x⁺⊙Jᵀ_{W⁺}g₊ + x⁻⊙Jᵀ_{W⁻}g₊ + x⁺⊙Jᵀ_{W⁻}g₋ + x⁻⊙Jᵀ_{W⁺}g₋
  WSquare    : R_in = Jᵀ_{W²}( R / stab(f(1; W², b²)) )            (no x⊙)
  Flat       : as WSquare with W → 1, b → 0
  Pass       : R_in = R
Layers without a rule use their plain gradient (ReLU, MaxPool [first max], Dropout
(eval), BatchNorm (eval), flatten), exactly like zennit's Gradient attributor.

Five execution modes share that arithmetic:
* ``mode="analytic"`` — each rule evaluated with explicit conv/conv-transpose calls.
* ``mode="zennit"``   — each rule evaluated the way zennit's BasicHook does it
  (modified forwards + ``torch.autograd.grad``), and the heatmap generator replicates
  the batch K+1 times like ``explainer.py:92``.  This is the representative CPU
  baseline that ``bench.py`` times; tests check both modes agree.
* ``mode="exact"``    — the analytic structure with every dot product computed as one
  sequential fp32 fma chain in a pinned order (``oracle/lrp_exact.c``): channel-major /
  tap-minor for convolutions, bias added last.  This is the order the HIP kernels
  accumulate in (f32 MFMA is an exact k-ordered fma chain), so this mode is the
  bit-exact parity oracle.
* ``mode="f64"``      — the analytic structure in float64: the accuracy anchor.  The parity
  tests bound every fp32 path's distance to it (tests/test_lrp_gpu.py, test_oracle_lrp.py).  The reference path is ill-conditioned with respect to
  rounding (the ProjectionModel's a' = (aU)Uᵀ differs from a at rounding level and the
  ε = 1e-6 stabilisers amplify that at dead ReLU channels: correctly rounded projections
  move subspace relevances by up to ~6 %), so only a pinned order can pin it.
* ``mode="bf16"``     — float64 with every conv's input and weights rounded to bf16 (class
  ``Bf16Ops``): the definition of the product's bf16 plan (no reference bf16 path).
* ``mode="bf16bwd"``  — ``bf16`` plus the transposed convs' g rounded to bf16 for layers with
  more than one input channel (``Bf16BwdOps``): the plan's ``bf16_backward`` option.
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
    if isinstance(m, (nn.Dropout, nn.Identity)):
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


@torch.no_grad()
def merge_batch_norm(model: nn.Module) -> nn.Module:
    """zennit 0.5.1 ``SequentialMergeBatchNorm`` (canonizers.py; used at getdrsadata.py:81,113):
    every BatchNorm directly after a Conv2d/Linear is merged into it,
    w' = w * (gamma / (var + eps) ** .5), b' = (b - mean) * (gamma / (var + eps) ** .5) + beta,
    and the BatchNorm becomes the identity.  Returns a merged deep copy (CPU)."""
    import copy
    m = copy.deepcopy(model).cpu()
    for seq in (m.features, m.classifier):
        kids = list(seq.children())
        for a, b in zip(kids[:-1], kids[1:]):
            if isinstance(b, (nn.BatchNorm1d, nn.BatchNorm2d)) and isinstance(a, (nn.Conv2d, nn.Linear)):
                scale = b.weight / (b.running_var + b.eps) ** .5
                shape = (-1,) + (1,) * (a.weight.dim() - 1)
                a.weight.data = a.weight.data * scale.reshape(shape)
                b0 = a.bias.data if a.bias is not None else torch.zeros_like(b.running_mean)
                if a.bias is None:
                    a.bias = nn.Parameter(b0.clone())
                a.bias.data = (b0 - b.running_mean) * scale + b.bias
        # the merged BatchNorm is the identity (zennit sets mean 0, var 1, eps 0; torch >= 2.x
        # rejects eps = 0, so the module is replaced by nn.Identity instead)
        for name, b in list(seq.named_children()):
            if isinstance(b, (nn.BatchNorm1d, nn.BatchNorm2d)):
                setattr(seq, name, nn.Identity())
    return m


def sequential_layers(model: nn.Module) -> List[Layer]:
    """features.* -> flatten -> classifier.* (the reference's model contract)."""
    out: List[Layer] = []
    for n, m in model.features.named_children():
        out.append(Layer(f"features.{n}", m, _kind(m)))
    out.append(Layer("flatten", nn.Identity(), "flatten"))
    for n, m in model.classifier.named_children():
        out.append(Layer(f"classifier.{n}", m, _kind(m)))
    return out


def _layer_fwd(L: Layer, x: torch.Tensor, ops=None) -> torch.Tensor:
    m = L.module
    if L.kind == "flatten":
        return x.reshape(x.size(0), -1)
    if L.kind == "dropout":
        return x
    if ops is not None and L.kind == "conv":
        return ops.conv(m, x, m.weight.detach(), None if m.bias is None else m.bias.detach())
    if ops is not None and L.kind == "linear":
        return ops.linear(x, m.weight.detach(), None if m.bias is None else m.bias.detach())
    if ops is not None and L.kind in ("proj", "invproj"):
        return _proj_fwd(L, x, ops)
    return m(x)


# ----------------------------------------------------------------------------
# primitive ops: torch (oneDNN order) or exact (pinned fma order, oracle/lrp_exact.c)
# ----------------------------------------------------------------------------
def _pad(m: nn.Conv2d):
    if isinstance(m.padding, str):   # 'same' (odd kernels, stride 1)
        return tuple((k - 1) // 2 for k in m.kernel_size)
    return m.padding


class TorchOps:
    name = "torch"

    @staticmethod
    def conv(m, x, w, b):
        return F.conv2d(x, w, b, stride=m.stride, padding=_pad(m), dilation=m.dilation, groups=m.groups)

    @staticmethod
    def conv_t(m, x_shape, w, g):
        return torch.nn.grad.conv2d_input(x_shape, w, g, stride=m.stride, padding=_pad(m),
                                          dilation=m.dilation, groups=m.groups)

    @staticmethod
    def linear(x, w, b):
        return F.linear(x, w, b)

    @staticmethod
    def linear_t(g, w):
        return g @ w

    @staticmethod
    def matmul(a, b):
        return a @ b

    @staticmethod
    def plane_sum(hm: np.ndarray) -> np.ndarray:
        return hm.sum(axis=(-2, -1))


class ExactOps:
    """Pinned-order primitives (each output one k-ordered fp32 fma chain; oracle/lrp_exact.c)."""
    name = "exact"
    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            import ctypes, os
            path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "liblrp_exact.so")
            if not os.path.exists(path):
                import subprocess
                subprocess.run(["make", "-C", os.path.dirname(path).rsplit("/lib", 1)[0]], check=True,
                               capture_output=True)
            L = ctypes.CDLL(path)
            P, I = ctypes.c_void_p, ctypes.c_int
            L.conv2d_exact.argtypes = [P, P, P, P, I, I, I, I, I]
            L.conv_transpose_exact.argtypes = [P, P, P, I, I, I, I, I]
            L.linear_exact.argtypes = [P, P, P, P, I, I, I]
            L.matmul_exact.argtypes = [P, P, P, I, I, I]
            cls._lib = L
        return cls._lib

    @staticmethod
    def _c(t):
        return t.detach().to(torch.float32).contiguous()

    @classmethod
    def conv(cls, m, x, w, b):
        if tuple(m.kernel_size) != (3, 3) or tuple(m.stride) != (1, 1) or tuple(_pad(m)) != (1, 1):
            raise NotImplementedError("exact ops: 3x3 same convs only")
        x, w = cls._c(x), cls._c(w)
        b = None if b is None else cls._c(b)
        B, Cin, H, W = x.shape
        out = torch.empty(B, w.size(0), H, W)
        cls.lib().conv2d_exact(x.data_ptr(), w.data_ptr(), None if b is None else b.data_ptr(), out.data_ptr(),
                               B, Cin, w.size(0), H, W)
        return out

    @classmethod
    def conv_t(cls, m, x_shape, w, g):
        g, w = cls._c(g), cls._c(w)
        B, Cout, H, W = g.shape
        out = torch.empty(B, w.size(1), H, W)
        cls.lib().conv_transpose_exact(g.data_ptr(), w.data_ptr(), out.data_ptr(), B, Cout, w.size(1), H, W)
        return out

    @classmethod
    def linear(cls, x, w, b):
        x, w = cls._c(x), cls._c(w)
        b = None if b is None else cls._c(b)
        out = torch.empty(x.size(0), w.size(0))
        cls.lib().linear_exact(x.data_ptr(), w.data_ptr(), None if b is None else b.data_ptr(), out.data_ptr(),
                               x.size(0), w.size(0), x.size(1))
        return out

    @classmethod
    def linear_t(cls, g, w):
        return cls.matmul(g, w)

    @classmethod
    def matmul(cls, a, b):
        shp = a.shape
        a2 = cls._c(a.reshape(-1, shp[-1]))
        b = cls._c(b)
        out = torch.empty(a2.size(0), b.size(1))
        cls.lib().matmul_exact(a2.data_ptr(), b.data_ptr(), out.data_ptr(), a2.size(0), b.size(1), a2.size(1))
        return out.reshape(*shp[:-1], b.size(1))

    @classmethod
    def inv_projection(cls, L, h, a_map):
        """a' = h U^T evaluated as a + a (U U^T - I): the product's projection kernels'
        order.  P = U U^T - I is formed in float64 (k ascending) and rounded once, so a' is
        accurate to its own rounding where a = 0 (dead ReLU channels), where the d-term chain
        h U^T leaves O(1e-8) noise that Epsilon(1e-6) amplifies (D13)."""
        m = L.module
        P = proj_residual(m.U_inv.t())
        b, d = a_map.size(0), a_map.size(1)
        av = cls._c(a_map).reshape(b, d, -1).transpose(1, 2)
        delta = cls.matmul(av, P)
        return (av + delta).transpose(1, 2).reshape(a_map.shape).contiguous()

    @classmethod
    def plane_sum(cls, hm: np.ndarray) -> np.ndarray:
        """The reference's own numpy float32 sum over (H, W) (explainer.py:120, :161): 0 + numpy's
        pairwise summation, which the heatmap_sort kernels reproduce bit for bit."""
        return np.asarray(hm, dtype=np.float32).sum(axis=(-2, -1))


def proj_residual(U: torch.Tensor) -> torch.Tensor:
    """fl32(U U^T - I) with each entry one float64 fma chain over k ascending, then minus the
    identity, rounded once (drsa_amd_projection_residual)."""
    Ud = U.detach().double()
    d = Ud.size(0)
    P = torch.zeros(d, d, dtype=torch.float64)
    for k in range(d):                       # k-ascending accumulation, as the kernel
        P += Ud[:, k:k + 1] * Ud[:, k:k + 1].t()
    return (P - torch.eye(d, dtype=torch.float64)).float()


def _bf16r(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(t.dtype)


class Bf16Ops(TorchOps):
    """The bf16 plan's arithmetic (the reference has no bf16 path, so this is the
    definition the product's bf16 mode is checked against): every conv rounds its input and its
    (rule-modified) weights to bf16, in both directions, and accumulates in float64 here; biases,
    dense layers, divisions and products with the activations stay at full precision.  The
    ProjectionModel GEMMs run as in the fp32 plan, in the kernels' pinned fp32 order (ExactOps):
    the inverse projection's eps = 1e-6 division amplifies any other rounding at dead channels."""
    name = "bf16"

    @staticmethod
    def conv(m, x, w, b):
        return TorchOps.conv(m, _bf16r(x), _bf16r(w), b)

    @staticmethod
    def conv_t(m, x_shape, w, g):
        return TorchOps.conv_t(m, x_shape, _bf16r(w), g)

    @staticmethod
    def matmul(a, b):
        return ExactOps.matmul(a, b).to(a.dtype)

    @staticmethod
    def inv_projection(L, h, a_map):
        return ExactOps.inv_projection(L, h, a_map).to(a_map.dtype)


class Bf16BwdOps(Bf16Ops):
    """Bf16Ops plus the bf16 relevance backward (engine option bf16_backward,
    drsa_amd_conv_bwd_bf16): every transposed conv of a layer with more than one input channel
    also rounds its input g (the quotient R / stab(den), after the pool backward) to bf16; the
    first layer (one input channel) keeps a full-precision g, as the product's fp32 kernel does."""
    name = "bf16bwd"

    @staticmethod
    def conv_t(m, x_shape, w, g):
        gi = _bf16r(g) if m.in_channels > 1 else g
        return TorchOps.conv_t(m, x_shape, _bf16r(w), gi)


# "f64": the analytic structure evaluated in float64 (model and input promoted): the accuracy
# anchor that fp32 implementations (the reference's own path, the HIP kernels) are measured against.
# "bf16": the same in float64 with Bf16Ops (input rounded to bf16 first).
OPS = {"analytic": TorchOps, "zennit": TorchOps, "exact": ExactOps, "f64": TorchOps, "bf16": Bf16Ops,
       "bf16bwd": Bf16BwdOps}


def _aff(L: Layer, x, w, b, ops=TorchOps):
    if L.kind == "conv":
        return ops.conv(L.module, x, w, b)
    return ops.linear(x, w, b)


def _aff_jt(L: Layer, x_shape, w, g, ops=TorchOps):
    if L.kind == "conv":
        return ops.conv_t(L.module, x_shape, w, g)
    return ops.linear_t(g, w)


def _params(m):
    return m.weight.detach(), (m.bias.detach() if m.bias is not None else None)


def _mod(p, fn):
    return None if p is None else fn(p)


def _proj_fwd(L: Layer, x, ops):
    """Projection / InvProjection forward through the given matmul (modify_model.py:89-123)."""
    m = L.module
    if L.kind == "proj":
        b, d = x.size(0), x.size(1)
        vecs = x.reshape(b, d, -1).transpose(1, 2)
        h = ops.matmul(vecs, m.U.to(x.dtype))
        return h.reshape(b, vecs.size(1), m.num_concepts, m.d_k)
    b, n = x.size(0), x.size(1)
    side = int(round(n ** 0.5))
    a = ops.matmul(x.reshape(b, n, m.d), m.U_inv.to(x.dtype).contiguous())
    return a.transpose(1, 2).reshape(b, m.d, side, side).contiguous()


def _proj_jt(L: Layer, x, g, ops):
    """Input-gradient of (inv)projection applied to g (linear maps, explicit)."""
    m = L.module
    if L.kind == "proj":        # h = a_vec U  ->  J^T g = g_vec U^T (back to [b, d, H, W])
        b, n = g.size(0), g.size(1)
        t = ops.matmul(g.reshape(b, n, -1), m.U.to(g.dtype).t().contiguous())
        return t.transpose(1, 2).reshape(x.shape)
    b, d = g.size(0), g.size(1)     # a' = h U^T  ->  J^T g = g_vec U
    gv = g.reshape(b, d, -1).transpose(1, 2)
    return ops.matmul(gv, m.U_inv.to(g.dtype).t().contiguous()).reshape(x.shape)


# ----------------------------------------------------------------------------
# analytic rules
# ----------------------------------------------------------------------------
def rule_backward_analytic(L: Layer, rule: RuleSpec, x: torch.Tensor, z: torch.Tensor,
                           R: torch.Tensor, ops=TorchOps) -> torch.Tensor:
    kind = rule[0]
    if kind == "pass":
        return R
    if L.kind in ("proj", "invproj"):
        # only Epsilon is meaningful here (explainer.py:200,202)
        if kind != "epsilon":
            raise ValueError("oracle: only Epsilon on (inv)projection")
        return x * _proj_jt(L, x, R / stabilize(z, rule[1]), ops)
    w, b = _params(L.module)
    if kind == "epsilon":
        g = R / stabilize(z, rule[1])
        return x * _aff_jt(L, x.shape, w, g, ops)
    if kind == "gamma":
        gam, eps = rule[1], rule[2]
        wp = w + gam * w.clamp(min=0)
        wn = w + gam * w.clamp(max=0)
        bp = _mod(b, lambda t: t + gam * t.clamp(min=0))
        bn = _mod(b, lambda t: t + gam * t.clamp(max=0))
        b0 = _mod(b, torch.zeros_like)
        xp, xn = x.clamp(min=0), x.clamp(max=0)
        # zennit 0.5.1 Gamma: the x- terms' modifiers are GammaMod(..., zero_params=zero_bias(...)),
        # so the bias enters each denominator once (as in ZPlus / AlphaBeta below)
        z0 = _aff(L, xp, wp, bp, ops)
        z1 = _aff(L, xn, wn, b0, ops)
        z2 = _aff(L, xp, wn, bn, ops)
        z3 = _aff(L, xn, wp, b0, ops)
        gpos = R * (z > 0) / stabilize(z0 + z1, eps)
        gneg = R * (z < 0) / stabilize(z2 + z3, eps)
        return (xp * _aff_jt(L, x.shape, wp, gpos, ops) + xn * _aff_jt(L, x.shape, wn, gpos, ops)
                + xp * _aff_jt(L, x.shape, wn, gneg, ops) + xn * _aff_jt(L, x.shape, wp, gneg, ops))
    if kind in ("wsquare", "flat"):
        eps = rule[1]
        if kind == "wsquare":
            w2, b2 = w * w, _mod(b, lambda t: t * t)
        else:
            w2, b2 = torch.ones_like(w), _mod(b, torch.zeros_like)
        den = _aff(L, torch.ones_like(x), w2, b2, ops)
        return _aff_jt(L, x.shape, w2, R / stabilize(den, eps), ops)
    if kind == "zplus":
        # zennit ZPlus: inputs (x+, x-), params (W+, b+) and (W-, 0); one shared denominator
        eps = rule[1]
        wp, wn = w.clamp(min=0), w.clamp(max=0)
        bp = _mod(b, lambda t: t.clamp(min=0))
        xp, xn = x.clamp(min=0), x.clamp(max=0)
        den = _aff(L, xp, wp, bp, ops) + _aff(L, xn, wn, _mod(b, torch.zeros_like), ops)
        g = R / stabilize(den, eps)
        return xp * _aff_jt(L, x.shape, wp, g, ops) + xn * _aff_jt(L, x.shape, wn, g, ops)
    if kind == "alphabeta":
        # zennit AlphaBeta: positive set (x+, W+, b+) + (x-, W-, 0), negative set (x+, W-, b-) +
        # (x-, W+, 0); one denominator per set; R_in = alpha * pos - beta * neg
        alpha, beta, eps = rule[1], rule[2], rule[3]
        wp, wn = w.clamp(min=0), w.clamp(max=0)
        bp, bn, b0 = (_mod(b, lambda t: t.clamp(min=0)), _mod(b, lambda t: t.clamp(max=0)),
                      _mod(b, torch.zeros_like))
        xp, xn = x.clamp(min=0), x.clamp(max=0)
        gp = R / stabilize(_aff(L, xp, wp, bp, ops) + _aff(L, xn, wn, b0, ops), eps)
        gn = R / stabilize(_aff(L, xp, wn, bn, ops) + _aff(L, xn, wp, b0, ops), eps)
        pos = xp * _aff_jt(L, x.shape, wp, gp, ops) + xn * _aff_jt(L, x.shape, wn, gp, ops)
        neg = xp * _aff_jt(L, x.shape, wn, gn, ops) + xn * _aff_jt(L, x.shape, wp, gn, ops)
        return alpha * pos - beta * neg
    raise ValueError(f"oracle: unknown rule {rule}")


# ----------------------------------------------------------------------------
# zennit-structured rules (modified forwards + autograd.grad), for the CPU baseline
# ----------------------------------------------------------------------------
def rule_backward_zennit(L: Layer, rule: RuleSpec, x: torch.Tensor, z: torch.Tensor,
                         R: torch.Tensor, ops=TorchOps) -> torch.Tensor:
    kind = rule[0]
    if kind == "pass" or L.kind in ("proj", "invproj"):
        return rule_backward_analytic(L, rule, x, z, R, ops)
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
        b0 = _mod(b, torch.zeros_like)
        inputs = [x.clamp(min=0), x.clamp(max=0), x.clamp(min=0), x.clamp(max=0), x]
        # GammaMod(min=0), GammaMod(max=0, zero_bias), GammaMod(max=0), GammaMod(min=0, zero_bias), NoMod
        params = [(wp, bp), (wn, b0), (wn, bn), (wp, b0), (w, b)]
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
    if kind == "zplus":
        eps = rule[1]
        params = [(w.clamp(min=0), _mod(b, lambda t: t.clamp(min=0))), (w.clamp(max=0), _mod(b, torch.zeros_like))]
        ins, outs = run([x.clamp(min=0), x.clamp(max=0)], params)
        g = R / stabilize(outs[0].detach() + outs[1].detach(), eps)
        grads = torch.autograd.grad(outs, ins, [g, g])
        return sum(i.detach() * gg for i, gg in zip(ins, grads))
    if kind == "alphabeta":
        alpha, beta, eps = rule[1], rule[2], rule[3]
        wp, wn = w.clamp(min=0), w.clamp(max=0)
        b0 = _mod(b, torch.zeros_like)
        params = [(wp, _mod(b, lambda t: t.clamp(min=0))), (wn, b0),
                  (wn, _mod(b, lambda t: t.clamp(max=0))), (wp, b0)]
        ins, outs = run([x.clamp(min=0), x.clamp(max=0)] * 2, params)
        o = [t.detach() for t in outs]
        gp = R / stabilize(o[0] + o[1], eps)
        gn = R / stabilize(o[2] + o[3], eps)
        grads = torch.autograd.grad(outs, ins, [gp, gp, gn, gn])
        r = [i.detach() * g for i, g in zip(ins, grads)]
        return alpha * (r[0] + r[1]) - beta * (r[2] + r[3])
    raise ValueError(f"oracle: unknown rule {rule}")


# ----------------------------------------------------------------------------
# plain-gradient layers
# ----------------------------------------------------------------------------
def _plain_backward(L: Layer, x: torch.Tensor, z: torch.Tensor, R: torch.Tensor, aux, ops=TorchOps) -> torch.Tensor:
    if L.kind == "relu":
        return torch.where(z > 0, R, torch.zeros_like(R))
    if L.kind == "maxpool":
        m = L.module
        return F.max_unpool2d(R, aux, m.kernel_size, m.stride, m.padding, output_size=x.shape[-2:])
    if L.kind in ("dropout",):
        return R
    if L.kind == "flatten":
        return R.reshape(x.shape)
    if L.kind == "conv":
        return ops.conv_t(L.module, x.shape, L.module.weight.detach(), R)
    if L.kind == "linear":
        return ops.linear_t(R, L.module.weight.detach())
    if L.kind in ("proj", "invproj"):
        return _proj_jt(L, x, R, ops)
    if L.kind in ("bn2d", "bn1d"):
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
        capture: Optional[str] = None, forced_inputs: Optional[Dict[str, torch.Tensor]] = None):
    """Returns (logits, R_input[, (act, rel) at layer ``capture``]).

    ``forced_inputs`` (layer name -> tensor): the input of that layer is replaced by the given
    values (the product's own activations, which differ from this forward's by accumulation-order
    rounding only), so that a bf16 rounding decision taken on them is the product's; the rest of
    the forward and the whole backward are evaluated here."""
    if mode in ("f64", "bf16", "bf16bwd"):
        import copy
        model = copy.deepcopy(model).double()
    if mode in ("bf16", "bf16bwd"):
        # the plan's weights are bf16 values (after any BN merge); rule-modified sets derived from
        # them are rounded again by Bf16Ops
        for mod in model.modules():
            if isinstance(mod, nn.Conv2d):
                mod.weight.data = _bf16r(mod.weight.data)
    layers = sequential_layers(model)
    ops = OPS[mode]
    acts: List[Tuple[torch.Tensor, torch.Tensor, object]] = []
    h = x.detach().to(torch.float64 if mode in ("f64", "bf16", "bf16bwd") else torch.float32)
    if mode in ("bf16", "bf16bwd"):
        h = _bf16r(h)
    for L in layers:
        aux = None
        if forced_inputs is not None and L.name in forced_inputs:
            h = forced_inputs[L.name].detach().to(h.device, h.dtype).reshape(h.shape)
        if L.kind == "maxpool":
            m = L.module
            out, aux = F.max_pool2d(h, m.kernel_size, m.stride, m.padding, m.dilation,
                                    m.ceil_mode, return_indices=True)
        elif L.kind == "invproj" and hasattr(ops, "inv_projection"):
            out = ops.inv_projection(L, h, proj_in)
        else:
            out = _layer_fwd(L, h, ops)
        if L.kind == "proj":
            proj_in = h
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
            R = rb(L, rule, xin, zout, R, ops)
        else:
            R = _plain_backward(L, xin, zout, R, aux, ops)
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


def numpy_pairwise_sum(a: np.ndarray) -> np.float32:
    """numpy's float32 add-reduce of a contiguous run (the order sort_subspaces' ``sum(axis=(-2,
    -1))`` uses, explainer.py:161).  The reduction iterator hands the inner loop chunks of at most
    8192 elements (numpy's buffer size) and folds them left to right into the identity 0; each
    chunk is summed pairwise: n < 8 a left-to-right chain from 0; n <= 128 eight stride-8
    accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus the n % 8 tail; otherwise the
    two halves split at n/2 - (n/2 % 8).  Scalar restatement of what heatmap_sort_kernel computes
    (small inputs only: pure Python)."""
    f = np.float32
    a = np.asarray(a, dtype=np.float32).reshape(-1)

    def pw(lo, n):
        if n < 8:
            r = f(0)
            for i in range(n):
                r = f(r + a[lo + i])
            return r
        if n <= 128:
            r = [a[lo + j] for j in range(8)]
            i = 8
            while i < n - n % 8:
                for j in range(8):
                    r[j] = f(r[j] + a[lo + i + j])
                i += 8
            res = f(f(f(r[0] + r[1]) + f(r[2] + r[3])) + f(f(r[4] + r[5]) + f(r[6] + r[7])))
            for k in range(i, n):
                res = f(res + a[lo + k])
            return res
        n2 = n // 2
        n2 -= n2 % 8
        return f(pw(lo, n2) + pw(lo + n2, n - n2))
    acc = f(0)
    for lo in range(0, a.size, 8192):
        acc = f(acc + pw(lo, min(8192, a.size - lo)))
    return acc


def sort_subspaces(sub: np.ndarray, ops=TorchOps):
    """explainer.py:151-176 with batch dims kept (defect D7: B=1 must not squeeze)."""
    rel = ops.plane_sum(sub).reshape(sub.shape[0], sub.shape[1])
    mask = np.argsort(rel, axis=-1)[..., ::-1]
    ar = np.arange(sub.shape[0])[:, None]
    return sub[ar, mask], rel[ar, mask], mask


@torch.no_grad()
def subspace_heatmaps(proj_model: nn.Module, name_map: Dict[str, RuleSpec], K: int,
                      x: torch.Tensor, class_idx: int, one_hot_encoded=False,
                      mode: str = "analytic", forced_inputs=None, standard: Optional[str] = None) -> Dict[str, np.ndarray]:
    """HeatmapGenerator.generate_subspace_heatmaps (explainer.py:87-123) on the CPU.
    ``forced_inputs``: per-sample layer inputs (see ``lrp``), replicated like the batch.
    ``standard``: "clone" = clone 0 of the replicated batch (the reference); "sum" = the K concept
    heatmaps summed, k ascending, in the heatmaps' precision (the product's HeatmapGenerator
    standard="sum" option; equal in exact arithmetic since every rule is linear in the relevance).
    Default: "clone", as the product's HeatmapGenerator default."""
    if standard is None:
        standard = "clone"
    rules = class_composite_rules(name_map, K)
    xr = x.repeat_interleave(K + 1, dim=0)
    if forced_inputs is not None:
        forced_inputs = {k: v.repeat_interleave(K + 1, dim=0) for k, v in forced_inputs.items()}
    _, R = lrp(proj_model, rules, xr, class_idx=class_idx, one_hot_encoded=one_hot_encoded, mode=mode,
               forced_inputs=forced_inputs)
    H, W = R.shape[-2:]
    hm = R.reshape(-1, K + 1, H, W).numpy()
    std, sub = hm[:, 0:1], hm[:, 1:]
    if standard == "sum":
        acc = sub[:, 0:1].copy()
        for k in range(1, K):
            acc = acc + sub[:, k:k + 1]
        std = acc
    elif standard != "clone":
        raise ValueError(standard)
    ops = OPS[mode]
    sub_s, rel_s, mask = sort_subspaces(sub, ops)
    return {
        "standard_heatmaps": std,
        "standard_relevance": ops.plane_sum(std).flatten(),
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
