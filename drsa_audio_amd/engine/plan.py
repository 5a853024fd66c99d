"""LRP kernel plan: compile (model, composite) once, then run batches through HIP kernels.

The reference attaches zennit hooks and lets autograd re-run 1-5 modified forwards per
layer (attribute.py:98-107).  Here the sequential VGG structure (create_model.py:8-97,
optionally with the ProjectionModel virtual layers, modify_model.py:19-60) is compiled
into *stages*:

  ConvStage   Conv2d [+BN folded by SequentialMergeBatchNorm] -> ReLU
              [-> Projection/SubspaceFilter/InvProjection] [-> MaxPool2d(2)]
  DenseStage  Linear [+BN folded] [-> ReLU] [-> Dropout]

Forward: one ``drsa_amd_conv_fwd`` per conv stage computes y = pool(relu(conv)), the pool
argmax and the rule's denominator at the argmax (the only place relevance arrives).
Backward: one ``drsa_amd_conv_bwd`` per conv stage, the max-pool/ReLU backward folded
into its input, the next lower layer's division folded into its output.  The subspace
path fans one forward out into K+1 relevance clones at the projection
(``drsa_amd_projection_bwd``), instead of replicating the batch K+1 times
(explainer.py:92).

Weights are prepared on the device once per plan (rule-modified, flipped/transposed for
the backward, padded to the kernels' channel tiles).  Activation buffers are cached per
batch size.

Precision: a model whose parameters are bfloat16 (``model.bfloat16()``) compiles a bf16 plan
(the reference has no bf16 path): every conv weight set (rule-modified, forward and
backward) is rounded to bf16, the network input is rounded to bf16, and every conv with Cin > 1
runs forward on ``drsa_amd_conv_fwd_bf16`` (inputs rounded to bf16 as they are staged,
v_mfma_f32_32x32x16_bf16, fp32 accumulation).  Biases, activations, denominators, the dense head
and the whole relevance backward stay fp32 (oracle: ``lrp_ref.lrp(mode="bf16")``).  With
``bf16_backward`` (``DRSA_AMD_BF16_BACKWARD=1``) every backward conv with Cin > 1 (ng = 1) also runs
on bf16 operands: ``drsa_amd_conv_bwd_bf16`` rounds the quotient g = R / stab(den) to bf16 as it is
staged, accumulates in fp32, and keeps the epilogue fp32 (oracle: ``mode="bf16bwd"``).
"""
from __future__ import annotations

import os
import weakref
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from .. import _capi
from .._capi import POST_DIV, POST_DIV_MAP, POST_DIV_RING, POST_MASK, POST_NONE, XM_MUL, XM_NONE, XM_SPLIT
from ..zennit import rules as R
from ..zennit.canonizers import SequentialMergeBatchNorm

# Alternative plan forms, bit-identical to the defaults, that the parity tests switch on to prove
# it (module attributes, not run-time knobs):
# _PROJ_STORE: the projection forward stores h and a' and projection_bwd reads them (instead of
#   recomputing them from a);
# _DEN_COPY: the WSquare/Flat layer's forward stores its per-sample denominator at the argmax
#   everywhere and the next backward reads it there (POST_DIV) instead of the ring form;
# _POOL24_SPARSE = False: the (2,4) pool backward as a separate unpool before a dense-g backward
#   instead of folded into the backward conv's staging.
_PROJ_STORE = False
_DEN_COPY = False
_POOL24_SPARSE = True


def _pad32(c: int) -> int:
    return (c + 31) // 32 * 32


def _cin_pad(c: int) -> int:
    return 1 if c == 1 else _pad32(c)


def _kind(rule) -> Optional[str]:
    k = None if rule is None else getattr(rule, "kind", type(rule).__name__)
    # zennit Norm(stabilizer) on a conv/dense layer is Epsilon(epsilon=stabilizer): same
    # input/output modifiers, parameters unmodified (NoMod with no keys), gradient mapper
    # out_grad / stabilize(z) and reducer x * grad
    return "epsilon" if k == "norm" else k


def _eps_of(rule) -> float:
    return float(getattr(rule, "epsilon", getattr(rule, "stabilizer", 0.0)))


@dataclass

class ProjGroup:
    U: torch.Tensor
    K: int
    P: Optional[torch.Tensor]   # U U^T - I (drsa_amd_projection_residual), set at plan build
    eps_inv: float
    eps_proj: float
    mask: bool          # SubspaceHook on the filter
    pool_after: bool


@dataclass
class ConvStage:
    name: str
    cin: int
    cout: int
    rule_kind: Optional[str]
    eps: float
    pool: bool
    proj: Optional[ProjGroup]
    input_nonneg: bool
    W: torch.Tensor = None
    b: torch.Tensor = None
    rule: object = None
    # prepared
    ng_fwd: int = 1
    wts_fwd: torch.Tensor = None
    bias3: torch.Tensor = None
    den_kind: Optional[str] = None       # "gamma" | "eps" | "map" | "ab" | None
    # AlphaBeta: second forward (W, W-) for den_n, and the two backward weight sets
    wts_fwd_n: torch.Tensor = None
    bias3_n: torch.Tensor = None
    wts_bwd_n: torch.Tensor = None
    wts_fwd_bf: torch.Tensor = None      # bf16 plan: [ng][cin_p/16][9][2][cout_p][8] bfloat16
    wts_fwd_n_bf: torch.Tensor = None
    wts_bwd_bf: torch.Tensor = None       # bf16 backward: [cout_p/16][9][2][pad32(cin)][8] bfloat16
    alpha: float = 1.0
    beta: float = 0.0
    ng_bwd: int = 1
    wts_bwd: torch.Tensor = None
    xmode_bwd: int = XM_NONE
    w2_first: Optional[torch.Tensor] = None
    den_maps: Dict[Tuple[int, int], torch.Tensor] = field(default_factory=dict)
    relu_name: Optional[str] = None      # features.<i> of the ReLU after the conv
    pool_name: Optional[str] = None      # features.<i> of the MaxPool2d (None: no pool)
    pool_k: Tuple[int, int] = (2, 2)     # max-pool kernel (= stride); 2x2 is fused into the conv


@dataclass
class DenseStage:
    name: str
    W: torch.Tensor
    b: Optional[torch.Tensor]
    rule_kind: Optional[str]
    eps: float
    relu_after: bool


class EngineError(NotImplementedError):
    pass


class LRPEngine:
    def __init__(self, model: nn.Module, composite, device: Optional[torch.device] = None,
                 precision: Optional[str] = None, bf16_backward: Optional[bool] = None):
        _capi.load()
        # no strong references to the model / composite: the plan owns prepared copies of what it
        # needs, and get_engine's cache is keyed by weak references (engine/__init__.py)
        self._model_ref = weakref.ref(model)
        self._composite_ref = (lambda: None) if composite is None else weakref.ref(composite)
        p0 = next(model.parameters())
        self.device = device or p0.device
        if precision is None:
            precision = "bf16" if p0.dtype == torch.bfloat16 else "fp32"
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        self.precision = precision
        self.bf16 = precision == "bf16"
        # bf16 plan option: the relevance backward convs on bf16 operands too (g rounded to bf16 as it
        # is staged, fp32 accumulation and epilogue); default from DRSA_AMD_BF16_BACKWARD (off)
        if bf16_backward is None:
            bf16_backward = bf16_backward_default()
        self.bf16_backward = bool(bf16_backward) and self.bf16
        if self.device.type != "cuda":
            raise _capi.DrsaAmdError("the LRP engine runs on the GPU only; move the model to a HIP device")
        rules = composite.rules(model) if composite is not None else {}
        self.rules = rules
        merge_bn = any(isinstance(c, SequentialMergeBatchNorm) for c in getattr(composite, "canonizers", []))
        self.stages: List[ConvStage] = []
        self.dense: List[DenseStage] = []
        self._parse(model, rules, merge_bn)
        for st in self.stages:
            self._prepare_conv(st)
        self._buffers: Dict[tuple, dict] = {}
        self.last: Optional[dict] = None
        self.trace: Optional[list] = None      # set to [] to record (tag, start_event, end_event)

    @property
    def model(self):
        return self._model_ref()

    @property
    def composite(self):
        return self._composite_ref()

    def release(self) -> None:
        """Free the cached activation/relevance buffers and prepared per-shape state."""
        self._buffers.clear()
        self._cur_bufs = {}
        for st in self.stages:
            st.den_maps.clear()
        self.last = None

    def _call(self, tag: str, name: str, *args) -> None:
        if self.trace is None:
            _capi.call(name, *args)
            return
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _capi.call(name, *args)
        e1.record()
        self.trace.append((tag, e0, e1))

    # ------------------------------------------------------------------ parse
    def _parse(self, model, rules, merge_bn):
        feats = list(model.features.named_children())
        i, n = 0, len(feats)
        prev_nonneg = False          # raw network input may be negative
        while i < n:
            name, m = feats[i]
            if isinstance(m, (nn.Dropout, nn.Identity)):
                i += 1
                continue
            if not isinstance(m, nn.Conv2d):
                raise EngineError(f"engine: unexpected feature layer features.{name} ({type(m).__name__})")
            self._check_conv(m, name)
            # weights are prepared on the host in fp32 (the BN merge there is the same IEEE
            # arithmetic as zennit's canonizer on CPU) and then moved to the device once
            W = m.weight.detach().cpu().to(torch.float32)
            b = (m.bias.detach().cpu().to(torch.float32) if m.bias is not None
                 else torch.zeros(m.out_channels))
            j = i + 1
            if j < n and isinstance(feats[j][1], nn.BatchNorm2d):
                if not merge_bn:
                    raise EngineError("BatchNorm2d in the trunk needs the SequentialMergeBatchNorm canonizer")
                W, b = SequentialMergeBatchNorm.fold(W, b, _bn_to(feats[j][1], torch.device("cpu")))
                j += 1
            if self.bf16:
                W = _bf16r(W)
            W, b = W.to(self.device), b.to(self.device)
            if j >= n or not isinstance(feats[j][1], nn.ReLU):
                raise EngineError(f"engine: conv features.{name} must be followed by ReLU")
            self._rule_ok_on_activation(rules.get(f"features.{feats[j][0]}"))
            relu_name = f"features.{feats[j][0]}"
            j += 1
            proj = None
            if j < n and type(feats[j][1]).__name__ == "Projection":
                if not (j + 2 < n and type(feats[j + 1][1]).__name__ == "SubspaceFilter"
                        and type(feats[j + 2][1]).__name__ == "InvProjection"):
                    raise EngineError("engine: Projection must be followed by SubspaceFilter, InvProjection")
                pm, fm, im = feats[j][1], feats[j + 1][1], feats[j + 2][1]
                r_p = rules.get(f"features.{feats[j][0]}")
                r_f = rules.get(f"features.{feats[j + 1][0]}")
                r_i = rules.get(f"features.{feats[j + 2][0]}")
                if _kind(r_p) != "epsilon" or _kind(r_i) != "epsilon":
                    raise EngineError("engine: projection layers need Epsilon rules (get_class_composite)")
                if r_f is not None and type(r_f).__name__ != "SubspaceHook":
                    raise EngineError("engine: only SubspaceHook is supported on the subspace filter")
                U = pm.U.detach().to(self.device, torch.float32).contiguous()
                Pm = torch.empty_like(U)
                _capi.call("drsa_amd_projection_residual", U.data_ptr(), U.size(0), Pm.data_ptr(),
                           _capi.stream_ptr(self.device))
                proj = ProjGroup(U=U, K=int(pm.num_concepts), P=Pm, eps_inv=_eps_of(r_i), eps_proj=_eps_of(r_p),
                                 mask=r_f is not None, pool_after=False)
                if r_f is not None and int(r_f.num_concepts) != proj.K:
                    raise EngineError("engine: SubspaceHook num_concepts differs from the projection")
                j += 3
            pool = False
            pool_name = None
            pool_k = (2, 2)
            if j < n and isinstance(feats[j][1], nn.MaxPool2d):
                pool_k = self._check_pool(feats[j][1])
                self._rule_ok_on_activation(rules.get(f"features.{feats[j][0]}"))
                pool = True
                pool_name = f"features.{feats[j][0]}"
                j += 1
            if proj is not None:
                proj.pool_after = pool
                if pool and pool_k != (2, 2):
                    raise EngineError("engine: a ProjectionModel layer must be followed by MaxPool2d(2) or no pool")
            rule = rules.get(f"features.{name}")
            kind = _kind(rule)
            if kind not in (None, "epsilon", "gamma", "wsquare", "flat", "zplus", "alphabeta"):
                raise EngineError(f"engine: rule {type(rule).__name__} on conv features.{name} is not supported yet")
            if kind == "alphabeta" and (not prev_nonneg or (pool and pool_k != (2, 2))):
                raise EngineError(f"engine: AlphaBeta on features.{name} needs a non-negative input (not the first "
                                  "conv) and a 2x2 or no max-pool after it")
            eps = {None: 0.0, "epsilon": _eps_of(rule), "gamma": getattr(rule, "stabilizer", 0.0),
                   "wsquare": getattr(rule, "stabilizer", 0.0), "flat": getattr(rule, "stabilizer", 0.0),
                   "zplus": getattr(rule, "stabilizer", 0.0), "alphabeta": getattr(rule, "stabilizer", 0.0)}[kind]
            st = ConvStage(name=f"features.{name}", cin=m.in_channels, cout=m.out_channels, rule_kind=kind,
                           eps=float(eps), pool=pool, proj=proj, input_nonneg=prev_nonneg, W=W, b=b, rule=rule,
                           relu_name=relu_name, pool_name=pool_name, pool_k=pool_k)
            self.stages.append(st)
            prev_nonneg = proj is None      # outputs are post-ReLU (pooled) unless a' follows
            i = j
        # classifier
        cl = list(model.classifier.named_children())
        i, n = 0, len(cl)
        while i < n:
            name, m = cl[i]
            if isinstance(m, (nn.Dropout, nn.Identity)):
                i += 1
                continue
            if not isinstance(m, nn.Linear):
                raise EngineError(f"engine: unexpected classifier layer classifier.{name} ({type(m).__name__})")
            W = m.weight.detach().cpu().to(torch.float32)
            b = m.bias.detach().cpu().to(torch.float32) if m.bias is not None else None
            j = i + 1
            if j < n and isinstance(cl[j][1], nn.BatchNorm1d):
                if not merge_bn:
                    raise EngineError("BatchNorm1d in the head needs the SequentialMergeBatchNorm canonizer")
                W, b = SequentialMergeBatchNorm.fold(W, b, _bn_to(cl[j][1], torch.device("cpu")))
                j += 1
            W = W.to(self.device)
            b = None if b is None else b.to(self.device)
            relu = False
            while j < n and isinstance(cl[j][1], (nn.ReLU, nn.Dropout)):
                if isinstance(cl[j][1], nn.ReLU):
                    relu = True
                    self._rule_ok_on_activation(rules.get(f"classifier.{cl[j][0]}"))
                j += 1
            rule = rules.get(f"classifier.{name}")
            kind = _kind(rule)
            if kind not in (None, "epsilon"):
                raise EngineError(f"engine: rule {type(rule).__name__} on classifier.{name} is not supported yet")
            if rule is not None and "bias" in getattr(rule, "zero_params", ()):
                raise EngineError("engine: zero_params on dense layers is not supported yet")
            self.dense.append(DenseStage(name=f"classifier.{name}", W=W.contiguous(),
                                         b=None if b is None else b.contiguous(), rule_kind=kind,
                                         eps=_eps_of(rule) if kind else 0.0, relu_after=relu))
            i = j
        if not self.stages or not self.dense:
            raise EngineError("engine: model must have a conv trunk and a dense head")

    @staticmethod
    def _check_conv(m: nn.Conv2d, name):
        pad = m.padding
        ok = (tuple(m.kernel_size) == (3, 3) and tuple(m.stride) == (1, 1) and tuple(m.dilation) == (1, 1)
              and m.groups == 1 and (pad == "same" or tuple(pad) == (1, 1)) and m.padding_mode == "zeros")
        if not ok:
            raise EngineError(f"engine: features.{name} must be a 3x3 stride-1 'same' zero-padded conv")

    @staticmethod
    def _check_pool(m: nn.MaxPool2d):
        ks = m.kernel_size if isinstance(m.kernel_size, tuple) else (m.kernel_size, m.kernel_size)
        st = m.stride if isinstance(m.stride, tuple) else (m.stride, m.stride)
        pd = m.padding if isinstance(m.padding, tuple) else (m.padding, m.padding)
        dl = m.dilation if isinstance(m.dilation, tuple) else (m.dilation, m.dilation)
        if tuple(ks) != tuple(st) or tuple(pd) != (0, 0) or tuple(dl) != (1, 1) or m.ceil_mode or ks[0] * ks[1] > 256:
            raise EngineError(f"engine: MaxPool2d must have stride = kernel, no padding/dilation (got kernel {ks}, "
                              f"stride {st})")
        return (int(ks[0]), int(ks[1]))

    @staticmethod
    def _rule_ok_on_activation(rule):
        if rule is not None and _kind(rule) != "pass":
            raise EngineError(f"engine: rule {type(rule).__name__} on an activation/pool layer is not supported")

    # ---------------------------------------------------------------- prepare
    @torch.no_grad()
    def _prepare_conv(self, st: ConvStage):
        dev = self.device
        W, b = st.W, st.b
        cin_p, cout_p = _cin_pad(st.cin), _pad32(st.cout)
        zero_bias = "bias" in getattr(st.rule, "zero_params", ())
        bd = torch.zeros_like(b) if zero_bias else b

        def fwd_layout(Wx):   # [cout][cin][3][3] -> [9*cin_p][cout_p], row k = ci*9 + ky*3 + kx
            t = torch.zeros(cin_p, 3, 3, cout_p, device=dev)
            t[:st.cin, :, :, :st.cout] = Wx.permute(1, 2, 3, 0)
            return t.reshape(9 * cin_p, cout_p)

        def bwd_layout(Wx):   # transposed conv as 'same' conv: [9*cout_p][pad32(cin)], flipped taps
            cin_o = _pad32(st.cin)
            t = torch.zeros(cout_p, 3, 3, cin_o, device=dev)
            t[:st.cout, :, :, :st.cin] = Wx.flip(2, 3).permute(0, 2, 3, 1)
            return t.reshape(9 * cout_p, cin_o)

        bias3 = torch.zeros(3, cout_p, device=dev)
        bias3[0, :st.cout] = b
        k = st.rule_kind
        if k == "gamma":
            g = st.rule.gamma
            # zennit 0.5.1 Gamma: den+ = (conv(x+; W+) + b+) + conv(x-; W-), the x- term's
            # modifier zeroing the bias (zero_bias), as for ZPlus below. Only den+ is
            # formed: R reaches the conv through its ReLU, so g- = R [z < 0] / den- is 0
            Wp, Wn = W + g * W.clamp(min=0), W + g * W.clamp(max=0)
            bias3[1, :st.cout], bias3[2, :st.cout] = bd + g * bd.clamp(min=0), 0.0
            sets = [W, Wp] + ([Wn] if not st.input_nonneg else [])
            st.ng_fwd = len(sets)
            st.den_kind = "gamma"
            if st.input_nonneg:
                st.ng_bwd, st.xmode_bwd, bsets = 1, XM_MUL, [Wp]
            else:
                st.ng_bwd, st.xmode_bwd, bsets = 2, XM_SPLIT, [Wp, Wn]
        elif k == "zplus":
            # zennit ZPlus: (x+, W+, b+) and (x-, W-, 0) with one shared denominator: the Gamma
            # kernels with the clamped weight sets and a zero second bias
            Wp, Wn = W.clamp(min=0), W.clamp(max=0)
            bias3[1, :st.cout], bias3[2, :st.cout] = bd.clamp(min=0), 0.0
            sets = [W, Wp] + ([Wn] if not st.input_nonneg else [])
            st.ng_fwd = len(sets)
            st.den_kind = "gamma"
            if st.input_nonneg:
                st.ng_bwd, st.xmode_bwd, bsets = 1, XM_MUL, [Wp]
            else:
                st.ng_bwd, st.xmode_bwd, bsets = 2, XM_SPLIT, [Wp, Wn]
        elif k == "alphabeta":
            # zennit AlphaBeta on a non-negative input (oracle lrp_ref.py alphabeta): positive set
            # (x, W+, b+) and negative set (x, W-, b-), the x- terms vanish; den_p and den_n come
            # from two Gamma-form forwards (den = (conv(x; W+-) + b+-) + 0)
            Wp, Wn = W.clamp(min=0), W.clamp(max=0)
            bias3[1, :st.cout] = bd.clamp(min=0)
            bias3n = torch.zeros(3, cout_p, device=dev)
            bias3n[0, :st.cout] = b
            bias3n[1, :st.cout] = bd.clamp(max=0)
            sets, st.ng_fwd, st.den_kind = [W, Wp], 2, "ab"
            st.wts_fwd_n = torch.stack([fwd_layout(s_) for s_ in (W, Wn)]).contiguous()
            st.bias3_n = bias3n.contiguous()
            st.ng_bwd, st.xmode_bwd, bsets = 1, XM_MUL, [Wp]
            st.wts_bwd_n = torch.stack([bwd_layout(Wn)]).contiguous()
            st.alpha, st.beta = float(st.rule.alpha), float(st.rule.beta)
        elif k == "epsilon":
            bias3[1, :st.cout] = bd
            sets, st.ng_fwd, st.den_kind = [W], 1, "eps"
            st.ng_bwd, st.xmode_bwd, bsets = 1, XM_MUL, [W]
        elif k in ("wsquare", "flat"):
            if k == "wsquare":
                W2, b2 = W * W, bd * bd
            else:
                W2, b2 = torch.ones_like(W), torch.zeros_like(b)
            st.W2, st.b2 = W2.contiguous(), b2.contiguous()
            sets, st.ng_fwd, st.den_kind = [W], 1, "map"
            st.ng_bwd, st.xmode_bwd, bsets = 1, XM_NONE, [W2]
            if st.cin == 1:
                st.w2_first = W2.reshape(st.cout, 9).contiguous()
        else:   # no rule: plain gradient
            sets, st.ng_fwd, st.den_kind = [W], 1, None
            st.ng_bwd, st.xmode_bwd, bsets = 1, XM_NONE, [W]
        if self.bf16:
            # every weight set the kernels see holds bf16 values (forward and backward alike)
            sets, bsets = [_bf16r(s_) for s_ in sets], [_bf16r(s_) for s_ in bsets]
            if k in ("wsquare", "flat"):
                st.W2 = _bf16r(st.W2)
                if st.w2_first is not None:
                    st.w2_first = _bf16r(st.w2_first)
            if st.wts_fwd_n is not None:
                st.wts_fwd_n = _bf16r(st.wts_fwd_n)
                st.wts_bwd_n = _bf16r(st.wts_bwd_n)
        st.wts_fwd = torch.stack([fwd_layout(s) for s in sets]).contiguous()
        st.bias3 = bias3.contiguous()
        st.wts_bwd = torch.stack([bwd_layout(s) for s in bsets]).contiguous()
        if self.bf16 and st.cin > 1:
            st.wts_fwd_bf = _bf16_layout(st.wts_fwd, cin_p, cout_p)
            if st.wts_fwd_n is not None:
                st.wts_fwd_n_bf = _bf16_layout(st.wts_fwd_n, cin_p, cout_p)
        if (self.bf16_backward and st.cin > 1 and st.ng_bwd == 1 and st.den_kind != "ab" and
                _capi.lib().drsa_amd_conv_bwd_has_kernel_bf16(st.cout, st.cin, 32, 1, 0)):
            st.wts_bwd_bf = _bf16_layout(st.wts_bwd, cout_p, _pad32(st.cin))
        if st.proj is not None and st.proj.U.size(0) != st.cout:
            raise EngineError("engine: projection width differs from the conv channels")

    def _den_map(self, st: ConvStage, H: int, W: int) -> torch.Tensor:
        key = (H, W)
        if key not in st.den_maps:
            den = torch.empty(st.cout, H, W, device=self.device)
            _capi.call("drsa_amd_first_layer_den", st.W2.data_ptr(), st.b2.data_ptr(), den.data_ptr(), st.cout,
                       st.cin, H, W, _capi.stream_ptr(self.device))
            st.den_maps[key] = den
        return st.den_maps[key]

    def _den_const4(self, st: ConvStage, H: int, W: int) -> torch.Tensor:
        """[cout][4]: the map's interior value per channel (drsa_amd_first_layer_den computes every
        interior pixel with the same 9-tap chain, so map[c][1][1] is all of them), 4 copies."""
        key = ("c4", H, W)
        if key not in st.den_maps:
            m = self._den_map(st, H, W)
            st.den_maps[key] = m[:, 1, 1].reshape(-1, 1).expand(-1, 4).contiguous()
        return st.den_maps[key]

    def _conv_fwd(self, tag, st: ConvStage, neg: bool, cur, den_map, out, amax, den, B, h, w, ng, pool, s):
        """One conv forward launch: the bf16 kernel in a bf16 plan (Cin > 1), else fp32."""
        bias3 = st.bias3_n if neg else st.bias3
        if self.bf16 and st.cin > 1:
            name, wts = "drsa_amd_conv_fwd_bf16", (st.wts_fwd_n_bf if neg else st.wts_fwd_bf)
        else:
            name, wts = "drsa_amd_conv_fwd", (st.wts_fwd_n if neg else st.wts_fwd)
        self._call(tag, name, cur.data_ptr(), wts.data_ptr(), bias3.data_ptr(), _capi.ptr(den_map), out.data_ptr(),
                   _capi.ptr(amax), _capi.ptr(den), B, st.cin, st.cout, h, w, ng, pool, s)

    # ---------------------------------------------------------------- buffers
    def _buf(self, key, shape, dtype=torch.float32):
        t = self._cur_bufs.get(key)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = torch.empty(shape, dtype=dtype, device=self.device)
            self._cur_bufs[key] = t
        return t

    # ---------------------------------------------------------------- forward
    @torch.no_grad()
    def forward(self, x: torch.Tensor, capture: Optional[int] = None) -> torch.Tensor:
        """Model forward with all LRP state (argmax, denominators) kept on device.  ``capture``:
        index of a conv stage whose full-resolution ReLU output is kept even though a max-pool
        follows (the reference's store_hook, preprocessing.py:92-103)."""
        _capi.require_gpu(x, "input", dtype=None)
        x = x.detach()
        if self.bf16:
            x = x.to(torch.bfloat16)
        x = x.to(torch.float32).contiguous()
        if x.dim() != 4 or x.size(1) != self.stages[0].cin:
            raise ValueError(f"input must be [B, {self.stages[0].cin}, H, W]")
        B, _, H, W = x.shape
        self._cur_bufs = self._buffers.setdefault(("fwd", B, H, W), {})
        s = _capi.stream_ptr(self.device)
        state = {"B": B, "input": x, "stages": []}
        cur, h, w = x, H, W
        for li, st in enumerate(self.stages):
            ph, pw = st.pool_k if st.pool else (1, 1)
            if h % 2 or w % 2 or h % ph or w % pw:
                raise ValueError(f"{st.name}: feature map {h}x{w} must have even sides divisible by the pool")
            rec = {"in": cur, "H": h, "W": w}
            den_map = self._den_map(st, h, w) if st.den_kind == "map" else None
            need_den = st.den_kind is not None
            if st.den_kind == "ab" and li == capture and st.pool:
                raise EngineError("engine: capture at the ReLU of an AlphaBeta conv is not supported")
            # pools fused into the conv epilogue: 2x2 and 2x4 (code 1 / 2); others, and the capture
            # layer (its full-resolution ReLU output is kept), go through maxpool_capture
            fused_pool = {(2, 2): 1, (2, 4): 2}.get(st.pool_k) if st.pool else None
            if fused_pool == 2 and not _capi.lib().drsa_amd_conv_fwd_has_kernel(
                    st.cin, st.cout, w, st.ng_fwd, 2, int(self.bf16 and st.cin > 1)):
                fused_pool = None
            if st.proj is None and st.pool and (li == capture or fused_pool is None):
                a = self._buf((li, "a"), (B, st.cout, h, w))
                den_full = self._buf((li, "den_full"), (B, st.cout, h, w)) if need_den else None
                self._conv_fwd(f"conv_fwd:{st.name}", st, False, cur, den_map, a, None, den_full, B, h, w, st.ng_fwd, 0, s)
                out = self._buf((li, "y"), (B, st.cout, h // ph, w // pw))
                amax = self._buf((li, "amax"), (B, st.cout, h // ph, w // pw), torch.uint8)
                den = self._buf((li, "den"), (B, st.cout, h // ph, w // pw)) if need_den else None
                self._call(f"maxpool:{st.pool_name}", "drsa_amd_maxpool_capture", a.data_ptr(), _capi.ptr(den_full),
                           out.data_ptr(), amax.data_ptr(), _capi.ptr(den), B, st.cout, h, w, ph, pw, s)
                rec.update(a=a, y=out, amax=amax, den=den, Hout=h // ph, Wout=w // pw)
                cur, h, w = out, h // ph, w // pw
            elif st.proj is None and st.pool:
                ph, pw = st.pool_k
                # WSquare / Flat first layer under a 2x2 pool: its map is one value per channel off the
                # image's border ring, so the forward stores the per-sample denominator copy only on the
                # ring, compactly (drsa_amd_conv_fwd_den_ring), and the next conv's backward reads the
                # map's interior value elsewhere (drsa_amd_conv_bwd_den_ring; bit-identical)
                ring = (st.den_kind == "map" and st.pool_k == (2, 2) and st.cin == 1 and w % 16 == 0 and h >= 4
                        and li + 1 < len(self.stages) and self.stages[li + 1].den_kind != "ab" and not _DEN_COPY)
                out = self._buf((li, "y"), (B, st.cout, h // ph, w // pw))
                amax = self._buf((li, "amax"), (B, st.cout, h // ph, w // pw), torch.uint8)
                if ring:
                    den = self._buf((li, "den_ring"), (B, st.cout, 2 * (w // 2) + 8 * (h // 2 - 2)))
                    self._call(f"conv_fwd:{st.name}", "drsa_amd_conv_fwd_den_ring", cur.data_ptr(),
                               st.wts_fwd.data_ptr(), st.bias3.data_ptr(), den_map.data_ptr(), out.data_ptr(),
                               amax.data_ptr(), den.data_ptr(), B, st.cout, h, w, st.ng_fwd, s)
                else:
                    den = self._buf((li, "den"), (B, st.cout, h // ph, w // pw)) if need_den else None
                    self._conv_fwd(f"conv_fwd:{st.name}", st, False, cur, den_map, out, amax, den, B, h, w, st.ng_fwd,
                                   fused_pool, s)
                rec.update(y=out, amax=amax, den=den, Hout=h // ph, Wout=w // pw,
                           den_const4=self._den_const4(st, h, w) if ring else None)
                if st.den_kind == "ab":   # second pass: den_n (y and argmax rewritten with the same values)
                    den_n = self._buf((li, "den_n"), (B, st.cout, h // ph, w // pw))
                    self._conv_fwd(f"conv_fwd_n:{st.name}", st, True, cur, None, out, amax, den_n, B, h, w, 2,
                                   fused_pool, s)
                    rec.update(den_n=den_n)
                cur, h, w = out, h // ph, w // pw
            else:
                a = self._buf((li, "a"), (B, st.cout, h, w))
                # WSquare / Flat without a pool after it (VGGish conv0 -> conv3): the per-sample
                # denominator IS the input-independent map; the next backward reads the map itself
                # (drsa_amd_conv_bwd_den_map), no per-sample copy is written
                shared = (st.den_kind == "map" and st.proj is None and li + 1 < len(self.stages)
                          and self.stages[li + 1].den_kind != "ab" and not _DEN_COPY)
                den = self._buf((li, "den"), (B, st.cout, h, w)) if need_den and not shared else None
                self._conv_fwd(f"conv_fwd:{st.name}", st, False, cur, den_map, a, None, den, B, h, w, st.ng_fwd, 0, s)
                rec.update(a=a, den=den, den_map_shared=den_map if shared else None)
                if st.den_kind == "ab":
                    den_n = self._buf((li, "den_n"), (B, st.cout, h, w))
                    self._conv_fwd(f"conv_fwd_n:{st.name}", st, True, cur, None, a, None, den_n, B, h, w, 2, 0, s)
                    rec.update(den_n=den_n)
                if st.proj is not None:
                    P = st.proj
                    # h and a' are recomputed by projection_bwd from a (no HBM round trip); a' is
                    # stored only when it is the stage output (no pool after the projection)
                    hb = self._buf((li, "h"), (B, st.cout, h * w)) if _PROJ_STORE else None
                    ap = self._buf((li, "ap"), (B, st.cout, h, w)) if (_PROJ_STORE or not P.pool_after) else None
                    if P.pool_after:
                        pooled = self._buf((li, "y"), (B, st.cout, h // 2, w // 2))
                        amax = self._buf((li, "amax"), (B, st.cout, h // 2, w // 2), torch.uint8)
                    else:
                        pooled = amax = None
                    self._call("projection_fwd", "drsa_amd_projection_fwd", a.data_ptr(), P.U.data_ptr(), P.P.data_ptr(),
                               _capi.ptr(hb), _capi.ptr(ap),
                               _capi.ptr(pooled), _capi.ptr(amax), B, st.cout, h, w, 1 if P.pool_after else 0, s)
                    rec.update(h=hb, ap=ap, amax=amax)
                    if P.pool_after:
                        rec.update(y=pooled, Hout=h // 2, Wout=w // 2)
                        cur, h, w = pooled, h // 2, w // 2
                    else:
                        rec.update(y=ap, Hout=h, Wout=w)
                        cur = ap
                else:
                    rec.update(y=a, Hout=h, Wout=w)
                    cur = a
            state["stages"].append(rec)
        flat = cur.reshape(B, -1)
        if flat.size(1) != self.dense[0].W.size(1):
            raise ValueError(f"flattened trunk output {flat.size(1)} != classifier input {self.dense[0].W.size(1)}")
        state["flat"] = flat
        dense_recs = []
        inp = flat
        for di, ds in enumerate(self.dense):
            N, Kd = ds.W.shape
            z = self._buf(("d", di, "z"), (B, N))
            act = self._buf(("d", di, "a"), (B, N)) if ds.relu_after else None
            self._call(f"linear_fwd:{ds.name}", "drsa_amd_linear_fwd", inp.data_ptr(), ds.W.data_ptr(), _capi.ptr(ds.b), z.data_ptr(),
                       _capi.ptr(act), B, N, Kd, s)
            dense_recs.append({"x": inp, "z": z, "a": act})
            inp = act if act is not None else z
        state["dense"] = dense_recs
        self.last = state
        return dense_recs[-1]["z"]

    # --------------------------------------------------------------- backward
    def _post_for(self, li: int):
        """(post, den, eps) for relevance arriving at the OUTPUT of conv stage li."""
        st = self.stages[li]
        rec = self.last["stages"][li]
        if st.proj is not None:
            return POST_NONE, None, 0.0
        if st.den_kind is None or st.den_kind == "ab":
            return POST_MASK, None, 0.0
        if rec.get("den_map_shared") is not None:
            return POST_DIV_MAP, rec["den_map_shared"], st.eps
        if rec.get("den_const4") is not None:
            return POST_DIV_RING, rec, st.eps        # den = rec["den"] on the ring, rec["den_const4"] elsewhere
        return POST_DIV, rec["den"], st.eps

    @torch.no_grad()
    def backward(self, seed: Optional[torch.Tensor] = None, cls: Optional[torch.Tensor] = None,
                 one_hot: bool = False, fanout: int = 0, stop_after: Optional[int] = None) -> torch.Tensor:
        """Relevance at the input.  ``seed`` [B, n_out] (output relevance) or ``cls`` [B] int32
        (lrp_output_modifier semantics).  ``fanout``: the projection stage emits K+1 clones per
        sample (HeatmapGenerator path); otherwise rows are treated as the reference's
        replicated batch.  ``stop_after``: stop once the relevance at the OUTPUT of conv stage
        ``stop_after`` is known and return it (pool resolution when that stage pools)."""
        st0 = self.last
        if st0 is None:
            raise RuntimeError("backward() before forward()")
        B = st0["B"]
        s = _capi.stream_ptr(self.device)
        self._cur_bufs = self._buffers.setdefault(("bwd", B, fanout), {})
        # ---- dense head, top-down ----
        L = len(self.stages)
        R = seed
        for di in range(len(self.dense) - 1, -1, -1):
            ds, rec = self.dense[di], st0["dense"][di]
            N, Kd = ds.W.shape
            out = self._buf(("d", di), (B, Kd))
            post, den, eps_post = POST_NONE, None, 0.0
            if di == 0:
                post, den, eps_post = self._post_for(L - 1)
                if stop_after == L - 1:
                    post, den, eps_post = POST_NONE, None, 0.0
                x_mask = rec["x"]
            else:
                x_mask = rec["x"]
            relu_mask = 1 if ds.relu_after else 0
            xmode = XM_MUL if ds.rule_kind == "epsilon" else XM_NONE
            den_flat = None if den is None else den.reshape(B, -1)
            if di == len(self.dense) - 1 and cls is not None:
                self._call(f"linear_bwd:{ds.name}", "drsa_amd_linear_bwd", None, cls.data_ptr(), 1 if one_hot else 0, rec["z"].data_ptr(),
                           relu_mask, 1 if ds.rule_kind == "epsilon" else 0, ds.eps, ds.W.data_ptr(),
                           x_mask.data_ptr(), xmode, _capi.ptr(den_flat), post, eps_post, out.data_ptr(), B, N, Kd, s)
            else:
                if R is None:
                    raise ValueError("backward needs a seed or class indices")
                R = R.to(self.device, torch.float32).contiguous()
                self._call(f"linear_bwd:{ds.name}", "drsa_amd_linear_bwd", R.data_ptr(), None, 0, rec["z"].data_ptr(), relu_mask,
                           1 if ds.rule_kind == "epsilon" else 0, ds.eps, ds.W.data_ptr(), x_mask.data_ptr(), xmode,
                           _capi.ptr(den_flat), post, eps_post, out.data_ptr(), B, N, Kd, s)
            R = out
        # ---- conv trunk, top-down ----
        g = R.reshape(B, self.stages[-1].cout, st0["stages"][-1]["Hout"], st0["stages"][-1]["Wout"])
        clones, Bq = 1, B
        for li in range(L - 1, -1, -1):
            if stop_after is not None and li == stop_after:
                return g
            st, rec = self.stages[li], st0["stages"][li]
            h, w = rec["H"], rec["W"]
            amax_in = None
            pool_w = 2          # pool width of a pool-sparse g (4: VGGish (2,4), bf16 backward)
            if st.proj is not None:
                P = st.proj
                K = P.K if P.mask else P.K
                fan = int(fanout) if P.mask else 0
                nq = (K + 1) if fan == 1 else K if fan == 2 else 1
                G = self._buf((li, "G"), (B * nq, st.cout, h, w))
                post, den, eps = ((POST_DIV, rec["den"], st.eps) if st.den_kind not in (None, "ab")
                                  else (POST_MASK, None, 0.0))
                if not P.mask:
                    raise EngineError("engine: projection without SubspaceHook is not supported yet")
                self._call("projection_bwd", "drsa_amd_projection_bwd", g.data_ptr(), _capi.ptr(rec["amax"] if P.pool_after else None),
                           _capi.ptr(rec["ap"] if _PROJ_STORE else None), _capi.ptr(rec["h"]), rec["a"].data_ptr(),
                           _capi.ptr(den if post == POST_DIV else None), P.U.data_ptr(), P.P.data_ptr(), G.data_ptr(),
                           B, st.cout,
                           h, w, K, P.eps_inv, eps, fan, s)
                g, clones, Bq = G, nq, B * nq
            elif st.pool and st.pool_k == (2, 2):
                amax_in = rec["amax"]
            elif (_POOL24_SPARSE and st.pool and st.pool_k == (2, 4) and st.wts_bwd_bf is not None
                  and st.den_kind != "ab" and li > 0
                  and self._post_for(li - 1)[0] != POST_DIV_RING
                  and _capi.lib().drsa_amd_conv_bwd_has_kernel_bf16_pw(st.cout, st.cin, w, 4)):
                # the (2,4) pool backward folded into the bf16 backward's staging (no unpooled g)
                amax_in, pool_w = rec["amax"], 4
            elif (_POOL24_SPARSE and st.pool and st.pool_k == (2, 4) and st.wts_bwd_bf is None and st.den_kind != "ab" and li > 0
                  and stop_after != li - 1 and self._post_for(li - 1)[0] == POST_DIV_MAP
                  and _capi.lib().drsa_amd_conv_bwd_has_kernel_pw(st.cout, st.cin, w, st.ng_bwd, 4)):
                # the same fold in the fp32 backward (VGGish block 1 above the WSquare layer: the den-map
                # backward takes the pooled g and its argmax bytes)
                amax_in, pool_w = rec["amax"], 4
            elif st.pool:
                ph, pw = st.pool_k
                gf = self._buf((li, "g_unpool"), (Bq, st.cout, h, w))
                self._call(f"maxpool_bwd:{st.pool_name}", "drsa_amd_relevance_unpool", g.data_ptr(),
                           rec["amax"].data_ptr(), Bq, clones, st.cout, h, w, ph, pw, gf.data_ptr(), s)
                g = gf
            # rule backward of conv li
            x_in = rec["in"]
            if li > 0:
                post, den, eps = self._post_for(li - 1)
                if stop_after == li - 1:
                    post, den, eps = POST_NONE, None, 0.0
            else:
                post, den, eps = POST_NONE, None, 0.0
            if li == 0 and st.w2_first is not None:
                out = self._buf((li, "R"), (Bq, 1, h, w))
                self._call(f"first_layer_bwd:{st.name}", "drsa_amd_first_layer_bwd", g.data_ptr(), _capi.ptr(amax_in), st.w2_first.data_ptr(),
                           out.data_ptr(), Bq, clones, st.cout, h, w, s)
            elif st.den_kind == "ab":
                # R (ReLU-masked) at the conv output -> gp, gn -> two backward convs -> combine + post
                n_out = g.numel() // Bq
                gp = self._buf((li, "ab_gp"), tuple(g.shape))
                gn = self._buf((li, "ab_gn"), tuple(g.shape))
                self._call(f"ab_split:{st.name}", "drsa_amd_ab_split", g.data_ptr(), rec["den"].data_ptr(),
                           rec["den_n"].data_ptr(), gp.data_ptr(), gn.data_ptr(), Bq, clones, n_out, float(st.eps), s)
                pos = self._buf((li, "ab_pos"), (Bq, st.cin, h, w))
                neg = self._buf((li, "ab_neg"), (Bq, st.cin, h, w))
                for gg, wts, dst in ((gp, st.wts_bwd, pos), (gn, st.wts_bwd_n, neg)):
                    self._call(f"conv_bwd:{st.name}", "drsa_amd_conv_bwd", gg.data_ptr(), _capi.ptr(amax_in),
                               wts.data_ptr(), x_in.data_ptr(), None, dst.data_ptr(), Bq, clones, st.cout, st.cin, h, w,
                               1, XM_MUL, POST_NONE, 0.0, s)
                out = self._buf((li, "R"), (Bq, st.cin, h, w))
                self._call(f"ab_combine:{st.name}", "drsa_amd_ab_combine", pos.data_ptr(), neg.data_ptr(), st.alpha,
                           st.beta, x_in.data_ptr() if post != POST_NONE else None, _capi.ptr(den), out.data_ptr(), Bq,
                           clones, st.cin * h * w, post, float(eps), s)
            elif post == POST_DIV_RING:
                out = self._buf((li, "R"), (Bq, st.cin, h, w))
                bf = st.wts_bwd_bf is not None and _capi.lib().drsa_amd_conv_bwd_has_kernel_bf16(
                    st.cout, st.cin, w, 1, int(amax_in is not None))
                self._call(f"conv_bwd:{st.name}", "drsa_amd_conv_bwd_den_ring", g.data_ptr(), _capi.ptr(amax_in),
                           (st.wts_bwd_bf if bf else st.wts_bwd).data_ptr(), 1 if bf else 0, x_in.data_ptr(),
                           den["den"].data_ptr(), den["den_const4"].data_ptr(), out.data_ptr(), Bq, clones, st.cout,
                           st.cin, h, w, st.ng_bwd, st.xmode_bwd, float(eps), s)
            elif post == POST_DIV_MAP:
                out = self._buf((li, "R"), (Bq, st.cin, h, w))
                bf = st.wts_bwd_bf is not None and (
                    _capi.lib().drsa_amd_conv_bwd_has_kernel_bf16_pw(st.cout, st.cin, w, pool_w) if amax_in is not None
                    else _capi.lib().drsa_amd_conv_bwd_has_kernel_bf16(st.cout, st.cin, w, 1, 0))
                self._call(f"conv_bwd:{st.name}", "drsa_amd_conv_bwd_den_map", g.data_ptr(), _capi.ptr(amax_in), pool_w,
                           (st.wts_bwd_bf if bf else st.wts_bwd).data_ptr(), 1 if bf else 0, x_in.data_ptr(),
                           den.data_ptr(), out.data_ptr(), Bq, clones, st.cout, st.cin, h, w, st.ng_bwd,
                           st.xmode_bwd, float(eps), s)
            elif pool_w == 4:
                out = self._buf((li, "R"), (Bq, st.cin, h, w))
                self._call(f"conv_bwd:{st.name}", "drsa_amd_conv_bwd_bf16_pw", g.data_ptr(), amax_in.data_ptr(), 4,
                           st.wts_bwd_bf.data_ptr(),
                           x_in.data_ptr() if (st.xmode_bwd != XM_NONE or post != POST_NONE) else None,
                           _capi.ptr(den), out.data_ptr(), Bq, clones, st.cout, st.cin, h, w, st.xmode_bwd, post,
                           float(eps), s)
            else:
                out = self._buf((li, "R"), (Bq, st.cin, h, w))
                bf = st.wts_bwd_bf is not None and _capi.lib().drsa_amd_conv_bwd_has_kernel_bf16(
                    st.cout, st.cin, w, 1, int(amax_in is not None))
                self._call(f"conv_bwd:{st.name}", "drsa_amd_conv_bwd_bf16" if bf else "drsa_amd_conv_bwd", g.data_ptr(),
                           _capi.ptr(amax_in), (st.wts_bwd_bf if bf else st.wts_bwd).data_ptr(),
                           x_in.data_ptr() if (st.xmode_bwd != XM_NONE or post != POST_NONE) else None,
                           _capi.ptr(den), out.data_ptr(), Bq, clones, st.cout, st.cin, h, w, st.ng_bwd,
                           st.xmode_bwd, post, float(eps), s)
            g = out
        return g

    # ------------------------------------------------------------ DRSA data
    def capture_stage(self, layer_name: str) -> Tuple[int, str]:
        """(stage index, "relu" | "pool") of a trunk module name (features.<layer_idx>)."""
        for li, st in enumerate(self.stages):
            if st.relu_name == layer_name:
                if st.proj is not None:
                    raise EngineError("engine: capture inside a ProjectionModel layer is not supported")
                return li, "relu"
            if st.pool_name == layer_name and st.proj is None:
                return li, "pool"
        raise EngineError(f"engine: {layer_name} is not a ReLU or MaxPool2d output of the conv trunk "
                          "(DRSA data is captured at ReLU/pool outputs, preprocessing.py:60)")

    @torch.no_grad()
    def capture(self, x: torch.Tensor, layer_name: str, cls: Optional[torch.Tensor] = None, one_hot: bool = False,
                seed_fn=None) -> dict:
        """get_intermediate (preprocessing.py:106-176) for one batch: forward, LRP backward
        down to layer ``layer_name`` only, and that layer's activation and relevance.  The
        relevance of a pooled ReLU output is returned pooled with its argmax (``amax``); the
        activation is the full map."""
        li, where = self.capture_stage(layer_name)
        st = self.stages[li]
        out = self.forward(x, capture=li if (where == "relu" and st.pool) else None)
        rec = self.last["stages"][li]
        if seed_fn is not None:
            R = self.backward(seed=seed_fn(out).contiguous(), stop_after=li)
        else:
            R = self.backward(cls=cls, one_hot=one_hot, stop_after=li)
        ph, pw = st.pool_k
        if where == "pool":
            return {"act": rec["y"], "rel": R, "amax": None, "H": rec["Hout"], "W": rec["Wout"], "C": st.cout,
                    "ph": 1, "pw": 1}
        return {"act": rec["a"], "rel": R, "amax": rec["amax"] if st.pool else None, "H": rec["H"], "W": rec["W"],
                "C": st.cout, "ph": ph, "pw": pw}

    # -------------------------------------------------------------- heatmaps
    @torch.no_grad()
    def subspace_heatmaps(self, x: torch.Tensor, class_idx=None, cls: Optional[torch.Tensor] = None,
                          one_hot: bool = False, standard: str = "sum") -> dict:
        """HeatmapGenerator.generate_subspace_heatmaps on device: one shared forward, the top
        backward once, relevance clones below the projection, then split/sum/sort.
        ``standard="sum"``: K clones, the standard heatmap is the sum of the K concept heatmaps (every
        rule is linear in the relevance, so this is clone 0 up to fp32 rounding; the bottom of the
        network runs K instead of K+1 times).  ``"clone"``: K+1 clones, the standard heatmap is clone
        0 as in the reference's replicated batch (explainer.py:92)."""
        if standard not in ("sum", "clone"):
            raise ValueError("standard must be 'sum' or 'clone'")
        proj = [st.proj for st in self.stages if st.proj is not None]
        if len(proj) != 1 or not proj[0].mask:
            raise EngineError("subspace heatmaps need exactly one projection group with a SubspaceHook")
        K = proj[0].K
        self.forward(x)
        B = x.size(0)
        if cls is None:
            cls = torch.full((B,), int(class_idx), dtype=torch.int32, device=self.device)
        ssum = standard == "sum"
        hm = self.backward(cls=cls, one_hot=one_hot, fanout=2 if ssum else 1)   # [B*(K or K+1), 1, H, W]
        H, W = hm.shape[-2:]
        HW = H * W
        out = {
            "standard_heatmaps": torch.empty(B, 1, H, W, device=self.device),
            "standard_relevance": torch.empty(B, device=self.device),
            "subspace_heatmaps": torch.empty(B, K, H, W, device=self.device),
            "subspace_relevances": torch.empty(B, K, device=self.device),
            "mask": torch.empty(B, K, dtype=torch.int64, device=self.device),
        }
        self._call("heatmap_sort", "drsa_amd_heatmap_sort", hm.data_ptr(), B, K, HW, 1 if ssum else 0,
                   out["standard_heatmaps"].data_ptr(), out["standard_relevance"].data_ptr(),
                   out["subspace_heatmaps"].data_ptr(), out["subspace_relevances"].data_ptr(), out["mask"].data_ptr(),
                   _capi.stream_ptr(self.device))
        return out


def bf16_backward_default() -> bool:
    """DRSA_AMD_BF16_BACKWARD=1: bf16 plans also run the relevance backward convs on bf16 operands."""
    return os.environ.get("DRSA_AMD_BF16_BACKWARD", "0") not in ("", "0")


def _bf16r(t: torch.Tensor) -> torch.Tensor:
    """Round to bf16 (nearest even) and back: the values a bf16 plan's kernels see."""
    return t.to(torch.bfloat16).to(t.dtype)


def _bf16_layout(wf: torch.Tensor, cin_p: int, cout_p: int) -> torch.Tensor:
    """[ng][9*cin_p][cout_p] fp32 (row k = ci*9 + tap) -> [ng][cin_p/16][9][2][cout_p][8] bf16,
    input channel ci = 16*chunk + 8*half + j (drsa_amd_conv_fwd_bf16, include/drsa_amd.h)."""
    ng = wf.size(0)
    t = wf.reshape(ng, cin_p // 16, 2, 8, 9, cout_p).permute(0, 1, 4, 2, 5, 3)
    return t.to(torch.bfloat16).contiguous()


def _bn_to(bn, device):
    class _B:   # detached fp32 copies of the BN statistics
        pass
    o = _B()
    o.running_var = bn.running_var.detach().to(device, torch.float32)
    o.running_mean = bn.running_mean.detach().to(device, torch.float32)
    o.weight = (bn.weight.detach() if bn.weight is not None else torch.ones_like(bn.running_var)).to(device, torch.float32)
    o.bias = (bn.bias.detach() if bn.bias is not None else torch.zeros_like(bn.running_var)).to(device, torch.float32)
    o.eps = bn.eps
    return o
