"""PyTorch-ROCm custom ops over the C ABI (SURVEY 8(b) "Native op layer").

``import drsa_audio_amd.ops`` registers the namespace ``torch.ops.drsa_amd`` with one op per
hot-path stage.  Each op launches the HIP kernels of ``libdrsa_amd.so`` on the current HIP stream
(so ops compose with torch streams and are capturable in a CUDA/HIP graph: no host
synchronisation inside any of them), allocates its outputs with the torch caching allocator, and
has a fake (meta) implementation for tracing / ``torch.compile``.  Error behaviour: argument
errors raise ``DrsaAmdError`` (a ``RuntimeError``) with the library's message; there is no CPU
kernel (a CPU tensor raises).

  drsa_amd::drsa_step(A, C, U, K) -> (U_new, f)             drsa.py:84-106 (one run iteration)
  drsa_amd::drsa_objective(A, C, U, K) -> f                  drsa.py:122-155 + 224-238
  drsa_amd::drsa_run(A, C, U0, K, steps) -> (U, traj)        drsa.py:76-120 (traj: steps+1)
  drsa_amd::polar(V) -> U                                    drsa.py:201-221 (orthogonalize)
  drsa_amd::subspace_relevances(act, ctx, U, K) -> r         explainer.py:206-242
  drsa_amd::lrp_conv_fwd(x, wts, bias3, den_map?, cout, ng, pool) -> (y, amax, den)
  drsa_amd::lrp_conv_bwd(g, amax?, wts, x?, den?, cin, clones, ng, xmode, post, eps) -> R
  drsa_amd::lrp_linear_fwd(x, W, b?, relu) -> (z, a)
  drsa_amd::lrp_linear_bwd(R?, cls?, one_hot, z, relu_mask, rule_eps, eps, W, x, xmode, den?, post,
                           eps_post) -> out
  drsa_amd::projection_fwd(a, U, pool) -> (ap_or_pooled, amax)
  drsa_amd::projection_bwd(g, amax?, a, den?, U, K, eps_proj, eps_den, fanout) -> G
  drsa_amd::heatmap_sort(hm, K, std_from_sum) -> (std, std_rel, sub, rel, mask)   explainer.py:99-123, 151-176
  drsa_amd::logmel(wav, n_fft, hop, n_mels, width, peak_norm) -> mel  dataloading.py:138-176
The LRP stage ops take the engine's prepared weight layouts (engine/plan.py); the DRSA and
front-end ops take the reference's tensors directly.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import _capi
from ._capi import POST_DIV, POST_MASK, POST_NONE, XM_NONE

_NS = "drsa_amd"


def _s(t: Tensor) -> int:
    return _capi.stream_ptr(t.device)


def _chk(t: Tensor, name: str, dtype=torch.float32) -> Tensor:
    _capi.require_gpu(t, name, dtype=dtype)
    return t


# ----------------------------------------------------------------------------------- DRSA
@torch.library.custom_op(f"{_NS}::drsa_step", mutates_args=())
def drsa_step(A: Tensor, C: Tensor, U: Tensor, K: int) -> Tuple[Tensor, Tensor]:
    from .xai.drsa.drsa import drsa_step as _step
    U_new, f = _step(A, C, U, K)
    return U_new, f.reshape(())


@drsa_step.register_fake
def _(A, C, U, K):
    return torch.empty_like(U), U.new_empty(())


@torch.library.custom_op(f"{_NS}::drsa_objective", mutates_args=())
def drsa_objective(A: Tensor, C: Tensor, U: Tensor, K: int) -> Tensor:
    from .xai.drsa.drsa import drsa_objective as _obj
    return _obj(A, C, U, K).reshape(())


@drsa_objective.register_fake
def _(A, C, U, K):
    return U.new_empty(())


@torch.library.custom_op(f"{_NS}::drsa_run", mutates_args=())
def drsa_run(A: Tensor, C: Tensor, U0: Tensor, K: int, steps: int) -> Tuple[Tensor, Tensor]:
    from .xai.drsa.drsa import drsa_run as _run
    # inside a stream capture the library records the plain launch sequence (no nested graph)
    U, traj = _run(A, C, U0, K, steps)
    return U, traj


@drsa_run.register_fake
def _(A, C, U0, K, steps):
    return torch.empty_like(U0), U0.new_empty(steps + 1)


@torch.library.custom_op(f"{_NS}::polar", mutates_args=())
def polar(V: Tensor) -> Tensor:
    from .xai.drsa.drsa import orthogonalize
    return orthogonalize(V.contiguous())


@polar.register_fake
def _(V):
    return torch.empty_like(V)


@torch.library.custom_op(f"{_NS}::subspace_relevances", mutates_args=())
def subspace_relevances(act: Tensor, ctx: Tensor, U: Tensor, K: int) -> Tensor:
    from .xai.explain.explainer import compute_subspace_relevances
    return compute_subspace_relevances(act, ctx, U, K)


@subspace_relevances.register_fake
def _(act, ctx, U, K):
    b = act.shape[0] if act.dim() == 3 else 1
    return act.new_empty(b, K)


# ------------------------------------------------------------------------------ LRP stages
@torch.library.custom_op(f"{_NS}::lrp_conv_fwd", mutates_args=())
def lrp_conv_fwd(x: Tensor, wts: Tensor, bias3: Tensor, den_map: Optional[Tensor], cout: int, ng: int,
                 pool: bool) -> Tuple[Tensor, Tensor, Tensor]:
    _chk(x, "x"), _chk(wts, "wts"), _chk(bias3, "bias3")
    B, cin, H, W = x.shape
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    y = x.new_empty(B, cout, Ho, Wo)
    amax = torch.empty(B, cout, Ho, Wo, dtype=torch.uint8, device=x.device) if pool else x.new_empty(0, dtype=torch.uint8)
    den = x.new_empty(B, cout, Ho, Wo)
    _capi.call("drsa_amd_conv_fwd", x.data_ptr(), wts.data_ptr(), bias3.data_ptr(), _capi.ptr(den_map), y.data_ptr(),
               amax.data_ptr() if pool else None, den.data_ptr(), B, cin, cout, H, W, ng, 1 if pool else 0, _s(x))
    return y, amax, den


@lrp_conv_fwd.register_fake
def _(x, wts, bias3, den_map, cout, ng, pool):
    B, cin, H, W = x.shape
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    amax = x.new_empty(B, cout, Ho, Wo, dtype=torch.uint8) if pool else x.new_empty(0, dtype=torch.uint8)
    return x.new_empty(B, cout, Ho, Wo), amax, x.new_empty(B, cout, Ho, Wo)


@torch.library.custom_op(f"{_NS}::lrp_conv_bwd", mutates_args=())
def lrp_conv_bwd(g: Tensor, amax: Optional[Tensor], wts: Tensor, x: Optional[Tensor], den: Optional[Tensor], cin: int,
                 H: int, W: int, clones: int, ng: int, xmode: int, post: int, eps: float) -> Tensor:
    _chk(g, "g"), _chk(wts, "wts")
    Bq, cout = g.shape[0], g.shape[1]
    out = g.new_empty(Bq, cin, H, W)
    _capi.call("drsa_amd_conv_bwd", g.data_ptr(), _capi.ptr(amax), wts.data_ptr(), _capi.ptr(x), _capi.ptr(den),
               out.data_ptr(), Bq, clones, cout, cin, H, W, ng, xmode, post, float(eps), _s(g))
    return out


@lrp_conv_bwd.register_fake
def _(g, amax, wts, x, den, cin, H, W, clones, ng, xmode, post, eps):
    return g.new_empty(g.shape[0], cin, H, W)


@torch.library.custom_op(f"{_NS}::lrp_linear_fwd", mutates_args=())
def lrp_linear_fwd(x: Tensor, W: Tensor, b: Optional[Tensor], relu: bool) -> Tuple[Tensor, Tensor]:
    _chk(x, "x"), _chk(W, "W")
    M, K = x.shape
    N = W.shape[0]
    z = x.new_empty(M, N)
    a = x.new_empty(M, N) if relu else x.new_empty(0)
    _capi.call("drsa_amd_linear_fwd", x.data_ptr(), W.data_ptr(), _capi.ptr(b), z.data_ptr(),
               a.data_ptr() if relu else None, M, N, K, _s(x))
    return z, a


@lrp_linear_fwd.register_fake
def _(x, W, b, relu):
    return x.new_empty(x.shape[0], W.shape[0]), (x.new_empty(x.shape[0], W.shape[0]) if relu else x.new_empty(0))


@torch.library.custom_op(f"{_NS}::lrp_linear_bwd", mutates_args=())
def lrp_linear_bwd(R: Optional[Tensor], cls: Optional[Tensor], one_hot: bool, z: Tensor, relu_mask: bool,
                   rule_eps: bool, eps: float, W: Tensor, x: Tensor, xmode: int, den: Optional[Tensor], post: int,
                   eps_post: float) -> Tensor:
    _chk(z, "z"), _chk(W, "W"), _chk(x, "x")
    M, Nout = z.shape
    Kin = W.shape[1]
    out = z.new_empty(M, Kin)
    _capi.call("drsa_amd_linear_bwd", _capi.ptr(R), _capi.ptr(cls), 1 if one_hot else 0, z.data_ptr(),
               1 if relu_mask else 0, 1 if rule_eps else 0, float(eps), W.data_ptr(), x.data_ptr(), xmode,
               _capi.ptr(den), post, float(eps_post), out.data_ptr(), M, Nout, Kin, _s(z))
    return out


@lrp_linear_bwd.register_fake
def _(R, cls, one_hot, z, relu_mask, rule_eps, eps, W, x, xmode, den, post, eps_post):
    return z.new_empty(z.shape[0], W.shape[1])


def _residual(U: Tensor) -> Tensor:
    """P = U U^T - I for the projection kernels (drsa_amd_projection_residual)."""
    P = torch.empty_like(U)
    _capi.call("drsa_amd_projection_residual", U.data_ptr(), U.size(0), P.data_ptr(), _s(U))
    return P


@torch.library.custom_op(f"{_NS}::projection_fwd", mutates_args=())
def projection_fwd(a: Tensor, U: Tensor, pool: bool) -> Tuple[Tensor, Tensor]:
    _chk(a, "a"), _chk(U, "U")
    B, D, H, W = a.shape
    P = _residual(U)
    if pool:
        y = a.new_empty(B, D, H // 2, W // 2)
        amax = torch.empty(B, D, H // 2, W // 2, dtype=torch.uint8, device=a.device)
        _capi.call("drsa_amd_projection_fwd", a.data_ptr(), U.data_ptr(), P.data_ptr(), None, None, y.data_ptr(),
                   amax.data_ptr(), B, D, H, W, 1, _s(a))
    else:
        y = torch.empty_like(a)
        amax = torch.empty(0, dtype=torch.uint8, device=a.device)
        _capi.call("drsa_amd_projection_fwd", a.data_ptr(), U.data_ptr(), P.data_ptr(), None, y.data_ptr(), None,
                   None, B, D, H, W, 0, _s(a))
    return y, amax


@projection_fwd.register_fake
def _(a, U, pool):
    B, D, H, W = a.shape
    if pool:
        return a.new_empty(B, D, H // 2, W // 2), a.new_empty(B, D, H // 2, W // 2, dtype=torch.uint8)
    return torch.empty_like(a), a.new_empty(0, dtype=torch.uint8)


@torch.library.custom_op(f"{_NS}::projection_bwd", mutates_args=())
def projection_bwd(g: Tensor, amax: Optional[Tensor], a: Tensor, den: Optional[Tensor], U: Tensor, K: int,
                   eps_proj: float, eps_den: float, fanout: bool) -> Tensor:
    _chk(g, "g"), _chk(a, "a"), _chk(U, "U")
    B, D, H, W = a.shape
    nq = (K + 1) if fanout else 1
    G = a.new_empty(B * nq, D, H, W)
    P = _residual(U)
    _capi.call("drsa_amd_projection_bwd", g.data_ptr(), _capi.ptr(amax), None, None, a.data_ptr(), _capi.ptr(den),
               U.data_ptr(), P.data_ptr(), G.data_ptr(), B, D, H, W, K, float(eps_proj), float(eps_den),
               1 if fanout else 0, _s(a))
    return G


@projection_bwd.register_fake
def _(g, amax, a, den, U, K, eps_proj, eps_den, fanout):
    B, D, H, W = a.shape
    return a.new_empty(B * ((K + 1) if fanout else 1), D, H, W)


@torch.library.custom_op(f"{_NS}::heatmap_sort", mutates_args=())
def heatmap_sort(hm: Tensor, K: int, std_from_sum: bool = False) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    _chk(hm, "hm")
    H, W = hm.shape[-2:]
    B = hm.numel() // ((K if std_from_sum else K + 1) * H * W)
    std = hm.new_empty(B, 1, H, W)
    std_rel = hm.new_empty(B)
    sub = hm.new_empty(B, K, H, W)
    rel = hm.new_empty(B, K)
    mask = torch.empty(B, K, dtype=torch.int64, device=hm.device)
    _capi.call("drsa_amd_heatmap_sort", hm.data_ptr(), B, K, H * W, 1 if std_from_sum else 0, std.data_ptr(),
               std_rel.data_ptr(), sub.data_ptr(),
               rel.data_ptr(), mask.data_ptr(), _s(hm))
    return std, std_rel, sub, rel, mask


@heatmap_sort.register_fake
def _(hm, K, std_from_sum=False):
    H, W = hm.shape[-2:]
    B = hm.numel() // ((K if std_from_sum else K + 1) * H * W)
    return (hm.new_empty(B, 1, H, W), hm.new_empty(B), hm.new_empty(B, K, H, W), hm.new_empty(B, K),
            hm.new_empty(B, K, dtype=torch.int64))


# ------------------------------------------------------------------------------ front end
_LOADERS = {}


@torch.library.custom_op(f"{_NS}::logmel", mutates_args=())
def logmel(wav: Tensor, n_fft: int, hop: int, n_mels: int, width: int, peak_norm: bool) -> Tensor:
    """Rows of `wav` [R, L] -> [R, 1, n_mels, width] (Loader.transform_wav; peak_normalizer first
    when peak_norm, as Loader.load does)."""
    from .utils.dataloading import Loader
    key = (n_fft, hop, n_mels, width, str(wav.device))
    ld = _LOADERS.get(key)
    if ld is None:
        ld = _LOADERS[key] = Loader(None, n_fft=n_fft, hop_length=hop, n_mels=n_mels, width=width, device=wav.device)
    w = _chk(wav.contiguous(), "wav")
    return ld._run(w, w.shape[0], w.shape[1], 1, 0, w.shape[1], peak_norm, True)


@logmel.register_fake
def _(wav, n_fft, hop, n_mels, width, peak_norm):
    return wav.new_empty(wav.shape[0], 1, n_mels, width)


__all__ = ["drsa_step", "drsa_objective", "drsa_run", "polar", "subspace_relevances", "lrp_conv_fwd", "lrp_conv_bwd",
           "lrp_linear_fwd", "lrp_linear_bwd", "projection_fwd", "projection_bwd", "heatmap_sort", "logmel"]
