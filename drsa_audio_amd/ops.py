"""PyTorch-ROCm custom ops over the C ABI (SURVEY 8(b) "Native op layer").

``import drsa_audio_amd.ops`` loads ``lib/libdrsa_amd_torch.so``, whose C++ ``TORCH_LIBRARY(drsa_amd,
m)`` registers the namespace ``torch.ops.drsa_amd`` with one op per hot-path stage
(``csrc_torch/ops_torch.cpp``): TorchScript and C++ callers see the same operators.  Each op
launches the HIP kernels of ``libdrsa_amd.so`` on the current HIP stream (so ops compose with
torch streams and are capturable in a CUDA/HIP graph: no host synchronisation inside any of them)
and allocates its outputs with the torch caching allocator.  This module adds the fake (meta)
implementations for tracing / ``torch.compile`` and the front-end op ``logmel`` (its filterbank
setup is host Python).  Error behaviour: argument errors raise ``RuntimeError`` with the library's
message; there is no CPU kernel (a CPU tensor raises); a missing ``libdrsa_amd_torch.so`` raises
``DrsaAmdError`` at import.

  drsa_amd::drsa_step(A, C, U, K) -> (U_new, f)             drsa.py:84-106 (one run iteration)
  drsa_amd::drsa_objective(A, C, U, K) -> f                  drsa.py:122-155 + 224-238
  drsa_amd::drsa_run(A, C, U0, K, steps) -> (U, traj)        drsa.py:76-120 (traj: steps+1)
  drsa_amd::polar(V) -> U                                    drsa.py:201-221 (orthogonalize)
  drsa_amd::subspace_relevances(act, ctx, U, K) -> r         explainer.py:206-242
  drsa_amd::lrp_conv_fwd(x, wts, bias3, den_map?, cout, ng, pool) -> (y, amax, den)
  drsa_amd::lrp_conv_bwd(g, amax?, wts, x?, den?, cin, H, W, clones, ng, xmode, post, eps) -> R
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

import os

import torch
from torch import Tensor

from . import _capi

_NS = "drsa_amd"
TORCH_LIB_PATH = os.path.join(os.path.dirname(_capi.LIB_PATH), "libdrsa_amd_torch.so")


def _load_torch_library() -> None:
    if not os.path.exists(TORCH_LIB_PATH):
        raise _capi.DrsaAmdError(f"{TORCH_LIB_PATH} is missing: build it with drsa_audio_amd.build "
                                 "(__graft_entry__.build())")
    _capi.load()                      # libdrsa_amd.so first (the op library links it)
    torch.ops.load_library(TORCH_LIB_PATH)


_load_torch_library()
_ops = getattr(torch.ops, _NS)


def _s(t: Tensor) -> int:
    return _capi.stream_ptr(t.device)


def _chk(t: Tensor, name: str, dtype=torch.float32) -> Tensor:
    _capi.require_gpu(t, name, dtype=dtype)
    return t


def _fake(name):
    return torch.library.register_fake(f"{_NS}::{name}")


# ------------------------------------------------------------------ fake kernels (C++ ops)
@_fake("drsa_step")
def _(A, C, U, K):
    return torch.empty_like(U), U.new_empty(())


@_fake("drsa_objective")
def _(A, C, U, K):
    return U.new_empty(())


@_fake("drsa_run")
def _(A, C, U0, K, steps):
    return torch.empty_like(U0), U0.new_empty(steps + 1)


@_fake("polar")
def _(V):
    return torch.empty_like(V)


@_fake("subspace_relevances")
def _(act, ctx, U, K):
    b = act.shape[0] if act.dim() == 3 else 1
    return act.new_empty(b, K, dtype=torch.float32)


@_fake("lrp_conv_fwd")
def _(x, wts, bias3, den_map, cout, ng, pool):
    B, cin, H, W = x.shape
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    amax = x.new_empty(B, cout, Ho, Wo, dtype=torch.uint8) if pool else x.new_empty(0, dtype=torch.uint8)
    return x.new_empty(B, cout, Ho, Wo), amax, x.new_empty(B, cout, Ho, Wo)


@_fake("lrp_conv_bwd")
def _(g, amax, wts, x, den, cin, H, W, clones, ng, xmode, post, eps):
    return g.new_empty(g.shape[0], cin, H, W)


@_fake("lrp_linear_fwd")
def _(x, W, b, relu):
    return x.new_empty(x.shape[0], W.shape[0]), (x.new_empty(x.shape[0], W.shape[0]) if relu else x.new_empty(0))


@_fake("lrp_linear_bwd")
def _(R, cls, one_hot, z, relu_mask, rule_eps, eps, W, x, xmode, den, post, eps_post):
    return z.new_empty(z.shape[0], W.shape[1])


@_fake("projection_fwd")
def _(a, U, pool):
    B, D, H, W = a.shape
    if pool:
        return a.new_empty(B, D, H // 2, W // 2), a.new_empty(B, D, H // 2, W // 2, dtype=torch.uint8)
    return torch.empty_like(a), a.new_empty(0, dtype=torch.uint8)


@_fake("projection_bwd")
def _(g, amax, a, den, U, K, eps_proj, eps_den, fanout):
    B, D, H, W = a.shape
    return a.new_empty(B * ((K + 1) if fanout else 1), D, H, W)


@_fake("heatmap_sort")
def _(hm, K, std_from_sum=False):
    H, W = hm.shape[-2:]
    B = hm.numel() // ((K if std_from_sum else K + 1) * H * W)
    return (hm.new_empty(B, 1, H, W), hm.new_empty(B), hm.new_empty(B, K, H, W), hm.new_empty(B, K),
            hm.new_empty(B, K, dtype=torch.int64))


drsa_step = _ops.drsa_step
drsa_objective = _ops.drsa_objective
drsa_run = _ops.drsa_run
polar = _ops.polar
subspace_relevances = _ops.subspace_relevances
lrp_conv_fwd = _ops.lrp_conv_fwd
lrp_conv_bwd = _ops.lrp_conv_bwd
lrp_linear_fwd = _ops.lrp_linear_fwd
lrp_linear_bwd = _ops.lrp_linear_bwd
projection_fwd = _ops.projection_fwd
projection_bwd = _ops.projection_bwd
heatmap_sort = _ops.heatmap_sort


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
