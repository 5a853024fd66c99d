"""HIP LRP engine: plan compilation + execution (see ``plan.py``).

``get_engine`` caches compiled plans per (model, composite) while the model's parameters are
unchanged.  The cache holds the model and the composite only through weak references (the
engine itself keeps no strong reference to either), drops an entry as soon as its model or
composite is garbage-collected, and keeps at most ``DRSA_AMD_ENGINE_CACHE`` (default 8) entries
in LRU order; an evicted engine releases its device buffers.  So a workflow that builds a new
``HeatmapGenerator`` per pass (the reference does, cxai/xai/pixelflipping/cpf.py:161) keeps a
bounded device footprint.  A composite that maps a module to a user-written ``Hook`` (its own
``backward``) gets the autograd slow path ``HookedAutograd`` (``hooks.py``) instead of a plan.
"""
from __future__ import annotations

import os
import weakref
from collections import OrderedDict

import torch

from .hooks import HookedAutograd, has_custom_hooks
from .plan import EngineError, LRPEngine, bf16_backward_default

_MAX = max(1, int(os.environ.get("DRSA_AMD_ENGINE_CACHE", "8")))
_CACHE: "OrderedDict[tuple, _Entry]" = OrderedDict()


class _Entry:
    __slots__ = ("model_ref", "comp_ref", "fp", "eng", "finalizers")

    def __init__(self, model_ref, comp_ref, fp, eng):
        self.model_ref, self.comp_ref, self.fp, self.eng = model_ref, comp_ref, fp, eng
        self.finalizers = []


def _fingerprint(model):
    """Parameters AND buffers: the plan folds BatchNorm running statistics into the weights, so a
    train-mode forward or a buffers-only load_state_dict must recompile.  Also the DRSA projection
    matrices, which are plain tensor attributes (``Projection.U``, ``InvProjection.U_inv``,
    ``ProjectionModel.U``; cxai/model/modify_model.py:4-123): the plan caches U and P = UU^T - I, so
    an in-place update (``_version``) or a rebinding (``data_ptr``) of U must recompile too."""
    proj = []
    for m in model.modules():
        for attr in ("U", "U_inv"):
            t = getattr(m, attr, None)
            if isinstance(t, torch.Tensor):
                proj.append((attr, t.data_ptr(), t._version))
    return (tuple((p.data_ptr(), p._version) for p in model.parameters()) +
            tuple((b.data_ptr(), b._version) for b in model.buffers()) + tuple(proj))


def _ref(obj):
    if obj is None:
        return lambda: None
    return weakref.ref(obj)


def _evict(key) -> None:
    e = _CACHE.pop(key, None)
    if e is not None:
        for f in e.finalizers:        # one live finalizer per cached entry, never a pile-up
            f.detach()
        e.eng.release()


def get_engine(model, composite) -> LRPEngine:
    """Compiled plan for (model, composite), cached while the model's parameters are unchanged."""
    key = (id(model), id(composite))
    fp = (_fingerprint(model), bf16_backward_default())   # the option selects different kernels
    e = _CACHE.get(key)
    if e is not None:
        if e.model_ref() is model and e.comp_ref() is composite and e.fp == fp:
            _CACHE.move_to_end(key)
            return e.eng
        _evict(key)          # stale: ids reused by new objects, or the weights changed
    rules = composite.rules(model) if composite is not None else {}
    # a composite with a user-written Hook (its own backward) cannot be compiled: autograd slow path
    eng = HookedAutograd(model, composite) if has_custom_hooks(rules) else LRPEngine(model, composite)
    entry = _Entry(_ref(model), _ref(composite), fp, eng)
    _CACHE[key] = entry
    entry.finalizers.append(weakref.finalize(model, _evict, key))
    if composite is not None:
        entry.finalizers.append(weakref.finalize(composite, _evict, key))
    while len(_CACHE) > _MAX:
        _evict(next(iter(_CACHE)))
    return eng


def cache_size() -> int:
    return len(_CACHE)


def clear_cache() -> None:
    for key in list(_CACHE):
        _evict(key)


__all__ = ["LRPEngine", "HookedAutograd", "EngineError", "get_engine", "cache_size", "clear_cache"]
