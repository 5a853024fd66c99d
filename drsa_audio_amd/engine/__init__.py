"""HIP LRP engine: plan compilation + execution (see ``plan.py``)."""
from __future__ import annotations

from .plan import EngineError, LRPEngine

_CACHE = {}


def _fingerprint(model):
    return tuple((p.data_ptr(), p._version) for p in model.parameters())


def get_engine(model, composite) -> LRPEngine:
    """Compiled plan for (model, composite), cached while the model's parameters are unchanged."""
    key = (id(model), id(composite))
    fp = _fingerprint(model)
    hit = _CACHE.get(key)
    if hit is not None and hit[0] == fp and hit[1].model is model and hit[1].composite is composite:
        return hit[1]
    eng = LRPEngine(model, composite)
    _CACHE[key] = (fp, eng)
    return eng


__all__ = ["LRPEngine", "EngineError", "get_engine"]
