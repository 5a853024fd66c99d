"""Composites (zennit.composites): declarative maps from modules to rules."""
from __future__ import annotations

import contextlib
from typing import List, Optional, Sequence, Tuple

import torch.nn as nn


class Composite:
    """Base composite: ``module_map(ctx, name, module) -> rule or None``."""

    def __init__(self, module_map=None, canonizers=None):
        self._module_map = module_map
        self.canonizers = list(canonizers or [])

    def rule_for(self, name: str, module: nn.Module):
        if self._module_map is None:
            return None
        return self._module_map({}, name, module)

    def rules(self, model: nn.Module) -> dict:
        return {n: r for n, m in model.named_modules() if (r := self.rule_for(n, m)) is not None}

    @contextlib.contextmanager
    def context(self, module):
        yield module

    def register(self, module):
        return None

    def remove(self):
        return None


class NameMapComposite(Composite):
    """``name_map = [([module names], rule), ...]`` (reference constants.py:27-51)."""

    def __init__(self, name_map: Sequence[Tuple[Sequence[str], object]], canonizers=None):
        super().__init__(canonizers=canonizers)
        self.name_map = list(name_map)
        self._by_name = {}
        for names, rule in self.name_map:
            for n in names:
                self._by_name[n] = rule

    def rule_for(self, name: str, module: nn.Module):
        return self._by_name.get(name)


class LayerMapComposite(Composite):
    """``layer_map = [(module type, rule), ...]``: first matching type wins."""

    def __init__(self, layer_map, canonizers=None):
        super().__init__(canonizers=canonizers)
        self.layer_map = list(layer_map)

    def rule_for(self, name: str, module: nn.Module):
        for typ, rule in self.layer_map:
            if isinstance(module, typ):
                return rule
        return None


class SpecialFirstLayerMapComposite(LayerMapComposite):
    """Like LayerMapComposite, but the first matching layer gets ``first_map``."""

    def __init__(self, layer_map, first_map, canonizers=None):
        super().__init__(layer_map, canonizers=canonizers)
        self.first_map = list(first_map)
        self._first = None

    def rules(self, model: nn.Module) -> dict:
        out = {}
        first_done = False
        for n, m in model.named_modules():
            if not first_done:
                for typ, rule in self.first_map:
                    if isinstance(m, typ):
                        out[n] = rule
                        first_done = True
                        break
                if first_done and n in out:
                    continue
            r = LayerMapComposite.rule_for(self, n, m)
            if r is not None:
                out[n] = r
        return out

    def rule_for(self, name, module):
        raise RuntimeError("SpecialFirstLayerMapComposite resolves rules per model; use .rules(model)")


class NameLayerMapComposite(Composite):
    """zennit NameLayerMapComposite (used at reference pf.py:219-227): a module's rule comes from
    ``name_map`` if its name is listed there, else from ``layer_map`` (first matching type)."""

    def __init__(self, name_map=None, layer_map=None, canonizers=None):
        super().__init__(canonizers=canonizers)
        self.name_map_composite = NameMapComposite(name_map or [])
        self.layer_map_composite = LayerMapComposite(layer_map or [])

    def rule_for(self, name: str, module: nn.Module):
        r = self.name_map_composite.rule_for(name, module)
        return r if r is not None else self.layer_map_composite.rule_for(name, module)
