"""Pixel / concept flipping evaluation (reference cxai/xai/pixelflipping): ``Flipper`` (core.py),
``PixelFlipping`` (pf.py), ``concept_flipping`` (cpf.py)."""
from .core import Flipper
from .pf import PixelFlipping, rule_mapper
from .cpf import concept_flipping

__all__ = ["Flipper", "PixelFlipping", "rule_mapper", "concept_flipping"]
