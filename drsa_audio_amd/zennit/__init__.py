"""Zennit-0.5.1-compatible front end (rules, composites, canonizers, attribution).

The reference builds explanations with zennit (``requirements.txt:23``), which is absent
here.  This namespace keeps the names and signatures the reference's code uses
(``constants.py:1,27-51``, ``attribute.py:7-9,98-107``, ``explainer.py:6-7,198-203``,
``getdrsadata.py:9-13,81-114``) so that name maps and ``SubspaceHook`` code run
unchanged, but rules are *descriptors*: ``attribution.Gradient`` compiles the model and
the composite into a HIP kernel plan (``drsa_audio_amd.engine``) instead of attaching
autograd hooks.
"""
from . import attribution, canonizers, composites, core, rules  # noqa: F401
