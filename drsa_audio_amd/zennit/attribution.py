"""``Gradient`` attributor (zennit.attribution.Gradient) backed by the HIP LRP engine.

``with Gradient(model, composite) as attributor: output, relevance = attributor(x, attr_output)``
(reference call sites attribute.py:98-107, preprocessing.py:143-162).  ``attr_output`` is a
callable mapping the (detached) model output to the output relevance, or a tensor.
"""
from __future__ import annotations

from typing import Callable, Optional, Union

import torch


class Attributor:
    def __init__(self, model, composite=None, attr_output=None):
        self.model = model
        self.composite = composite
        self.attr_output = attr_output
        self.engine = None

    def __enter__(self):
        from ..engine import get_engine
        self.engine = get_engine(self.model, self.composite)
        return self

    def __exit__(self, *exc):
        return False

    def __call__(self, input: torch.Tensor, attr_output=None):
        if self.engine is None:
            with self:
                return self.forward(input, attr_output)
        return self.forward(input, attr_output)

    def forward(self, input, attr_output):
        raise NotImplementedError


class Gradient(Attributor):
    def __init__(self, model, composite=None, attr_output=None, create_graph=False, retain_graph=None):
        if create_graph:
            raise NotImplementedError("create_graph is not supported by the HIP engine")
        super().__init__(model, composite, attr_output)

    def forward(self, input: torch.Tensor, attr_output=None):
        fn = attr_output if attr_output is not None else self.attr_output
        out = self.engine.forward(input)
        if fn is None:
            seed = torch.ones_like(out)
        elif callable(fn):
            seed = fn(out.detach())
        else:
            seed = torch.as_tensor(fn, device=out.device, dtype=out.dtype).expand_as(out).contiguous()
        relevance = self.engine.backward(seed=seed.contiguous())
        # the engine's output buffers are reused by its next call: hand out copies (the
        # reference returns fresh tensors; results of consecutive calls must not alias)
        return out.clone(), relevance.clone()
