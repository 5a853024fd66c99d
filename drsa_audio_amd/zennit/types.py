"""Abstract layer types (zennit.types, used by LayerMapComposite maps, e.g. reference
pf.py:215-236): ``isinstance(module, Convolution)`` etc. without a common base class.
As in zennit, ``Linear`` covers dense AND convolution layers (so map order matters:
the reference lists Convolution before Linear)."""
from __future__ import annotations

import torch.nn as nn


class _SubclassMeta(type):
    def __instancecheck__(cls, inst):
        return isinstance(inst, cls.__subclass__)

    def __subclasscheck__(cls, sub):
        return issubclass(sub, cls.__subclass__)


class ConvolutionStandard(metaclass=_SubclassMeta):
    __subclass__ = (nn.Conv1d, nn.Conv2d, nn.Conv3d)


class ConvolutionTranspose(metaclass=_SubclassMeta):
    __subclass__ = (nn.ConvTranspose1d, nn.ConvTranspose2d, nn.ConvTranspose3d)


class Convolution(metaclass=_SubclassMeta):
    __subclass__ = ConvolutionStandard.__subclass__ + ConvolutionTranspose.__subclass__


class Linear(metaclass=_SubclassMeta):
    __subclass__ = (nn.Linear,) + Convolution.__subclass__


class BatchNorm(metaclass=_SubclassMeta):
    __subclass__ = (nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d)


class AvgPool(metaclass=_SubclassMeta):
    __subclass__ = (nn.AvgPool1d, nn.AvgPool2d, nn.AvgPool3d, nn.AdaptiveAvgPool1d, nn.AdaptiveAvgPool2d,
                    nn.AdaptiveAvgPool3d)


class MaxPool(metaclass=_SubclassMeta):
    __subclass__ = (nn.MaxPool1d, nn.MaxPool2d, nn.MaxPool3d, nn.AdaptiveMaxPool1d, nn.AdaptiveMaxPool2d,
                    nn.AdaptiveMaxPool3d)


class Activation(metaclass=_SubclassMeta):
    __subclass__ = (nn.ELU, nn.Hardshrink, nn.Hardsigmoid, nn.Hardtanh, nn.Hardswish, nn.LeakyReLU, nn.LogSigmoid,
                    nn.PReLU, nn.ReLU, nn.ReLU6, nn.RReLU, nn.SELU, nn.CELU, nn.GELU, nn.Sigmoid, nn.SiLU, nn.Mish,
                    nn.Softplus, nn.Softshrink, nn.Softsign, nn.Tanh, nn.Tanhshrink, nn.Threshold, nn.Softmin,
                    nn.Softmax, nn.Softmax2d, nn.LogSoftmax)
