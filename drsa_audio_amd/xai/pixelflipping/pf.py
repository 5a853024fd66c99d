"""Pixel-flipping experiments over LRP configurations, drop-in for
``cxai.xai.pixelflipping.pf.PixelFlipping`` (reference pf.py:29-292).

The relevances of every configuration come from the HIP LRP engine (compute_relevances per
class block, pf.py:165-176).  The perturbed forwards are the model's own ``model(x)``, one call per
flipping step, exactly the reference's ``forward_func`` (pf.py:83) -- the default,
``forward="torch"``.  ``forward="engine"`` runs them on the engine's HIP forward instead, with
BatchNorm merged by the canonizer and several steps fused per call (at most ``fuse_max_rows``
rows): the logits then differ from model(x) by fp32 accumulation order (AUPC within 1e-4 of the
torch forward's, tests/test_pixelflipping_gpu.py).
Composites: ``SpecialFirstLayerMapComposite`` (first conv -> the 'first_layer' rule, then
(Activation, Pass), (Convolution, conv rule), (Linear, dense rule)) or, with a 'name_map' key,
``NameLayerMapComposite`` (pf.py:196-236).  Rules by key: ``rule_mapper`` (pf.py:18-27).
"""
from __future__ import annotations

import warnings
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn as nn

from ...engine import get_engine
from ...zennit.canonizers import SequentialMergeBatchNorm
from ...zennit.composites import Composite, NameLayerMapComposite, NameMapComposite, SpecialFirstLayerMapComposite
from ...zennit.rules import AlphaBeta, Epsilon, Flat, Gamma, Norm, Pass, WSquare, ZPlus
from ...zennit.types import Activation, Convolution, Linear
from ..explain.attribute import compute_relevances
from .core import Flipper

rule_mapper = {
    "epsilon": Epsilon,
    "gamma": Gamma,
    "zplus": ZPlus,
    "alphabeta": AlphaBeta,
    "flat": Flat,
    "wsquare": WSquare,
    "pass": Pass,
    "norm": Norm,
}


class PixelFlipping:
    def __init__(self, model: nn.Module, input_batch: torch.Tensor, perturbation_size: int = 8,
                 perturbation_mode: str = "constant", num_classes: int = 10, data_normaliaztion: str = "normalized",
                 device: torch.device = torch.device("cuda"), forward: str = "torch",
                 fuse_max_rows: int = 2048) -> None:
        self.device = torch.device(device) if isinstance(device, str) else device
        self.input_batch = input_batch.to(self.device)
        self.num_classes = int(num_classes)
        self.samples_per_class = self.input_batch.size(0) // self.num_classes
        self.model = model.to(self.device).eval()
        if forward not in ("engine", "torch"):
            raise ValueError("forward must be 'engine' or 'torch'")
        self.forward = forward
        self.pixel_flipper = Flipper(perturbation_size=perturbation_size, perturbation_mode=perturbation_mode,
                                     data_normaliaztion=data_normaliaztion, device=self.device,
                                     fuse_steps=forward == "engine", fuse_max_rows=fuse_max_rows)

    def _forward_func(self, canonizer):
        if self.forward == "torch":
            return lambda x: self.model(x)
        # the engine's forward (HIP kernels), BatchNorm merged by the canonizer when present
        comp = NameMapComposite([], canonizers=[canonizer] if canonizer is not None else None)
        self._fwd_comp = comp                      # keep the engine cache entry alive
        return lambda x: get_engine(self.model, comp).forward(x).clone()

    def __call__(self, configuration_grid: List[Dict[str, Tuple]], stabilizers: Dict[str, float] | None = None,
                 canonizer=None, scaled_gamma=False, plot: bool = True):
        self.canonizer = canonizer if canonizer is not None else SequentialMergeBatchNorm()
        self.stabilizers = stabilizers
        self.aupc_scores, self.averaged_pertubed_prediction_logits, self.pertubed_inputs, self.heatmaps = {}, {}, {}, {}
        forward_func = self._forward_func(self.canonizer)
        flips = None
        for conf in configuration_grid:
            name = self._get_configuration_name(conf)
            if scaled_gamma == "peak4":
                composite = self._get_scaled_composite(conf, ("classifier.0", "classifier.3", "classifier.6"))
            elif scaled_gamma in ("toy", "toynone"):
                composite = self._get_scaled_composite(conf, ("classifier.0", "classifier.2", "classifier.4"))
            else:
                composite = self._get_composite(conf)
            spc = self.samples_per_class
            rel = torch.cat([compute_relevances(self.model, self.input_batch[i * spc:(i + 1) * spc], composite=composite,
                                                class_idx=i) for i in range(self.num_classes)], 0)
            self.heatmaps[name] = rel
            aupc, preds, flips = self.pixel_flipper(forward_func=forward_func, input_batch=self.input_batch.clone(), R=rel)
            self.aupc_scores[name] = aupc
            self.averaged_pertubed_prediction_logits[name] = preds
        if plot:
            self.plot_aupcs(flips)
        return self.aupc_scores, self.averaged_pertubed_prediction_logits, flips, self.heatmaps

    # ----------------------------------------------------------------- composites
    def _get_composite(self, conf) -> Composite:
        for key in ("convolutional", "dense", "first_layer"):
            if key not in conf:
                raise AssertionError(f"rule for {key} layers has to be passed")
        conv_rule = self._get_rule("convolutional", conf)
        dense_rule = self._get_rule("dense", conf)
        first_rule = self._get_rule("first_layer", conf)
        layer_map = [(Activation, Pass()), (Convolution, conv_rule), (Linear, dense_rule)]
        if "name_map" in conf:
            return NameLayerMapComposite(name_map=conf["name_map"], layer_map=layer_map, canonizers=[self.canonizer])
        return SpecialFirstLayerMapComposite(layer_map=layer_map, first_map=[(Convolution, first_rule)],
                                             canonizers=[self.canonizer])

    def _get_name_map(self, conf):
        return [([key], self._get_rule(key, conf)) for key in conf
                if key not in ("convolutional", "dense", "first_layer")]

    def _get_rule(self, layertype: str, conf):
        rule = conf[layertype][0]
        if rule not in rule_mapper:
            raise ValueError(f"Not a valid zennit rule for {layertype} layers!")
        # pf.py:262-266 (the reference leaves the stabilizer unset when a stabilizers dict lacks the
        # layer type, defect; 1e-7 here)
        stabilizer = (self.stabilizers or {}).get(layertype, 1e-7)
        if rule == "gamma":
            return Gamma(gamma=conf[layertype][1], stabilizer=stabilizer)
        if rule == "epsilon":
            return Epsilon(epsilon=conf[layertype][1])
        if rule == "alphabeta":
            alpha = conf[layertype][1]
            return AlphaBeta(alpha=alpha, beta=alpha - 1, stabilizer=stabilizer)
        if rule == "pass":
            return Pass()
        return rule_mapper[rule](stabilizer=stabilizer)

    def _get_scaled_composite(self, conf, dense_names) -> Composite:
        """pf.py:339-411: Gamma gamma, gamma, gamma/2, gamma/4 on features.3/6/9/12."""
        gamma, eps = conf["convolutional"][-1], conf["dense"][-1]
        first = Flat(stabilizer=1e-7) if conf["first_layer"][0] == "flat" else WSquare(stabilizer=1e-7)
        name_map = [(["features.0"], first),
                    (["features.3"], Gamma(gamma=gamma, stabilizer=1e-7)),
                    (["features.6"], Gamma(gamma=gamma, stabilizer=1e-7)),
                    (["features.9"], Gamma(gamma=gamma / 2, stabilizer=1e-7)),
                    (["features.12"], Gamma(gamma=gamma / 4, stabilizer=1e-7))]
        name_map += [([n], Epsilon(epsilon=eps)) for n in dense_names]
        return NameMapComposite(name_map=name_map, canonizers=[self.canonizer])

    @staticmethod
    def _get_configuration_name(conf) -> str:
        """pf.py:275-292 (parameter-free rules such as ('norm',) also accepted outside 'first_layer')."""
        out = ""
        for key in conf:
            rt = conf[key][0]
            if rt == "alphabeta":
                out += "alpha_%3.1f_beta_%3.1f" % (conf[key][1], conf[key][1] - 1.0)
            elif rt == "zplus":
                out += rt + "_"
            elif key == "first_layer":
                out += rt
            elif key == "name_map":
                continue
            elif len(conf[key]) > 1:
                out += rt + "_" + str(conf[key][1]) + "_"
            else:   # parameter-free rule on a non-first layer (the reference indexes [1] and fails)
                out += rt + "_"
        return out

    def plot_aupcs(self, flips_per_perturbation_step, title="EpsGammaWSquare"):
        try:
            import matplotlib.pyplot as plt
        except ImportError:
            warnings.warn("matplotlib is not installed: AUPC plot skipped")
            return
        f = np.array(flips_per_perturbation_step)
        x = np.cumsum(f) / f.sum() * 100
        for key, aupc in self.aupc_scores.items():
            plt.plot(x, np.array(self.averaged_pertubed_prediction_logits[key]), marker="o",
                     label=f"{key} AUPC: {aupc.mean():.3f}")
        plt.title(f"AUPC Curve {title}")
        plt.xlabel("Flipped patches [%]")
        plt.ylabel("Averaged target class logit")
        plt.grid(ls=":", alpha=0.5)
        plt.legend()
