"""Concept (subspace) heatmaps, drop-in for ``cxai.xai.explain.explainer``.

* ``HeatmapGenerator``            — reference explainer.py:15-176
* ``get_class_composite``         — reference explainer.py:179-203
* ``compute_subspace_relevances`` — reference explainer.py:206-242

``generate_subspace_heatmaps`` does NOT replicate the batch K+1 times (explainer.py:92):
the HIP plan runs one forward and the layers above the projection once, fans out K+1
relevance clones in the fused projection backward, and splits / sums / sorts on device.
The result equals the reference's clone semantics (every rule is linear in the relevance
given the shared forward).  ``info`` holds numpy arrays exactly like the reference;
``info_device`` keeps the same results as device tensors.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch
import torch.nn as nn

from ... import _capi
from ...engine import get_engine
from ...model.modify_model import ProjectionModel
from ...utils.constants import CLASS_IDX_MAPPER, CLASS_IDX_MAPPER_TOY
from ...zennit.composites import Composite, NameMapComposite
from ...zennit.rules import Epsilon
from .attribute import SubspaceHook, compute_relevances, seed_class_indices


class HeatmapGenerator:
    def __init__(self, model: nn.Module, U: torch.Tensor, name_map: List[Tuple[List[str], object]],
                 sample_class: str, num_concepts: int = 4, layer_idx: int = 10,
                 device: str | torch.device = torch.device("cuda"), canonizers=None,
                 standard: str = "clone") -> None:
        """``canonizers`` (extension, default None = the reference's composite) is passed to the
        class composite, e.g. ``[SequentialMergeBatchNorm()]`` for the VGGish-BN models of the
        reference's DRSA scripts (getdrsadata.py:113), whose layer 19 has d = 100.
        ``standard`` (extension): "clone" (default, the reference's semantics) propagates clone 0
        as the reference's replicated batch does (explainer.py:92); "sum" computes the standard
        heatmap as the sum of the K concept heatmaps -- every LRP rule is linear in the relevance,
        so this is the reference's clone 0 up to fp32 rounding (as close to float64 as clone 0,
        tests/test_lrp_gpu.py), and the network below the projection runs K instead of K+1 times
        (the bench headline's mode; ties in the standard relevance may order differently)."""
        if standard not in ("sum", "clone"):
            raise ValueError("standard must be 'sum' or 'clone'")
        self.standard = standard
        self.device = torch.device(device) if isinstance(device, str) else device
        self.num_concepts = int(num_concepts)
        case = "toy" if sample_class.endswith("1") or sample_class.endswith("2") else "gtzan"
        mapper = CLASS_IDX_MAPPER if case == "gtzan" else CLASS_IDX_MAPPER_TOY
        self.class_idx = mapper[sample_class]
        self.num_classes = len(mapper)
        self.projectionmodel = ProjectionModel(model, layer_idx, U.to(self.device), self.num_concepts, case=case)
        self.composite = get_class_composite(name_map, self.num_concepts, device=device, canonizers=canonizers)
        self.info = {}
        self.info_device = {}

    def generate_subspace_heatmaps(self, input_batch: torch.Tensor, one_hot_encoded: bool = False,
                                   concept_flipping: bool = False, flip_all_classes: bool = False,
                                   to_host: bool = True) -> None:
        x = input_batch.to(self.device, torch.float32).contiguous()
        eng = get_engine(self.projectionmodel, self.composite)
        B = x.size(0)
        cls = seed_class_indices(B, None if flip_all_classes else self.class_idx,
                                 self.num_classes if flip_all_classes else None, self.device)
        if to_host and B >= 2 * self.host_chunk_min:
            self._heatmaps_to_host_pipelined(eng, input_batch, x, cls, one_hot_encoded)
            return
        out = eng.subspace_heatmaps(x, cls=cls, one_hot=one_hot_encoded, standard=self.standard)
        self.info_device = out
        if to_host:
            # the reference returns numpy (explainer.py:111): D2H into fresh pinned buffers (torch's
            # caching host allocator), all copies queued on the stream, one wait
            info = {}
            inp = input_batch.detach()
            if inp.dtype == torch.bfloat16:   # numpy has no bf16: the input as float32 (exact)
                inp = inp.float()
            if inp.device.type == "cpu":
                info["input"] = inp.numpy()
            else:
                info["input"] = torch.empty(inp.shape, dtype=inp.dtype, pin_memory=True)
                info["input"].copy_(inp, non_blocking=True)
            for k, v in out.items():
                info[k] = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
                info[k].copy_(v, non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
            self.info = {k: (v.numpy() if torch.is_tensor(v) else v) for k, v in info.items()}

    # to_host with a large batch: two halves, the second computed while the first one's results
    # (and the input, which is ready at the start) cross PCIe on a side stream.  Every sample's
    # results are independent of the batch it is computed in, so the output is bit-identical.
    host_chunk_min = 128

    def _heatmaps_to_host_pipelined(self, eng, input_batch, x, cls, one_hot):
        B = x.size(0)
        main = torch.cuda.current_stream(self.device)
        if getattr(self, "_d2h_stream", None) is None:
            self._d2h_stream = torch.cuda.Stream(self.device)
        side = self._d2h_stream
        inp = input_batch.detach()
        if inp.dtype == torch.bfloat16:   # numpy has no bf16: the input as float32 (exact)
            inp = inp.float()
        info = {}
        side.wait_stream(main)            # the input (and anything queued before) is ready
        if inp.device.type == "cpu":
            info["input"] = inp.numpy()
        else:
            info["input"] = torch.empty(inp.shape, dtype=inp.dtype, pin_memory=True)
            with torch.cuda.stream(side):
                info["input"].copy_(inp, non_blocking=True)
        half = (B + 1) // 2
        parts = []
        for s0, s1 in ((0, half), (half, B)):
            out = eng.subspace_heatmaps(x[s0:s1], cls=cls[s0:s1], one_hot=one_hot, standard=self.standard)
            parts.append(out)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                for k, v in out.items():
                    if k not in info:
                        info[k] = torch.empty((B,) + tuple(v.shape[1:]), dtype=v.dtype, pin_memory=True)
                    info[k][s0:s1].copy_(v, non_blocking=True)
        self.info_device = {k: torch.cat([o[k] for o in parts]) for k in parts[0]}
        side.synchronize()
        main.synchronize()
        self.info = {k: (v.numpy() if torch.is_tensor(v) else v) for k, v in info.items()}

    def obtain_heatmaps(self, input_batch: torch.Tensor, one_hot_encoded: bool = False,
                        flip_all_classes: bool = False) -> torch.Tensor:
        """Reference semantics on an already replicated batch (rows = K+1 clones per sample)."""
        return compute_relevances(self.projectionmodel, input_batch.to(self.device), self.composite,
                                  one_hot_encoded=one_hot_encoded,
                                  class_idx=self.class_idx if not flip_all_classes else None,
                                  num_classes=self.num_classes if flip_all_classes else None)

    def sort_subspaces(self, subspace_heatmaps: np.ndarray):
        """Per-instance descending order of subspace relevance (keeps the batch dim at B=1,
        unlike the reference's squeeze, defect D7)."""
        b, K = subspace_heatmaps.shape[:2]
        rel = subspace_heatmaps.sum(axis=(-2, -1)).reshape(b, K)
        mask = np.argsort(rel, axis=-1)[..., ::-1]
        ar = np.arange(b)[:, None]
        return subspace_heatmaps[ar, mask], rel[ar, mask], mask


def get_class_composite(name_map: List[Tuple[List[str], object]], num_concepts: int,
                        device: str | torch.device = torch.device("cpu"), canonizers=None) -> Composite:
    """name_map + Epsilon() on (inv)projection + SubspaceHook on the filter (``canonizers``:
    extension, see HeatmapGenerator)."""
    nm = list(name_map)
    nm.append((["features.invprojection"], Epsilon()))
    nm.append((["features.subspacefilter"], SubspaceHook(num_concepts, device=device)))
    nm.append((["features.projection"], Epsilon()))
    return NameMapComposite(name_map=nm, canonizers=canonizers)


def compute_subspace_relevances(act_vecs: torch.Tensor, ctx_vecs: torch.Tensor, U: torch.Tensor,
                                n_concepts: int = 4) -> torch.Tensor:
    """r[b, k] = sum_n sum_{j in block k} (a_n U)_j (c_n U)_j  for act/ctx [b, N, d] (or [N, d]),
    any d <= 128 with n_concepts | d (drsa_amd_subspace_relevances)."""
    assert act_vecs.dim() < 4 or ctx_vecs.dim() < 4, "Please provide act and ctx vectors reshaped to [batch, N, d]"
    a = act_vecs if act_vecs.dim() == 3 else act_vecs.unsqueeze(0)
    c = ctx_vecs if ctx_vecs.dim() == 3 else ctx_vecs.unsqueeze(0)
    for t, name in ((a, "act_vecs"), (c, "ctx_vecs"), (U, "U")):
        if not isinstance(t, torch.Tensor) or not t.is_cuda:
            raise _capi.DrsaAmdError(f"compute_subspace_relevances: {name} must be a GPU tensor "
                                     f"(drsa_audio_amd has no CPU path)")
    if c.device != a.device or U.device != a.device:
        raise ValueError("compute_subspace_relevances: act_vecs, ctx_vecs and U must be on one device")
    if a.dim() != 3 or c.shape != a.shape:
        raise ValueError(f"act_vecs and ctx_vecs must have the same [batch, N, d] shape "
                         f"(got {tuple(act_vecs.shape)} and {tuple(ctx_vecs.shape)})")
    b, N, d = a.shape
    if U.shape != (d, d):
        raise ValueError(f"U must be [{d}, {d}] for d={d} (got {tuple(U.shape)})")
    if n_concepts <= 0 or d % n_concepts:
        raise ValueError(f"n_concepts={n_concepts} must be a positive divisor of d={d}")
    a = a.to(torch.float32).contiguous()
    c = c.to(torch.float32).contiguous()
    U = U.to(torch.float32).contiguous()
    out = torch.empty(b, n_concepts, device=a.device)
    nbytes = _capi.lib().drsa_amd_subspace_relevances_workspace_bytes(b, N, d, n_concepts)
    if nbytes == 0:
        raise _capi.DrsaAmdError(f"compute_subspace_relevances: unsupported problem b={b} N={N} d={d} "
                                 f"n_concepts={n_concepts} (d <= 128)")
    ws = torch.empty(int(nbytes), dtype=torch.uint8, device=a.device)
    _capi.call("drsa_amd_subspace_relevances", a.data_ptr(), c.data_ptr(), b, N, d, n_concepts, U.data_ptr(),
               out.data_ptr(), ws.data_ptr(), ws.numel(), _capi.stream_ptr(a.device))
    return out
