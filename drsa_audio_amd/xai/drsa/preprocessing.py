"""DRSA training data on device, drop-in for ``cxai.xai.drsa.preprocessing``.

* ``preprocess_data``          — preprocessing.py:18-89 (intended semantics: the shipped call
                                 of get_intermediate has its arguments swapped, defect D2, and
                                 the inference branch misreads the map size, D3)
* ``get_intermediate``         — preprocessing.py:106-176
* ``compute_context_vectors``  — preprocessing.py:179-193
* ``sample_spatial_locations`` — preprocessing.py:196-216 (host numpy RNG: the reference's stream)
* ``normalize_vectors``        — preprocessing.py:219-231
* ``get_vectors_from_maps``    — preprocessing.py:234-256 (its row order, defect D12, kept)
* ``drsa_training_data``       — preprocess_data + load_and_normalize_data
                                 (getdrsadata.py:47-59) in one call, ready for ``drsa.main``

The LRP pass runs on the HIP engine and stops at layer j (nothing below it is needed); the
activation map is kept by the forward, the relevance arrives in pooled form with its argmax,
and ``drsa_amd_drsa_vectors`` gathers A and C = R / (A + 1e-7) at the sampled locations in one
kernel, so the reference's [B, d, H, W] relevance maps never exist.  Every tensor op here is a
HIP kernel behind the C ABI; there is no CPU path.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from ... import _capi
from ...engine import get_engine
from ..explain.attribute import lrp_output_modifier

LAYOUT_REFERENCE, LAYOUT_ROWS = 0, 1


def _as_device_batch(input_batch, device) -> torch.Tensor:
    if isinstance(input_batch, np.ndarray):
        input_batch = torch.from_numpy(input_batch)
    x = input_batch.detach()
    dev = torch.device(device) if device is not None else x.device
    if dev.type != "cuda":
        raise _capi.DrsaAmdError("preprocess_data runs on the GPU only (pass a HIP device)")
    return x.to(dev, torch.float32).contiguous()


def _class_rows(B: int, class_idx: int, device) -> torch.Tensor:
    return torch.full((B,), int(class_idx), dtype=torch.int32, device=device)


def _seed_fn(class_idx, num_classes, one_hot_encoded):
    if class_idx is not None:
        return None
    return lrp_output_modifier(None, num_classes, one_hot_encoded)


def sample_spatial_locations(batch_size: int, map_size: Tuple[int, int], num_locations: int) -> np.ndarray:
    """preprocessing.py:196-216: per sample np.random.choice(H*W, L, replace=False) from the
    global numpy RNG (same stream as the reference)."""
    idcs = np.zeros((batch_size, num_locations), dtype=int)
    for i in range(batch_size):
        idcs[i, :] = np.random.choice(map_size[0] * map_size[1], num_locations, replace=False)
    return idcs


def get_intermediate(model: nn.Module, input_batch: torch.Tensor, composite, layer: nn.Module | str | int,
                     class_idx: int, attr_batch_size: int = 64, one_hot_encoded: bool = False,
                     num_classes: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Activation and relevance maps [B, d, H, W] at ``layer`` (module, name or feature index)."""
    x = _as_device_batch(input_batch, None)
    name = _layer_name(model, layer)
    eng = get_engine(model, composite)
    B = x.size(0)
    acts, rels = [], []
    step = B if attr_batch_size is None else max(1, int(attr_batch_size))
    for i in range(0, B, step):
        xb = x[i:i + step]
        cap = eng.capture(xb, name, cls=None if class_idx is None else _class_rows(xb.size(0), class_idx, x.device),
                          one_hot=one_hot_encoded, seed_fn=_seed_fn(class_idx, num_classes, one_hot_encoded))
        acts.append(cap["act"].clone())
        if cap["amax"] is not None:
            full = torch.empty_like(cap["act"])
            _capi.call("drsa_amd_relevance_unpool", cap["rel"].data_ptr(), cap["amax"].data_ptr(), xb.size(0), 1,
                       cap["C"], cap["H"], cap["W"], cap["ph"], cap["pw"], full.data_ptr(), _capi.stream_ptr(x.device))
            rels.append(full)
        else:
            rels.append(cap["rel"].clone())
    return torch.cat(acts, 0), torch.cat(rels, 0)


def _layer_name(model, layer) -> str:
    if isinstance(layer, str):
        return layer if layer.startswith("features.") else f"features.{layer}"
    if isinstance(layer, int):
        return f"features.{layer}"
    for n, m in model.features.named_children():
        if m is layer:
            return f"features.{n}"
    raise ValueError("layer is not a child of model.features")


def _vectors(cap: dict, idx: Optional[torch.Tensor], L: int, layout: int, A_out: torch.Tensor,
             C_out: torch.Tensor, B: int, device) -> None:
    _capi.call("drsa_amd_drsa_vectors", cap["act"].data_ptr(), cap["rel"].data_ptr(), _capi.ptr(cap["amax"]),
               _capi.ptr(idx), B, cap["C"], cap["H"], cap["W"], cap["ph"], cap["pw"], L, layout, A_out.data_ptr(),
               C_out.data_ptr(),
               _capi.stream_ptr(device))


def preprocess_data(model: nn.Module, input_batch, composite, layer_idx: int, class_idx: Optional[int],
                    num_locations: Optional[int] = None, one_hot_encoded: bool = False, device=None,
                    attr_batch_size: int = 1024, layout: int = LAYOUT_REFERENCE,
                    num_classes: Optional[int] = None, group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(activation_vectors, context_vectors) at model.features[layer_idx].

    num_locations given: [B*L, d] rows at L sampled locations per sample (training data);
    None: every location, [B, H*W, d] (inference).  ``layout`` LAYOUT_REFERENCE keeps the
    reference's get_vectors_from_maps row order (D12); LAYOUT_ROWS gives one d-vector per
    (sample, location).  ``attr_batch_size`` bounds the LRP working set (the reference uses
    64; results do not depend on it).  ``group``: ``input_batch`` is this rank's slice of a
    global batch (ranks in order) and the sampled locations are this slice's draws from the
    global numpy stream (every rank draws for all samples, as one process would)."""
    x = _as_device_batch(input_batch, device)
    dev = x.device
    name = _layer_name(model, layer_idx)
    eng = get_engine(model, composite)
    B = x.size(0)
    # with a group every rank joins the size exchange first, so an empty slice on one rank cannot
    # strand the others in a collective; an empty GLOBAL batch raises on every rank together
    off, B_all = (0, B) if group is None else _sample_offset(B, group, dev)
    if B_all == 0:
        raise _capi.DrsaAmdError("preprocess_data: empty input batch")
    li, where = eng.capture_stage(name)
    if B == 0:
        # this rank holds no samples: empty rows of the layer's width (one dummy sample through the
        # engine gives the geometry); the numpy stream still advances over all B_all draws
        cap = eng.capture(torch.zeros((1,) + tuple(x.shape[1:]), device=dev, dtype=x.dtype), name,
                          cls=None if class_idx is None else _class_rows(1, class_idx, dev),
                          one_hot=one_hot_encoded, seed_fn=_seed_fn(class_idx, num_classes, one_hot_encoded))
        C, H, W = cap["C"], cap["H"], cap["W"]
        if num_locations:
            sample_spatial_locations(B_all, (H, W), num_locations)
            return torch.empty(0, C, device=dev), torch.empty(0, C, device=dev)
        return torch.empty(0, H * W, C, device=dev), torch.empty(0, H * W, C, device=dev)
    idx_all = None
    out_a = out_c = None
    step = max(1, int(attr_batch_size))
    for i in range(0, B, step):
        xb = x[i:i + step]
        b = xb.size(0)
        cap = eng.capture(xb, name, cls=None if class_idx is None else _class_rows(b, class_idx, dev),
                          one_hot=one_hot_encoded, seed_fn=_seed_fn(class_idx, num_classes, one_hot_encoded))
        C, H, W = cap["C"], cap["H"], cap["W"]
        if out_a is None:
            if num_locations:
                # sample after the maps exist, as the reference (one draw per sample, in order)
                draws = sample_spatial_locations(B_all, (H, W), num_locations)[off:off + B]
                idx_all = torch.from_numpy(draws.astype(np.int32)).to(dev)
                out_a = torch.empty(B * num_locations, C, device=dev)
                out_c = torch.empty(B * num_locations, C, device=dev)
            else:
                out_a = torch.empty(B, H * W, C, device=dev)
                out_c = torch.empty(B, H * W, C, device=dev)
        if num_locations:
            L = int(num_locations)
            _vectors(cap, idx_all[i:i + b].contiguous(), L, layout, out_a[i * L:(i + b) * L], out_c[i * L:(i + b) * L],
                     b, dev)
        else:
            _vectors(cap, None, H * W, LAYOUT_ROWS, out_a[i:i + b], out_c[i:i + b], b, dev)
    return out_a, out_c


def compute_context_vectors(activation_vectors: torch.Tensor, relevance_vectors: torch.Tensor) -> torch.Tensor:
    """preprocessing.py:179-193: R / (A + 1e-7) (fused into drsa_amd_drsa_vectors on the
    preprocess_data path; this standalone form is an elementwise op on device tensors)."""
    return relevance_vectors / (activation_vectors + 1e-7)


def get_vectors_from_maps(maps: torch.Tensor, idcs_batch: np.ndarray) -> torch.Tensor:
    """preprocessing.py:234-256 on a device map [B, d, H, W] (reference row order, D12)."""
    _capi.require_gpu(maps, "maps")
    B, d, H, W = maps.shape
    idx = torch.as_tensor(np.asarray(idcs_batch), dtype=torch.int32).to(maps.device).contiguous()
    L = idx.size(1)
    A = torch.empty(B * L, d, device=maps.device)
    Cc = torch.empty_like(A)
    _capi.call("drsa_amd_drsa_vectors", maps.data_ptr(), maps.data_ptr(), None, idx.data_ptr(), B, d, H, W, 1, 1, L,
               LAYOUT_REFERENCE, A.data_ptr(), Cc.data_ptr(), _capi.stream_ptr(maps.device))
    return A


class _HipNormalizeOps:
    """The two halves of drsa_amd_normalize_vectors for rows spread over ranks."""

    def sumsq(self, v: torch.Tensor) -> torch.Tensor:
        """This rank's fp64 sum of v^2 (a [1] device tensor; 0 for an empty shard)."""
        out = torch.empty(1, dtype=torch.float64, device=v.device)
        ws = torch.empty(_capi.lib().drsa_amd_normalize_workspace_bytes(), dtype=torch.uint8, device=v.device)
        _capi.call("drsa_amd_normalize_sumsq", _capi.ptr(v) if v.numel() else None, v.numel(), ws.data_ptr(),
                   ws.numel(), out.data_ptr(), _capi.stream_ptr(v.device))
        return out

    def scale(self, v: torch.Tensor, sums: torch.Tensor, n_total: int, out: torch.Tensor) -> None:
        """out = v / sqrt((sums[0] + sums[1] + ...) / n_total) / d^(1/4)."""
        _capi.call("drsa_amd_normalize_scale", _capi.ptr(v) if v.numel() else None, v.numel(), v.size(-1),
                   sums.data_ptr(), sums.numel(), int(n_total), _capi.ptr(out) if out.numel() else None,
                   _capi.stream_ptr(v.device))


def _all_gather_rows(t: torch.Tensor, group) -> torch.Tensor:
    """[world, *t.shape] with rank r's ``t`` in row r (RCCL on the device, gloo through the host)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        # RCCL moves device tensors only: a host tensor (e.g. a size) goes to this rank's device
        src = t if t.is_cuda else t.to(torch.device("cuda", torch.cuda.current_device()))
    else:
        src = t.cpu()
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src.contiguous(), group=group)
    return torch.stack(parts).to(t.device)


def normalize_vectors(vectors: torch.Tensor, out: Optional[torch.Tensor] = None, group=None,
                      _ops=None) -> torch.Tensor:
    """preprocessing.py:219-231: v / sqrt(mean(v^2)) / d^(1/4) (HIP, deterministic reduction).

    ``group`` (a process group, e.g. ``dist.group.WORLD``): ``vectors`` is this rank's share of the
    rows and the mean runs over ALL ranks' elements, as the reference normalises the whole
    1000-sample set at once (getdrsadata.py:47-59).  One all-gather of (sum v^2, count) per call in
    fp64; every rank adds the sums in rank order, so all ranks use the same E.  Without ``group``
    the mean is over ``vectors`` alone (the reference's single-process call)."""
    v = vectors.detach()
    out = torch.empty_like(v) if out is None else out
    if group is None:
        _capi.require_gpu(v, "vectors")
        ws = torch.empty(_capi.lib().drsa_amd_normalize_workspace_bytes(), dtype=torch.uint8, device=v.device)
        _capi.call("drsa_amd_normalize_vectors", v.data_ptr(), v.numel(), v.size(-1), out.data_ptr(), ws.data_ptr(),
                   ws.numel(), _capi.stream_ptr(v.device))
        return out
    ops = _ops or _HipNormalizeOps()
    if _ops is None:
        _capi.require_gpu(v, "vectors")
    local = torch.cat([ops.sumsq(v).reshape(1).to(torch.float64),
                       torch.tensor([float(v.numel())], dtype=torch.float64, device=v.device)])
    table = _all_gather_rows(local, group)                   # [world, 2]: (sum v^2, count) per rank
    n_total = int(table[:, 1].sum().item())
    if n_total == 0:
        raise _capi.DrsaAmdError("normalize_vectors: no elements on any rank")
    ops.scale(v, table[:, 0].contiguous(), n_total, out)
    return out


def _sample_offset(b_local: int, group, device=None) -> Tuple[int, int]:
    """(first global sample index of this rank, global batch size): ranks hold consecutive slices."""
    import torch.distributed as dist
    rank = dist.get_rank(group)
    sizes = _all_gather_rows(torch.tensor([b_local], dtype=torch.int64, device=device), group).reshape(-1).tolist()
    return int(sum(sizes[:rank])), int(sum(sizes))


def drsa_training_data(model: nn.Module, input_batch, composite, layer_idx: int, class_idx: int,
                       num_locations: int = 20, one_hot_encoded: bool = False, device=None,
                       attr_batch_size: int = 1024, group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """preprocess_data -> normalize_vectors on A and on C separately (getdrsadata.py:119-137 then
    :47-59 without the pickle round trip): normalised (A, C) [B*L, d], ready for drsa.main.

    ``group``: rank-local extraction for the row-sharded optimiser (SURVEY §8(e) "per-GPU
    extraction").  ``input_batch`` is this rank's slice of the global batch (rank 0 first); the
    locations are drawn from the global numpy stream for every global sample as one process would
    (each rank keeps its own rows) and the normalisation is over all ranks' rows.  The returned
    rows are this rank's rows of the single-process result; feed them to
    ``distributed.main_sharded(..., local_rows=True)``."""
    A, C = preprocess_data(model, input_batch, composite, layer_idx, class_idx, num_locations, one_hot_encoded,
                           device, attr_batch_size, group=group)
    return normalize_vectors(A, out=A, group=group), normalize_vectors(C, out=C, group=group)
