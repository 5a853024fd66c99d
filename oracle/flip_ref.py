"""ORACLE — test infrastructure only (imported by tests/, never by drsa_audio_amd).

Loop-for-loop CPU restatement of the reference pixel-flipping core
(cxai/xai/pixelflipping/core.py:6-312, class Flipper), 'constant' perturbation mode:

* patch ranking (core.py:197-222): R clamped at 0, summed per ps x ps patch (patches numbered
  row-major), argsort descending per (sample, concept) — here with a stable sort, the product
  does the same (the reference's unstable torch.argsort leaves ties implementation-defined);
* schedule (core.py:104-127): step s (s = 1, 2, ...) flips s^2 patches, the last step the rest;
* masks (core.py:224-271): the next s^2 ranks of EVERY concept are zeroed (a union), the mask is
  cumulative (masks *= step mask), perturbed input = input * mask (core.py:150-151);
* score (core.py:273-295): relu(logit of the sample's class), classes in consecutive blocks;
* AUPC (core.py:297-315): frac = (p[:-1] - p[1:]) / 2, weights = cumsum(flips[1:]) / sum,
  aupc = sum_s weights_s * frac_s, reshaped [n_classes, samples_per_class].
"""
from __future__ import annotations

import numpy as np
import torch


def patch_sums(R: torch.Tensor, ps: int) -> torch.Tensor:
    B, n_c, H, W = R.shape
    ny, nx = H // ps, W // ps
    Rc = R.detach().cpu().clamp(min=0)
    sums = torch.zeros(B, n_c, ny * nx, dtype=torch.float64)
    for py in range(ny):
        for px in range(nx):
            blk = Rc[:, :, py * ps:(py + 1) * ps, px * ps:(px + 1) * ps].double()
            sums[:, :, py * nx + px] = blk.sum(dim=(-2, -1))
    return sums


def patch_order(R: torch.Tensor, ps: int) -> torch.Tensor:
    """[B, n_c, H, W] relevance -> [B, n_c, P] patch indices by descending clamped patch sum."""
    return torch.argsort(patch_sums(R, ps), dim=-1, descending=True, stable=True)


def flip(forward_func, x: torch.Tensor, R: torch.Tensor | None, ps: int, n_classes: int | None = None,
         order: torch.Tensor | None = None):
    """Returns (aupc_per_class, mean prediction per step, flips per step, predictions [steps, B])."""
    B, C, H, W = x.shape
    if order is None:
        # core.py:61-64: the reference's R.unsqueeze(1) result is discarded; n_concepts = R.size(1)
        order = patch_order(R.reshape(B, R.size(1), H, W), ps)
    n_c = order.size(1)
    nx = W // ps
    P = (H // ps) * nx

    def score(inp):
        out = forward_func(inp)
        nc = out.size(1)
        per = B // nc if B // nc > 0 else 1
        cls = np.repeat(np.arange(nc), per)
        return torch.clamp(out[np.arange(B), cls], min=0).detach().cpu().numpy(), nc

    cur = x.clone()
    p0, nc = score(cur)
    preds = [p0]
    flips = [0]
    flipped = 0
    mask = torch.ones(B, C, H, W, dtype=torch.int16, device=x.device)
    while flipped < P:
        k = len(flips) ** 2 if len(flips) ** 2 < P - flipped else P - flipped
        step = torch.ones(B, C, H, W, dtype=torch.int16, device=x.device)
        idx = order[..., flipped:flipped + k].transpose(-2, -1).reshape(B, -1)
        for b in range(B):
            for i in range(k * n_c):
                r, c = int(idx[b, i]) // nx * ps, int(idx[b, i]) % nx * ps
                step[b, :, r:r + ps, c:c + ps] = 0
        mask = mask * step
        cur = cur * mask
        preds.append(score(cur)[0])
        flips.append(k)
        flipped += k
    preds = np.stack(preds, 0)
    flips = np.array(flips)
    frac = (preds[:-1] - preds[1:]) / 2
    weights = np.cumsum(flips[1:]) / flips[1:].sum()
    aupc = (weights[None].T * frac).sum(axis=0)
    return aupc.reshape(n_classes or nc, -1), preds.mean(axis=1), flips, preds
