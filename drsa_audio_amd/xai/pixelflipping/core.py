"""Patch-flipping AUPC core, drop-in for ``cxai.xai.pixelflipping.core.Flipper``
(reference core.py:6-312).

Semantics kept from the reference: patches of ``perturbation_size`` numbered row-major, ranked
per (sample, concept) by their summed clamped-at-0 relevance (core.py:197-222); step s flips the
next s^2 ranks of every concept (a union, the last step the remainder, core.py:104-127); the
mask is cumulative and the input is multiplied by it ('constant' mode, core.py:150-151); the
score is relu(logit of the sample's class) with classes in consecutive equal blocks
(core.py:273-295); AUPC = sum_s cumsum-weight_s * (p_{s-1} - p_s) / 2 (core.py:297-315).

Device design: no per-patch Python loop.  Every patch gets the step at which it is first
flipped (the minimum over concepts of its rank, against the cumulative flip counts), so the
mask of any step is one comparison, and all perturbed batches are built on the device.
``fuse_steps=True`` evaluates all steps in one forward call (exact for per-sample-independent
forwards such as the HIP engine's).  Ties in the ranking use a stable sort (the reference's
unstable ``torch.argsort`` leaves their order implementation-defined).  'inpainting' needs
OpenCV (``cv2``), which this image lacks: it raises.
"""
from __future__ import annotations

from typing import Callable, List

import numpy as np
import torch


class Flipper:
    def __init__(self, perturbation_size: int = 16, perturbation_mode: str = "constant",
                 data_normaliaztion: str = "normalized", device: str | torch.device = torch.device("cpu"),
                 fuse_steps: bool = False, fuse_max_rows: int = 2048) -> None:
        if perturbation_mode not in ("constant", "inpainting"):
            raise ValueError('Provided perturbation mode not available. Possible perturbation modes are '
                             '"constant" and "inpainting".')
        self.perturbation_size = int(perturbation_size)
        self.perturbation_mode = perturbation_mode
        self.data_normaliaztion = data_normaliaztion
        self.device = torch.device(device) if isinstance(device, str) else device
        self.fuse_steps = fuse_steps
        self.fuse_max_rows = max(1, int(fuse_max_rows))   # cap of one fused forward (device memory)

    # ------------------------------------------------------------------ schedule
    @staticmethod
    def schedule(num_patches: int) -> List[int]:
        """Patches flipped per step, step 0 (the unperturbed input) included (core.py:104-127)."""
        flips, done = [0], 0
        while done < num_patches:
            k = len(flips) ** 2 if len(flips) ** 2 < num_patches - done else num_patches - done
            flips.append(k)
            done += k
        return flips

    def _patch_order(self, R: torch.Tensor) -> torch.Tensor:
        B, n_c, H, W = R.shape
        ps = self.perturbation_size
        ny, nx = H // ps, W // ps
        Rc = R.clamp(min=0)[..., :ny * ps, :nx * ps]
        sums = Rc.reshape(B, n_c, ny, ps, nx, ps).sum(dim=(3, 5)).reshape(B, n_c, ny * nx)
        return torch.argsort(sums, dim=-1, descending=True, stable=True)

    def _first_step(self, order: torch.Tensor, flips: List[int]) -> torch.Tensor:
        """[B, P] step index (1-based) at which each patch is first zeroed."""
        B, n_c, P = order.shape
        rank = torch.empty_like(order)
        rank.scatter_(-1, order, torch.arange(P, device=order.device).expand(B, n_c, P).contiguous())
        best = rank.min(dim=1).values                                   # union over concepts
        cum = torch.tensor(np.cumsum(flips[1:]), device=order.device)   # ranks < cum[s-1] are flipped by step s
        return torch.searchsorted(cum, best, right=True) + 1

    def _masks(self, first: torch.Tensor, step: int, C: int, H: int, W: int) -> torch.Tensor:
        ps = self.perturbation_size
        ny, nx = H // ps, W // ps
        B = first.size(0)
        keep = (first > step).to(torch.int16).reshape(B, 1, ny, 1, nx, 1)
        m = keep.expand(B, C, ny, ps, nx, ps).reshape(B, C, ny * ps, nx * ps)
        if ny * ps != H or nx * ps != W:
            full = torch.ones(B, C, H, W, dtype=torch.int16, device=first.device)
            full[..., :ny * ps, :nx * ps] = m
            m = full
        return m

    def _scores(self, out: torch.Tensor, B: int) -> torch.Tensor:
        n_classes = out.size(1)
        self.n_classes = n_classes
        per = B // n_classes if B // n_classes > 0 else 1
        cls = torch.arange(n_classes, device=out.device).repeat_interleave(per)[:B]
        return torch.clamp(out[torch.arange(B, device=out.device), cls], min=0)

    # ------------------------------------------------------------------ call
    def __call__(self, forward_func: Callable, input_batch: torch.Tensor, R, flipping_mode: str | None = None):
        if self.perturbation_mode == "inpainting":
            raise NotImplementedError("inpainting perturbation needs OpenCV (cv2.inpaint), which is not installed")
        x = input_batch.detach().to(self.device)
        B, C, H, W = x.shape
        ps = self.perturbation_size
        self.batch_size, self.num_channels, self.height, self.width = B, C, H, W
        self.num_patches = P = (H // ps) * (W // ps)
        if flipping_mode == "random":
            order = torch.stack([torch.randperm(P, device=self.device) for _ in range(B)]).reshape(B, 1, P)
        else:
            R = torch.as_tensor(R).to(self.device)
            n_c = R.size(1)            # core.py:61-64 (the reference's unsqueeze result is discarded)
            order = self._patch_order(R.reshape(B, n_c, H, W).to(torch.float32))
        self.n_concepts = order.size(1)
        self.sorted_patch_indices_by_relevance = order
        flips = self.schedule(P)
        first = self._first_step(order, flips)
        S = len(flips)
        xs = [x] + [x * self._masks(first, s, C, H, W) for s in range(1, S)]
        with torch.no_grad():
            if self.fuse_steps:
                per = max(1, self.fuse_max_rows // B)         # steps per fused forward
                outs = [forward_func(torch.cat(xs[i:i + per], 0)) for i in range(0, S, per)]
                out = torch.cat(outs, 0)
                preds = torch.stack([self._scores(o, B) for o in out.reshape(S, B, -1)])
            else:
                preds = torch.stack([self._scores(forward_func(xi), B) for xi in xs])
        preds = preds.detach().cpu().numpy()                           # [steps, B], float32 like the reference
        flips = np.array(flips)
        frac = (preds[:-1] - preds[1:]) / 2
        weights = np.cumsum(flips[1:]) / flips[1:].sum()
        aupc = (weights[None].T * frac).sum(axis=0)
        return aupc.reshape(self.n_classes, -1), preds.mean(axis=1), flips
