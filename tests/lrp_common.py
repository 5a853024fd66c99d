"""Shared builders for the LRP tests (models, synthetic log-mels, rule specs for the oracle)."""
import numpy as np
import torch

from drsa_audio_amd.model.create_model import VGGType


def gtzan128(seed=0):
    torch.manual_seed(seed)
    return VGGType(n_filters=(32, 32, 64, 64, 128), n_dense=128, pool_kernels=((2, 2),) * 5, dropout=0.4,
                   input_size=(128, 128), conv_bn=False, dense_bn=False, block_depth=1).eval()


def toy(seed=0):
    torch.manual_seed(seed)
    return VGGType(n_filters=(8, 8, 16, 16, 16), n_dense=32, n_classes=2, pool_kernels=((2, 2),) * 5,
                   dropout=0.0, input_size=(64, 64), conv_bn=False, dense_bn=False, block_depth=1).eval()


def logmel(B, H=128, W=128, seed=1):
    """Synthetic log-mel: clamp(log10(e * tilt + 1e-7), -4), e ~ Exp(1)."""
    g = torch.Generator().manual_seed(seed)
    e = torch.empty(B, 1, H, W).exponential_(generator=g)
    tilt = 10 ** (-3 * torch.arange(H).float() / max(H - 1, 1))
    return torch.clamp(torch.log10(e * tilt[None, None, :, None] + 1e-7), min=-4)


def spec(name_map):
    """Product rule descriptors -> oracle rule specs."""
    out = {}
    for names, r in name_map:
        k = r.kind
        if k == "epsilon":
            t = ("epsilon", r.epsilon)
        elif k == "gamma":
            t = ("gamma", r.gamma, r.stabilizer)
        elif k in ("wsquare", "flat", "zplus"):
            t = (k, r.stabilizer)
        elif k == "norm":
            # zennit Norm(stabilizer) on conv/dense = Epsilon(stabilizer) (see engine/plan.py _kind)
            t = ("epsilon", r.stabilizer)
        elif k == "alphabeta":
            t = ("alphabeta", r.alpha, r.beta, r.stabilizer)
        elif k == "pass":
            t = ("pass",)
        else:
            raise ValueError(k)
        for n in names:
            out[n] = t
    return out


def u64():
    import os
    from conftest import GOLDEN
    return torch.from_numpy(np.load(os.path.join(GOLDEN, "u64_seed42.npy")))


def ortho(d, seed):
    q, _ = np.linalg.qr(np.random.default_rng(seed).standard_normal((d, d)))
    return torch.from_numpy(q.astype(np.float32))


def maxnorm_err(a, b):
    a = torch.as_tensor(a).reshape(a.shape[0], -1).double()
    b = torch.as_tensor(b).reshape(b.shape[0], -1).double()
    return float(((a - b).abs().amax(1) / b.abs().amax(1).clamp_min(1e-30)).max())


def vggish(seed=0, input_size=(128, 256), randomize_bn=True):
    """VGGish-BN of the reference's DRSA scripts (getdrsadata.py:68-73): filters (64,64,100,128,128),
    n_dense 100, pools ((2,4),(2,2),(2,2),(2,2),(2,2)), block_depth 2, BN in trunk and head.
    BN running statistics / affine parameters are randomised so that merging is not a no-op."""
    torch.manual_seed(seed)
    m = VGGType(n_filters=(64, 64, 100, 128, 128), n_dense=100,
                pool_kernels=((2, 4), (2, 2), (2, 2), (2, 2), (2, 2)), dropout=0.3, input_size=input_size,
                conv_bn=True, dense_bn=True).eval()
    if randomize_bn:
        g = torch.Generator().manual_seed(seed + 100)
        for mod in m.modules():
            if isinstance(mod, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)):
                n = mod.num_features
                mod.running_mean.copy_(0.1 * torch.randn(n, generator=g))
                mod.running_var.copy_(0.5 + torch.rand(n, generator=g))
                mod.weight.data.copy_(0.8 + 0.4 * torch.rand(n, generator=g))
                mod.bias.data.copy_(0.05 * torch.randn(n, generator=g))
    return m


def rel_l2(a, b):
    """Per-sample relative L2 error ||a - b|| / ||b|| (numpy, float64)."""
    a = torch.as_tensor(np.asarray(a)).reshape(a.shape[0], -1).double()
    b = torch.as_tensor(np.asarray(b)).reshape(b.shape[0], -1).double()
    return ((a - b).norm(dim=1) / b.norm(dim=1).clamp_min(1e-300)).numpy()


def f64_anchored_check(R32, R_ref32, R64, ratio_med=2.0, ratio_p75=4.0):
    """Accuracy of an fp32 LRP result R32 against the float64 evaluation R64 of the same rules,
    measured next to the reference's own fp32 evaluation R_ref32 (torch/oneDNN order).

    LRP-gamma/epsilon with bias divides by stabilised denominators that can be ~0 at single
    pixels; there ANY fp32 evaluation departs from float64 (one GTZAN-128 sample in 32 sits at
    0.18 relative L2 for the reference's own fp32 path), and per-sample errors of two fp32
    orders are uncorrelated.  So the bound is distributional, on the per-sample relative L2
    error: median within `ratio_med` x the reference path's median (+1e-6) and 75th percentile
    within `ratio_p75` x its 75th percentile (+1e-6).  Measured (32 samples, classes 0 / 7, the
    kernels' order = oracle mode "exact"): medians 2.3e-5 / 4.0e-5 vs 2.5e-5 / 2.8e-5, p75
    1.8e-4 / 1.5e-4 vs 7.7e-5 / 8.0e-5 -- one sequential fma chain over 9 * Cin terms per output
    has a heavier tail than oneDNN's blocked sums.  Returns the per-sample errors."""
    e32, eref = rel_l2(R32, R64), rel_l2(R_ref32, R64)
    assert np.median(e32) <= ratio_med * np.median(eref) + 1e-6, (np.median(e32), np.median(eref))
    assert np.percentile(e32, 75) <= ratio_p75 * np.percentile(eref, 75) + 1e-6, \
        (np.percentile(e32, 75), np.percentile(eref, 75))
    return e32, eref
