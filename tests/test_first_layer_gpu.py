"""drsa_amd_first_layer_bwd (WSquare / Flat backward of the one-channel input conv): the pool-sparse
kernel (cells staged through range-checked buffer loads into a pixel image that keeps its zeros)
against the dense kernel fed the host-unpooled relevance, bitwise -- both run the (channel, dy, dx)
chain of oracle/lrp_exact.c.  Shapes cover partial 16 x 64-cell tiles in both directions (the
out-of-range rows and columns of the staging), one channel, and 1-4 clones sharing one argmax map.
Reference: cxai/xai/explain/attribute.py (compute_relevances through zennit's WSquare / Flat)."""
import pytest
import torch

from drsa_audio_amd import _capi

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _unpool(gp, amax, clones):
    Bq, C, H2, W2 = gp.shape
    am = amax.repeat_interleave(clones, 0).long()
    up = torch.zeros(Bq, C, 2 * H2, 2 * W2, device=gp.device)
    for sb in range(4):
        up[:, :, sb // 2::2, sb % 2::2] = torch.where(am == sb, gp, torch.zeros_like(gp))
    return up


@pytest.mark.parametrize("H,W", [(128, 128), (34, 128), (2, 128), (64, 64), (34, 200), (2, 4), (96, 136)])
@pytest.mark.parametrize("C", [1, 5, 32])
@pytest.mark.parametrize("clones", [1, 4])
def test_pooled_equals_dense(H, W, C, clones):
    g = torch.Generator().manual_seed(H + W + C + clones)
    Bs = 3
    Bq = Bs * clones
    gp = torch.randn(Bq, C, H // 2, W // 2, generator=g).to(DEV)
    amax = torch.randint(0, 4, (Bs, C, H // 2, W // 2), generator=g, dtype=torch.uint8).to(DEV)
    w2 = torch.rand(C, 9, generator=g).to(DEV)
    s = _capi.stream_ptr(DEV)
    outs = []
    for pooled in (True, False):
        out = torch.full((Bq, 1, H, W), float("nan"), device=DEV)
        src = gp if pooled else _unpool(gp, amax, clones)
        _capi.call("drsa_amd_first_layer_bwd", src.data_ptr(), amax.data_ptr() if pooled else None, w2.data_ptr(),
                   out.data_ptr(), Bq, clones, C, H, W, s)
        outs.append(out)
    torch.cuda.synchronize()
    assert not torch.isnan(outs[0]).any()
    assert torch.equal(outs[0], outs[1])
    # semantics: the transposed 3 x 3 conv of the unpooled relevance with the squared weights
    ref = torch.nn.functional.conv_transpose2d(_unpool(gp, amax, clones).double(), w2.double().view(C, 1, 3, 3), padding=1)
    assert torch.allclose(outs[0].double(), ref, rtol=1e-5, atol=1e-5)
