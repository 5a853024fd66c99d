"""The (2,4) max-pool backward folded into the fp32 backward conv's staging (VGGish block 1 above the
WSquare layer): drsa_amd_conv_bwd_den_map with g at (2,4)-pool resolution and its
argmax bytes equals drsa_amd_relevance_unpool followed by the dense-g den-map backward bit for bit
(the same fp32 MFMA operands in the same chain order), and the VGGish plans no longer launch a
maxpool_bwd kernel."""
import pytest
import torch

from lrp_common import logmel, vggish
from drsa_audio_amd import _capi
from drsa_audio_amd.utils.constants import LRP_NAME_MAP_VGGISH
from drsa_audio_amd.zennit.canonizers import SequentialMergeBatchNorm
from drsa_audio_amd.zennit.composites import NameMapComposite

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
XM_NONE, XM_MUL = 0, 1


@pytest.mark.parametrize("W", [256, 128, 64, 32])
@pytest.mark.parametrize("xm", [XM_NONE, XM_MUL])
def test_den_map_pool24_sparse_equals_unpool_dense(W, xm):
    lib = _capi.lib()
    cin, cout, H, B, clones = 64, 64, 16, 2, 3
    assert lib.drsa_amd_conv_bwd_has_kernel_pw(cin, cout, W, 1, 4) == 1
    Bq = B * clones
    gen = torch.Generator().manual_seed(W + xm)
    wts = (torch.randn(9 * cin * cout, generator=gen) / 24).to(DEV)
    gp = torch.randn(Bq, cin, H // 2, W // 4, generator=gen).to(DEV)
    am = torch.randint(0, 8, (B, cin, H // 2, W // 4), generator=gen, dtype=torch.uint8).to(DEV)
    x = torch.randn(B, cout, H, W, generator=gen).clamp(min=0).to(DEV)
    dmap = (torch.rand(cout, H, W, generator=gen) + 0.1).to(DEV)
    gd = torch.empty(Bq, cin, H, W, device=DEV)
    s = _capi.stream_ptr()
    _capi.call("drsa_amd_relevance_unpool", gp.data_ptr(), am.data_ptr(), Bq, clones, cin, H, W, 2, 4, gd.data_ptr(), s)
    o_ref = torch.full((Bq, cout, H, W), -9.0, device=DEV)
    o_sp = torch.full_like(o_ref, -7.0)
    _capi.call("drsa_amd_conv_bwd_den_map", gd.data_ptr(), None, 2, wts.data_ptr(), 0, x.data_ptr(), dmap.data_ptr(),
               o_ref.data_ptr(), Bq, clones, cin, cout, H, W, 1, xm, 1e-7, s)
    _capi.call("drsa_amd_conv_bwd_den_map", gp.data_ptr(), am.data_ptr(), 4, wts.data_ptr(), 0, x.data_ptr(),
               dmap.data_ptr(), o_sp.data_ptr(), Bq, clones, cin, cout, H, W, 1, xm, 1e-7, s)
    torch.cuda.synchronize()
    assert torch.equal(o_sp, o_ref)
    assert not torch.equal(o_ref, torch.zeros_like(o_ref))


def test_den_map_pool24_bounds():
    lib = _capi.lib()
    assert lib.drsa_amd_conv_bwd_has_kernel_pw(64, 64, 24, 1, 4) == 0       # W / 4 = 6: not whole float4 groups
    assert lib.drsa_amd_conv_bwd_has_kernel_pw(64, 64, 16, 1, 4) == 0       # 8 x 8 tiles at W < 32: unpool path
    assert lib.drsa_amd_conv_bwd_has_kernel_pw(64, 64, 256, 2, 4) == 0      # ng 2 under a 2x4 pool: unpool path


def test_vggish_fp32_plan_has_no_unpool():
    from drsa_audio_amd.engine import get_engine
    from drsa_audio_amd.xai.explain.attribute import compute_relevances
    net = vggish().to(DEV)
    comp = NameMapComposite(LRP_NAME_MAP_VGGISH, canonizers=[SequentialMergeBatchNorm()])
    x = logmel(2, 128, 256, seed=8).to(DEV)
    compute_relevances(net, x, comp, class_idx=1)
    eng = get_engine(net, comp)
    eng.trace = []
    compute_relevances(net, x, comp, class_idx=1)
    torch.cuda.synchronize()
    tags = [t for t, _, _ in eng.trace]
    eng.trace = None
    assert "conv_bwd:features.3" in tags and not any(t.startswith("maxpool_bwd") for t in tags), tags
