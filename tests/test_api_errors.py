"""Error behaviour of the host layer and the C ABI (CPU: every check fires before device work).

Mirrors the reference's runtime asserts (drsa.py:61-62, modify_model.py:40-41,
sound.py:37,41, dataloading.py:174-175) and the no-CPU-fallback rule: product entry points
raise on CPU tensors instead of computing there."""
import ctypes

import numpy as np
import pytest
import torch

from drsa_audio_amd import _capi


def test_subspace_optimizer_asserts_like_reference():
    from drsa_audio_amd.xai.drsa.drsa import SubspaceOptimizer
    U = torch.eye(8)
    A = torch.rand(10, 8)
    with pytest.raises(AssertionError):
        SubspaceOptimizer(U, A, A, ".", num_concepts=0)
    with pytest.raises(AssertionError):
        SubspaceOptimizer(U, A, A, ".", num_concepts=3)
    with pytest.raises(_capi.DrsaAmdError):
        SubspaceOptimizer(U, A, A, ".", num_concepts=4, device="cpu")


def test_projection_model_layer_range():
    from drsa_audio_amd.model.create_model import VGGType
    from drsa_audio_amd.model.modify_model import ProjectionModel
    m = VGGType(n_filters=(8, 8, 16, 16, 16), n_dense=32, n_classes=2, pool_kernels=((2, 2),) * 5,
                input_size=(64, 64), conv_bn=False, dense_bn=False, block_depth=1)
    for bad in (0, len(m.features)):
        with pytest.raises(ValueError):
            ProjectionModel(m, bad, torch.eye(16), 4)


def test_product_paths_refuse_cpu_tensors():
    from drsa_audio_amd.utils.dataloading import Loader
    from drsa_audio_amd.xai.drsa.preprocessing import normalize_vectors
    from drsa_audio_amd.xai.drsa.drsa import orthogonalize
    ld = Loader("gtzan", device="cpu")
    with pytest.raises(_capi.DrsaAmdError):
        ld.transform_wav(torch.zeros(1, 48000))
    with pytest.raises(_capi.DrsaAmdError):
        normalize_vectors(torch.rand(4, 8))
    with pytest.raises(_capi.DrsaAmdError):
        orthogonalize(torch.eye(8))


def test_lrp_engine_refuses_cpu_model():
    from drsa_audio_amd.model.create_model import VGGType
    from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN
    from drsa_audio_amd.zennit.composites import NameMapComposite
    from drsa_audio_amd.xai.explain.attribute import compute_relevances
    m = VGGType(n_filters=(32, 32, 64, 64, 128), n_dense=128, pool_kernels=((2, 2),) * 5, input_size=(128, 128),
                conv_bn=False, dense_bn=False, block_depth=1).eval()
    with pytest.raises(_capi.DrsaAmdError):
        compute_relevances(m, torch.zeros(1, 1, 128, 128), NameMapComposite(LRP_NAME_MAP_GTZAN), class_idx=0)


def test_get_slice_asserts():
    from drsa_audio_amd.utils.sound import get_slice
    # sound.py:41 compares the start point (seconds) with a sample count, as the reference does
    get_slice(torch.zeros(1, 16000 * 4), 3, 0, 1, 16000)
    with pytest.raises(AssertionError):
        get_slice(torch.zeros(1, 16000 * 4), 3, 17000, 1, 16000)
    with pytest.raises(AssertionError):                      # sound.py:37 not enough audio for 8 chunks
        get_slice(torch.zeros(1, 16000 * 10), 3, 0, 8, 16000)


def test_c_abi_argument_validation_without_gpu():
    lib = _capi.load()
    P = ctypes.c_void_p
    # logmel: null pointers, odd n_fft, frames past the end
    assert lib.drsa_amd_logmel(None, 1, 48000, 1, 0, 48000, 800, 360, 128, 128, 1, None, None, None, None, None, 0,
                               1, 1, -4.0, 1e-7, None, None) == -1
    assert b"null" in lib.drsa_amd_last_error()
    buf = (ctypes.c_float * 4)()
    ib = (ctypes.c_int * 4)()
    p, q = ctypes.cast(buf, P).value, ctypes.cast(ib, P).value
    assert lib.drsa_amd_logmel(p, 1, 48000, 1, 0, 48000, 801, 360, 128, 128, 1, p, q, q, q, p, 1, 1, 1, -4.0, 1e-7,
                               p, None) == -1
    assert lib.drsa_amd_logmel(p, 1, 48000, 1, 0, 48000, 800, 360, 128, 140, 1, p, q, q, q, p, 1, 1, 1, -4.0, 1e-7,
                               p, None) == -1
    assert b"frames" in lib.drsa_amd_last_error()
    # DRSA vectors: bad layout; pooled relevance with an odd map
    assert lib.drsa_amd_drsa_vectors(p, p, None, q, 1, 4, 4, 4, 1, 1, 2, 7, p, p, None) == -1
    assert lib.drsa_amd_drsa_vectors(p, p, q, q, 1, 4, 5, 4, 2, 2, 2, 0, p, p, None) == -1
    # pool kernel must divide the map
    assert lib.drsa_amd_maxpool_capture(p, None, p, q, None, 1, 4, 6, 8, 4, 4, None) == -1
    # Cin = 1 forward: one sample's cout x H x W past 2^31 (32-bit offsets)
    assert lib.drsa_amd_conv_fwd(p, p, p, p, p, q, p, 1, 1, 1 << 16, 256, 256, 1, 1, None) == -1
    assert b"2^31" in lib.drsa_amd_last_error()
    # joint DRSA: no problems
    assert lib.drsa_amd_drsa_run_multi(0, None, 10, 1, None) == -1
    # workspace size query rejects unsupported problems
    assert lib.drsa_amd_drsa_workspace_bytes(100, 48, 5) == 0      # K must divide d
    assert lib.drsa_amd_drsa_workspace_bytes(100, 100, 5) == 0     # padded 5 x 32 > 128
    assert lib.drsa_amd_drsa_workspace_bytes(100, 100, 4) > 0      # VGGish layer 19 (padded to 128)
    assert lib.drsa_amd_drsa_slab_floats(100, 4) == 128 * 128 + 4
    assert lib.drsa_amd_drsa_slab_floats(64, 4) == 64 * 64 + 4
    assert lib.drsa_amd_drsa_workspace_bytes(100, 128, 3) == 0
    # padded size 128 carries the cooperative finish's hand-off area (two 128 x 128 X buffers, the
    # per-workgroup scalars and the ticket) beyond the slabs: at N = 16 (one leaf) the partial slabs,
    # the reduced slab and that area
    slab = 4 * (128 * 128 + 4)
    assert lib.drsa_amd_drsa_workspace_bytes(16, 128, 16) >= 2 * slab + 2 * 128 * 128 * 4
    assert lib.drsa_amd_drsa_workspace_bytes(16, 64, 4) < 2 * 4 * (64 * 64 + 4) + 4096
    # compact den ring backward: pooled W >= 8 (W % 8 == 0) and H >= 2, as the forward's layout needs
    for H, W in ((4, 4), (0, 8), (4, 12)):
        with pytest.raises(_capi.DrsaAmdError, match="pooled H >= 2"):
            _capi.call("drsa_amd_conv_bwd_den_ring", p, None, p, 0, p, p, p, p, 1, 1, 32, 32, H, W, 1, 1, 1e-7, None)


def test_alphabeta_parameter_checks_like_zennit():
    from drsa_audio_amd.zennit.rules import AlphaBeta
    AlphaBeta(2.0, 1.0)
    AlphaBeta(1.0, 0.0)
    for a, b in ((-1.0, -2.0), (1.0, -0.0 - 1.0), (2.0, 0.5), (0.5, 0.0)):
        with pytest.raises(ValueError):
            AlphaBeta(a, b)


def test_coop_status_and_spin_budget_argument_errors():
    """drsa_amd_drsa_coop_status / drsa_amd_debug_coop_spin_budget reject bad arguments before any
    device work (the status itself is read on the GPU: tests/test_drsa_gpu.py)."""
    lib = _capi.lib()
    st = ctypes.c_int(7)
    assert lib.drsa_amd_drsa_coop_status(None, 100, 128, 16, ctypes.addressof(st), None) == _capi.DRSA_EINVAL
    assert lib.drsa_amd_drsa_coop_status(ctypes.c_void_p(16), 100, 128, 3, ctypes.addressof(st), None) == _capi.DRSA_EINVAL
    assert lib.drsa_amd_drsa_coop_status(ctypes.c_void_p(16), 0, 128, 16, ctypes.addressof(st), None) == _capi.DRSA_EINVAL
    assert lib.drsa_amd_debug_coop_spin_budget(-2) == _capi.DRSA_EINVAL
    assert lib.drsa_amd_debug_coop_spin_budget(-1) == 0
