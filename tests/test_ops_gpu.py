"""PyTorch-ROCm custom ops (drsa_audio_amd/ops.py, torch.ops.drsa_amd.*): bit-identical to the
ctypes path, fake kernels for tracing, and capturable in a HIP (CUDA) graph."""
import numpy as np
import pytest
import torch

from gen_fixtures import drsa_inputs
from lrp_common import gtzan128, logmel, u64

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


@pytest.fixture(scope="module")
def ops():
    import drsa_audio_amd.ops  # noqa: F401  (registers torch.ops.drsa_amd)
    return torch.ops.drsa_amd


def _drsa(N=4000, d=64, seed=3):
    A, C = drsa_inputs(N, d, seed)
    U = np.linalg.qr(np.random.default_rng(seed).standard_normal((d, d)))[0].astype(np.float32)
    return [torch.from_numpy(v).to(DEV) for v in (A, C, U)]


def test_drsa_ops_equal_ctypes_path(ops):
    from drsa_audio_amd.xai.drsa.drsa import drsa_objective, drsa_run, drsa_step, orthogonalize
    from drsa_audio_amd.xai.explain.explainer import compute_subspace_relevances
    A, C, U = _drsa()
    Un, f = ops.drsa_step(A, C, U, 4)
    Ur, fr = drsa_step(A, C, U, 4)
    assert torch.equal(Un, Ur) and torch.equal(f, fr.reshape(()))
    assert torch.equal(ops.drsa_objective(A, C, U, 4), drsa_objective(A, C, U, 4).reshape(()))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        U1, t1 = ops.drsa_run(A, C, U, 4, 9)
        U2, t2 = drsa_run(A, C, U, 4, 9)
    torch.cuda.synchronize()
    assert torch.equal(U1, U2) and torch.equal(t1, t2)
    V = U + 0.1 * torch.randn_like(U)
    assert torch.equal(ops.polar(V), orthogonalize(V))
    act, ctx = A[:3000].reshape(3, 1000, 64), C[:3000].reshape(3, 1000, 64)
    assert torch.equal(ops.subspace_relevances(act, ctx, U, 4), compute_subspace_relevances(act, ctx, U, 4))


def test_fake_kernels_and_schema(ops):
    A, C, U = _drsa(N=512)
    torch.library.opcheck(ops.drsa_step, (A, C, U, 4), test_utils=("test_schema", "test_faketensor"))
    torch.library.opcheck(ops.subspace_relevances, (A.reshape(2, 256, 64), C.reshape(2, 256, 64), U, 4),
                          test_utils=("test_schema", "test_faketensor"))
    torch.library.opcheck(ops.polar, (U,), test_utils=("test_schema", "test_faketensor"))


def test_lrp_stage_ops_equal_engine_buffers(ops):
    """The stage ops reproduce the engine's own launches (conv forward of features.3, the
    projection forward, the final heatmap sort) bit for bit."""
    from drsa_audio_amd.engine import get_engine
    from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN
    from drsa_audio_amd.xai.explain.explainer import HeatmapGenerator
    net = gtzan128().to(DEV)
    hg = HeatmapGenerator(net, u64(), LRP_NAME_MAP_GTZAN, "blues", num_concepts=4, layer_idx=7, standard="sum")
    x = logmel(3, seed=7).to(DEV)
    hg.generate_subspace_heatmaps(x, to_host=False)
    eng = get_engine(hg.projectionmodel, hg.composite)
    st, rec = eng.stages[1], eng.last["stages"][1]
    y, amax, den = ops.lrp_conv_fwd(rec["in"], st.wts_fwd, st.bias3, None, st.cout, st.ng_fwd, True)
    assert torch.equal(y, rec["y"]) and torch.equal(amax, rec["amax"]) and torch.equal(den, rec["den"])
    st2, rec2 = eng.stages[2], eng.last["stages"][2]
    yp, ap = ops.projection_fwd(rec2["a"], st2.proj.U, True)
    assert torch.equal(yp, rec2["y"]) and torch.equal(ap, rec2["amax"])
    hm = eng.backward(cls=torch.full((3,), hg.class_idx, dtype=torch.int32, device=DEV), fanout=2)
    std, std_rel, sub, rel, mask = ops.heatmap_sort(hm, 4, True)
    for k, v in (("standard_heatmaps", std), ("standard_relevance", std_rel), ("subspace_heatmaps", sub),
                 ("subspace_relevances", rel), ("mask", mask)):
        assert torch.equal(v, hg.info_device[k]), k


def test_logmel_op_equals_loader(ops):
    import logmel_ref
    from drsa_audio_amd.utils.dataloading import Loader
    songs = torch.from_numpy(logmel_ref.synthetic_songs(2, seed=5)).to(DEV)
    chunks = songs[:, :48000].contiguous()
    a = ops.logmel(chunks, 800, 360, 128, 128, False)
    b = Loader("gtzan", device=DEV).transform_wav(chunks)
    assert torch.equal(a, b)


def test_graph_capture_of_ops_and_heatmap_generator(ops):
    """torch.cuda.graph captures the ops (no host sync inside) and the whole explain step of
    HeatmapGenerator; replays equal eager execution."""
    from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN
    from drsa_audio_amd.xai.explain.explainer import HeatmapGenerator
    A, C, U = _drsa()
    U_eager, f_eager = ops.drsa_step(A, C, U, 4)
    run_eager = ops.drsa_run(A, C, U, 4, 5)
    net = gtzan128().to(DEV)
    hg = HeatmapGenerator(net, u64(), LRP_NAME_MAP_GTZAN, "jazz", num_concepts=4, layer_idx=7)
    x = logmel(8, seed=3).to(DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):                     # warm-up: plans, buffers, workspaces
        hg.generate_subspace_heatmaps(x, to_host=False)
        ops.drsa_step(A, C, U, 4)
        ops.drsa_run(A, C, U, 4, 5)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    eager = {k: v.clone() for k, v in hg.info_device.items()}
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        Ug, fg = ops.drsa_step(A, C, U, 4)
        Ur, tr = ops.drsa_run(A, C, U, 4, 5)
        hg.generate_subspace_heatmaps(x, to_host=False)
        out = hg.info_device
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(Ug, U_eager) and torch.equal(fg, f_eager)
    assert torch.equal(Ur, run_eager[0]) and torch.equal(tr, run_eager[1])
    for k, v in eager.items():
        assert torch.equal(out[k], v), k
