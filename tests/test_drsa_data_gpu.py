"""DRSA training-data extraction (R16) on the HIP engine vs the oracle (GPU).

Parity: activation and context vectors are bit-identical to the exact-order oracle
(lrp_ref mode="exact" capturing (a, R) at the layer, then the reference's
get_vectors_from_maps / compute_context_vectors restated in drsa_ref); the same global numpy
RNG stream draws the locations.  normalize_vectors within 2e-6 relative (fp64 reduction vs
torch's float32 mean).
"""
import numpy as np
import pytest
import torch

import drsa_ref
import lrp_ref
from lrp_common import gtzan128, logmel, spec, toy
from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN, LRP_NAME_MAP_TOY
from drsa_audio_amd.zennit.composites import NameMapComposite

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _gpu(m):
    import copy
    return copy.deepcopy(m).to(DEV)


def _oracle_maps(m, nm, x, layer, class_idx):
    _, _, (act, rel) = lrp_ref.lrp(m, spec(nm), x, class_idx=class_idx, mode="exact", capture=layer)
    return act, rel


@pytest.mark.parametrize("layer_idx", [7, 4, 8, 13])
def test_get_intermediate_maps_bit_exact(layer_idx):
    from drsa_audio_amd.xai.drsa.preprocessing import get_intermediate
    net = gtzan128()
    x = logmel(3, seed=layer_idx)
    act, rel = _oracle_maps(net, LRP_NAME_MAP_GTZAN, x, f"features.{layer_idx}", 3)
    a, r = get_intermediate(_gpu(net), x.to(DEV), NameMapComposite(LRP_NAME_MAP_GTZAN), layer_idx, 3,
                            attr_batch_size=2)
    assert torch.equal(a.cpu(), act)
    assert torch.equal(r.cpu(), rel)


@pytest.mark.parametrize("layout", [0, 1])
def test_preprocess_data_sampled_bit_exact(layout):
    from drsa_audio_amd.xai.drsa.preprocessing import preprocess_data
    net = gtzan128()
    x = logmel(5, seed=2)
    act, rel = _oracle_maps(net, LRP_NAME_MAP_GTZAN, x, "features.7", 6)
    np.random.seed(123)
    idx = drsa_ref.sample_spatial_locations(5, act.shape[-2:], 20)
    if layout == 0:
        va = drsa_ref.get_vectors_from_maps(act, idx)
        vr = drsa_ref.get_vectors_from_maps(rel, idx)
    else:
        b, d = act.shape[:2]
        am, rm = act.reshape(b, d, -1), rel.reshape(b, d, -1)
        va = torch.stack([am[i][:, idx[i]].T for i in range(b)]).reshape(-1, d)
        vr = torch.stack([rm[i][:, idx[i]].T for i in range(b)]).reshape(-1, d)
    ctx = drsa_ref.compute_context_vectors(va, vr)
    np.random.seed(123)
    A, C = preprocess_data(_gpu(net), x.to(DEV), NameMapComposite(LRP_NAME_MAP_GTZAN), 7, 6, num_locations=20,
                           attr_batch_size=3, layout=layout)
    assert A.shape == (100, 64)
    assert torch.equal(A.cpu(), va)
    assert torch.equal(C.cpu(), ctx)


def test_preprocess_data_all_locations_inference_branch():
    from drsa_audio_amd.xai.drsa.preprocessing import preprocess_data
    net = toy()
    x = logmel(2, 64, 64, seed=3)
    act, rel = _oracle_maps(net, LRP_NAME_MAP_TOY, x, "features.4", 1)
    A, C = preprocess_data(_gpu(net), x.to(DEV), NameMapComposite(LRP_NAME_MAP_TOY), 4, 1)
    b, d = act.shape[:2]
    va = act.reshape(b, d, -1).transpose(-2, -1)              # intended D3 semantics
    vr = rel.reshape(b, d, -1).transpose(-2, -1)
    assert A.shape == va.shape
    assert torch.equal(A.cpu(), va)
    assert torch.equal(C.cpu(), drsa_ref.compute_context_vectors(va, vr))


def test_get_vectors_and_normalize_vs_reference_fixture(golden_dir):
    from drsa_audio_amd.xai.drsa.preprocessing import get_vectors_from_maps, normalize_vectors
    fx = np.load(f"{golden_dir}/preprocessing_fixture.npz")
    va = get_vectors_from_maps(torch.from_numpy(fx["maps_a"]).to(DEV), fx["idx"])
    assert np.array_equal(va.cpu().numpy(), fx["vec_a"])
    na = normalize_vectors(torch.from_numpy(fx["vec_a"]).to(DEV)).cpu().numpy()
    nc = normalize_vectors(torch.from_numpy(fx["ctx"]).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(na, fx["norm_a"], rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(nc, fx["norm_ctx"], rtol=2e-6, atol=1e-7)


def test_training_data_feeds_drsa_and_matches_oracle_objective(tmp_path):
    """C3 pipeline on device: LRP capture at j=7 -> 20 locations -> normalise -> DRSA step; the
    objective on the extracted data matches the oracle's on the oracle-extracted data."""
    from drsa_audio_amd.xai.drsa.preprocessing import drsa_training_data
    from drsa_audio_amd.xai.drsa.drsa import drsa_step
    from drsa_audio_amd.xai.drsa.cluster.getdrsadata import load_and_normalize_data, save_data
    net = gtzan128()
    x = logmel(8, seed=5)
    np.random.seed(7)
    A, C = drsa_training_data(_gpu(net), x.to(DEV), NameMapComposite(LRP_NAME_MAP_GTZAN), 7, 3, num_locations=20)
    act, rel = _oracle_maps(net, LRP_NAME_MAP_GTZAN, x, "features.7", 3)
    np.random.seed(7)
    idx = drsa_ref.sample_spatial_locations(8, act.shape[-2:], 20)
    va = drsa_ref.get_vectors_from_maps(act, idx)
    ctx = drsa_ref.compute_context_vectors(va, drsa_ref.get_vectors_from_maps(rel, idx))
    Ar, Cr = drsa_ref.normalize_vectors(va), drsa_ref.normalize_vectors(ctx)
    np.testing.assert_allclose(A.cpu().numpy(), Ar.numpy(), rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(C.cpu().numpy(), Cr.numpy(), rtol=2e-6, atol=1e-7)
    U0 = torch.from_numpy(np.linalg.qr(np.random.default_rng(0).standard_normal((64, 64)))[0].astype(np.float32))
    _, f = drsa_step(A, C, U0.to(DEV), 4)
    _, f_ref, _ = drsa_ref.step(Ar, Cr, U0, 4)
    assert abs(float(f) - f_ref) <= 1e-4 * abs(f_ref)
    # pickle round trip in the reference's dataset format
    p = save_data(va, ctx, layer=7, sample_class="blues", output_path=str(tmp_path))
    a2, c2 = load_and_normalize_data(p, DEV)
    np.testing.assert_allclose(a2.cpu().numpy(), Ar.numpy(), rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(c2.cpu().numpy(), Cr.numpy(), rtol=2e-6, atol=1e-7)


def test_prototype_search_matches_oracle():
    """get_prototypes_ts (prototypes.py:14-130) on device vs the oracle: same winning subset,
    objectives within 1e-5 relative, bit-exact prototype vectors."""
    from drsa_audio_amd.xai.drsa.prototypes import get_prototypes_ts, subset_objectives
    net = gtzan128()
    B, n, K = 16, 4, 4
    x = logmel(B, seed=31)
    U = torch.from_numpy(np.linalg.qr(np.random.default_rng(3).standard_normal((64, 64)))[0].astype(np.float32))
    a, c, names, sp = get_prototypes_ts(_gpu(net), 7, U.to(DEV), NameMapComposite(LRP_NAME_MAP_GTZAN), x.to(DEV), 3,
                                        loaded_samples=[f"s{i}" for i in range(B)], num_concepts=K, n=n, seed=42)
    perm = torch.randperm(B, generator=torch.Generator().manual_seed(42))
    act, rel = _oracle_maps(net, LRP_NAME_MAP_GTZAN, x[perm], "features.7", 3)
    b, d = act.shape[:2]
    va = act.reshape(b, d, -1).transpose(-2, -1)
    vc = drsa_ref.compute_context_vectors(va, rel.reshape(b, d, -1).transpose(-2, -1))
    objs = [float(drsa_ref.obj_val(va[i * n:(i + 1) * n].reshape(-1, d), vc[i * n:(i + 1) * n].reshape(-1, d), U, K,
                                   d // K)) for i in range(B // n)]
    best = int(np.argmax(objs))
    assert names == [f"s{int(i)}" for i in perm[best * n:(best + 1) * n]]
    assert torch.equal(a.cpu(), va[best * n:(best + 1) * n].reshape(-1, d))
    assert torch.equal(c.cpu(), vc[best * n:(best + 1) * n].reshape(-1, d))
    got = subset_objectives(va.to(DEV).contiguous(), vc.to(DEV).contiguous(), U.to(DEV), K, n).cpu().numpy()
    np.testing.assert_allclose(got, objs, rtol=1e-5)
    assert sp is not None and len(sp) == n


def _rank_local_worker(rank, world, port, x_local, q, backend="gloo", steps=30):
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests"), os.path.join(root, "oracle")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from lrp_common import gtzan128
    from drsa_audio_amd.xai.drsa.preprocessing import drsa_training_data
    from drsa_audio_amd.xai.drsa.distributed import sharded_run
    from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN
    from drsa_audio_amd.zennit.composites import NameMapComposite
    np.random.seed(7)
    A, C = drsa_training_data(gtzan128().to(dev), x_local.to(dev), NameMapComposite(LRP_NAME_MAP_GTZAN), 7, 3,
                              num_locations=20, group=dist.group.WORLD)
    U0 = torch.from_numpy(np.linalg.qr(np.random.default_rng(0).standard_normal((64, 64)))[0].astype(np.float32))
    if steps:
        U, traj = sharded_run(A, C, U0.to(dev), 4, steps)
    else:
        U, traj = U0, np.zeros(0)
    q.put((rank, A.cpu().numpy(), C.cpu().numpy(), traj, U.cpu().numpy(), float(np.random.rand())))
    dist.destroy_process_group()


def test_rank_local_training_data_two_ranks_equals_single_process():
    """SURVEY §8(e) per-GPU extraction: two ranks on cuda:0 (gloo) each extract only their own
    samples (5 + 3 of an 8-sample batch) with drsa_training_data(group=WORLD): the location draws
    follow the global numpy stream and the normalisation runs over both ranks' rows, so the rows
    equal the single-process result (within 1 ulp), and the row-sharded DRSA trajectory on them
    equals the unsharded run within 1e-5."""
    import socket
    import torch.multiprocessing as mp
    from drsa_audio_amd.xai.drsa.preprocessing import drsa_training_data
    from drsa_audio_amd.xai.drsa.drsa import DrsaWorkspace, drsa_run
    net = gtzan128()
    x = logmel(8, seed=5)
    np.random.seed(7)
    A, C = drsa_training_data(_gpu(net), x.to(DEV), NameMapComposite(LRP_NAME_MAP_GTZAN), 7, 3, num_locations=20)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    parts = [x[:5].clone(), x[5:].clone()]
    procs = [ctx.Process(target=_rank_local_worker, args=(r, 2, port, parts[r], q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r[0]: r[1:] for r in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    Ag = np.concatenate([res[0][0], res[1][0]])
    Cg = np.concatenate([res[0][1], res[1][1]])
    A_, C_ = A.cpu().numpy(), C.cpu().numpy()
    assert Ag.shape == A_.shape == (160, 64)
    for got, ref in ((Ag, A_), (Cg, C_)):
        ulp = np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
        assert ulp.max() <= 1, ulp.max()
    assert np.array_equal(res[0][2], res[1][2]) and np.array_equal(res[0][3], res[1][3])
    U0 = torch.from_numpy(np.linalg.qr(np.random.default_rng(0).standard_normal((64, 64)))[0].astype(np.float32))
    _, traj1 = drsa_run(A, C, U0.to(DEV), 4, 30, DrsaWorkspace(A.size(0), 64, 4, DEV))
    traj1 = traj1.cpu().numpy()
    assert np.max(np.abs(res[0][2] - traj1) / np.abs(traj1)) < 1e-5


def _spawn_ranks(parts, backend="gloo", steps=30):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_local_worker, args=(r, len(parts), port, parts[r], q, backend, steps))
             for r in range(len(parts))]
    for p in procs:
        p.start()
    res = {r[0]: r[1:] for r in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_rank_local_training_data_rccl_world1():
    """drsa_training_data(group=) over an RCCL ('nccl') group, whose size exchange
    starts from a host tensor: one rank, rows equal to the ungrouped call bit for bit."""
    from drsa_audio_amd.xai.drsa.preprocessing import drsa_training_data
    x = logmel(4, seed=9)
    np.random.seed(7)
    A, C = drsa_training_data(_gpu(gtzan128()), x.to(DEV), NameMapComposite(LRP_NAME_MAP_GTZAN), 7, 3,
                              num_locations=20)
    r_after = float(np.random.rand())
    res = _spawn_ranks([x.clone()], backend="nccl", steps=0)
    assert np.array_equal(res[0][0], A.cpu().numpy()) and np.array_equal(res[0][1], C.cpu().numpy())
    assert res[0][4] == r_after                       # the numpy stream advanced identically


def test_rank_local_training_data_empty_slice():
    """a rank with an empty slice returns empty rows instead of raising before the
    collectives (which stranded the other ranks); the other rank's rows equal the single-process
    result within 1 ulp and both ranks leave the numpy stream where one process would."""
    from drsa_audio_amd.xai.drsa.preprocessing import drsa_training_data
    x = logmel(3, seed=12)
    np.random.seed(7)
    A, C = drsa_training_data(_gpu(gtzan128()), x.to(DEV), NameMapComposite(LRP_NAME_MAP_GTZAN), 7, 3,
                              num_locations=20)
    r_after = float(np.random.rand())
    res = _spawn_ranks([x.clone(), x[:0].clone()], steps=0)
    assert res[1][0].shape == (0, 64) and res[1][1].shape == (0, 64)
    for got, ref in ((res[0][0], A.cpu().numpy()), (res[0][1], C.cpu().numpy())):
        ulp = np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
        assert ulp.max() <= 1, ulp.max()
    assert res[0][4] == res[1][4] == r_after
