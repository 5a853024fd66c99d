"""Concept-flipping evaluation (xai/pixelflipping/cpf.py, reference cpf.py:87-395) against the
loop-for-loop restatement oracle/cpf_ref.py: heatmaps from the exact-order oracle, flipping by
flip_ref with the same model forward.  Toy net (2 classes, 64x64 log-mels, layers 1 / 4 / 7 / 10),
so the CPU oracle stays small."""
import copy
import os
import pickle

import numpy as np
import pytest
import torch

import cpf_ref
from lrp_common import logmel, ortho, spec, toy
from drsa_audio_amd.utils.constants import LRP_NAME_MAP_TOY

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
GENRES = ["class1", "class2"]
LAYERS = [1, 4, 7, 10]
DIMS = {1: 8, 4: 8, 7: 16, 10: 16}


def _setup(seed=0):
    net = toy(seed)
    x = logmel(4, 64, 64, seed=40 + seed)           # 2 classes x 2 samples
    return net, x


def _gpu_forward(net):
    m = copy.deepcopy(net).to(DEV).eval()
    return m, (lambda b: m(b.to(DEV)))


def test_frob_and_separability_equal_oracle_on_identical_heatmaps():
    from drsa_audio_amd.xai.pixelflipping.cpf import frob, separability_peakness
    rng = np.random.default_rng(3)
    for K in (2, 4, 8):
        RU = (rng.standard_normal((5, K, 32, 32)) * np.exp(rng.standard_normal((5, K, 1, 1)))).astype(np.float32)
        assert frob(RU, K) == cpf_ref.frob(RU, K)
        assert separability_peakness(RU) == cpf_ref.separability_peakness(RU)


def test_interclass_concept_flipping_equals_oracle():
    from drsa_audio_amd.xai.pixelflipping.cpf import interclass_concept_flipping
    net, x = _setup(1)
    m, fwd = _gpu_forward(net)
    Us = {l: {g: ortho(DIMS[l], 10 * l + i) for i, g in enumerate(GENRES)} for l in LAYERS}
    got = interclass_concept_flipping(m, x, LRP_NAME_MAP_TOY, toy=True, num_concepts=4, device=DEV, Us=Us,
                                      layer_idcs=LAYERS, forward_func=fwd)
    ref = cpf_ref.interclass_concept_flipping(net, x, spec(LRP_NAME_MAP_TOY), Us, GENRES, 4, LAYERS, fwd, "toy")
    assert len(got) == len(LAYERS)
    for g, r in zip(got, ref):
        assert g.shape == (2, 2) and np.array_equal(g, r), (g, r)


def test_cf_random_subspace_equals_oracle():
    from drsa_audio_amd.xai.pixelflipping.cpf import cf_random_subspace
    net, x = _setup(2)
    m, _ = _gpu_forward(net)
    for layer, dim in ((4, 8), (7, 16)):
        np.random.seed(11)
        got = cf_random_subspace(m, x, LRP_NAME_MAP_TOY, layer, dim, case="toy", device=DEV, num_concepts=4)
        after = np.random.random()
        np.random.seed(11)
        ref = cpf_ref.cf_random_subspace(net, x, spec(LRP_NAME_MAP_TOY), layer, dim, GENRES, 4,
                                         "toy")
        assert np.random.random() == after                  # the global RNG consumed identically
        assert got.shape == (4, 4, 64, 64) and np.array_equal(got, ref)


def _write_runs(root, k, Us):
    """A directory of DRSA runs in drsa.main's format: {root}/{k}_concepts/{genre}/layer{L}/run{r}/."""
    import pandas as pd
    for L, per in Us.items():
        for g, U in per.items():
            for r, loss in ((1, 0.2), (2, 0.5), (3, 0.3)):    # run 2 is the best run
                p = os.path.join(root, f"{k}_concepts", g, f"layer{L}", f"run{r}")
                os.makedirs(p, exist_ok=True)
                Ur = U.numpy() if r == 2 else np.eye(U.size(0), dtype=np.float32)
                with open(os.path.join(p, "projection_matrix.pkl"), "wb") as fh:
                    pickle.dump(Ur.astype(np.float32), fh)
                pd.DataFrame({"loss": [0.1, loss]}).to_csv(os.path.join(p, "train_stats.csv"))


def test_perform_cf_and_sep_and_peak_equal_oracle(tmp_path):
    import flip_ref
    from drsa_audio_amd.xai.pixelflipping.cpf import perform_cf, sep_and_peak
    net, x = _setup(3)
    m, fwd = _gpu_forward(net)
    layers, ks = [4, 7], [2, 4]
    Us = {k: {l: {g: ortho(DIMS[l], 100 * k + 10 * l + i) for i, g in enumerate(GENRES)} for l in layers} for k in ks}
    runs = tmp_path / "runs"
    for k in ks:
        _write_runs(str(runs), k, Us[k])
    out = tmp_path / "out"
    res = perform_cf(m, x, LRP_NAME_MAP_TOY, str(out), path=str(runs), layer_idcs=layers, num_concepts=ks, toy=True,
                     device=DEV)
    rules = spec(LRP_NAME_MAP_TOY)
    for k in ks:
        for l in layers:
            R = np.concatenate([cpf_ref.heatmaps(net, rules, Us[k][l][g], k, l, x[2 * i:2 * i + 2], i, "toy")
                                for i, g in enumerate(GENRES)], 0)
            a_ref, _, _, _ = flip_ref.flip(fwd, x, torch.from_numpy(R), 16)
            with open(out / f"{k}_concepts" / f"aupcs_layer_{l}.pkl", "rb") as fh:
                saved = pickle.load(fh)                       # our own file
            assert np.array_equal(saved, a_ref) and np.array_equal(res[(k, l)], a_ref)
    # separability / peakness over the same DRSA subspaces (path/{prefix}/{k}_concepts layout)
    os.rename(runs, tmp_path / "runs_p")
    os.makedirs(tmp_path / "runs", exist_ok=True)
    os.rename(tmp_path / "runs_p", tmp_path / "runs" / "drsa")
    final = sep_and_peak(m, x, LRP_NAME_MAP_TOY, str(out), path=str(tmp_path / "runs"), layer_idcs=layers,
                         num_concepts=ks, toy=True, prefix="drsa", device=DEV)
    assert final.shape == (len(ks), 4, len(layers))
    for a, k in enumerate(ks):
        for b, l in enumerate(layers):
            RU = np.concatenate([cpf_ref.heatmaps(net, rules, Us[k][l][g], k, l, x[2 * i:2 * i + 2], i, "toy")
                                 for i, g in enumerate(GENRES)], 0)
            assert np.array_equal(final[a, :, b], np.array(cpf_ref.separability_peakness(RU)))
    with open(out / "drsa" / "sep_and_peak.pkl", "rb") as fh:
        assert np.array_equal(pickle.load(fh), final)
