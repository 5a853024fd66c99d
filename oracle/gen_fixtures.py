"""Generate golden fixtures under tests/golden/ by running the REFERENCE code.

Runs only in the build container (needs /root/reference); nothing here is imported by the
product.  Tests import this module for its input-case tables (SORT_CASES, SUBREL_CASES, ...);
the reference itself is imported only inside the generator functions, never at import time.
The seeded DRSA row generator lives in ``drsa_audio_amd/utils/synthetic.py`` (re-exported here
for the fixture scripts).  The reference's ``cxai/xai/drsa/drsa.py`` has an
import typo (``from pathilib import Path``, drsa.py:4, defect D1); a one-line
``sys.modules['pathilib']`` shim supplies the name, the file itself is unmodified.

Fixtures written (all small, numpy ``.npz`` / ``.npy``, no pickles):
* drsa_fixture.npz  — generalized_fmean/objective_fn values, obj_val + autograd grad,
                      orthogonalize, 10-step SubspaceOptimizer.run trajectories and
                      final U for a tiny (N=256, d=16, K=4) and a C3-width
                      (N=1000, d=64, K=4) problem, drsa.main's initial-U schedule.
* u64_seed42.npy    — ortho_group.rvs(64) after np.random.seed(42) (bench U, drsa.py:265-272).
* model_fixture.npz — module names of the GTZAN-128 / toy / ProjectionModel nets,
                      parameter checksums after torch.manual_seed(0) (reference
                      VGGType), ProjectionModel forward outputs.
* preprocessing_fixture.npz — get_vectors_from_maps / normalize_vectors /
                      compute_context_vectors on fixed small maps (reference
                      preprocessing formulas; module itself needs zennit, so these
                      are evaluated from the reference source text — see below).

Input data are generated with numpy ``default_rng`` (PCG64: stable across numpy
versions), so the tests regenerate them from the seed instead of storing them.
"""
from __future__ import annotations

import os
import pathlib
import sys
import tempfile
import types

import numpy as np
import torch

_ROOT = str(pathlib.Path(__file__).resolve().parent.parent)
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)
from drsa_audio_amd.utils.synthetic import drsa_inputs  # noqa: E402,F401  (fixture rows)

REF = "/root/reference"
OUT = pathlib.Path(__file__).resolve().parent.parent / "tests" / "golden"


def _import_reference():
    sys.modules.setdefault("pathilib", types.SimpleNamespace(Path=pathlib.Path))
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from cxai.xai.drsa import drsa as rdrsa
    from cxai.model import create_model as rcm
    from cxai.model import modify_model as rmm
    return rdrsa, rcm, rmm


def _drsa(rdrsa):
    out = {}
    # generalized_fmean / objective_fn on a fixed [N, K] input
    rng = np.random.default_rng(7)
    X = np.abs(rng.standard_normal((50, 4))).astype(np.float32)
    out["fmean_in"] = X
    out["fmean_p2"] = rdrsa.generalized_fmean(torch.from_numpy(X), 2).numpy()
    out["fmean_p05"] = rdrsa.generalized_fmean(torch.from_numpy(X), 0.5).numpy()
    out["objective"] = rdrsa.objective_fn(torch.from_numpy(X)).numpy()

    for tag, (N, d, K, seed, steps) in {"small": (256, 16, 4, 11, 10),
                                         "c3w": (1000, 64, 4, 12, 10)}.items():
        A, C = drsa_inputs(N, d, seed)
        np.random.seed(100 + seed)
        from scipy.stats import ortho_group
        U0 = ortho_group.rvs(d).astype(np.float32)
        At, Ct, Ut = map(torch.from_numpy, (A, C, U0))
        Ug = Ut.clone().requires_grad_(True)
        f = rdrsa.SubspaceOptimizer.obj_val(At, Ct, Ug, rdrsa.objective_fn, K, d // K)
        f.backward()
        out[f"{tag}_meta"] = np.array([N, d, K, seed, steps])
        out[f"{tag}_U0"] = U0
        out[f"{tag}_A_checksum"] = np.array([A.sum(dtype=np.float64), C.sum(dtype=np.float64)])
        out[f"{tag}_f0"] = np.array(float(f.detach()))
        out[f"{tag}_G0"] = Ug.grad.numpy().copy()
        out[f"{tag}_orth0"] = rdrsa.orthogonalize((Ut + Ug.grad).detach()).numpy()
        with tempfile.TemporaryDirectory() as td:
            opt = rdrsa.SubspaceOptimizer(Ut.clone(), At, Ct, td, num_concepts=K,
                                          device=torch.device("cpu"))
            losses = []
            orig_save = opt.save_train_stats
            opt.save_train_stats = lambda arr: losses.extend(float(a) for a in arr)
            opt.save_model = lambda: None
            opt.run(steps=steps)
            out[f"{tag}_traj"] = np.array(losses)
            out[f"{tag}_Ufinal"] = opt.U.detach().numpy().copy()

    # drsa.main initial-U schedule: record the U handed to each run's optimiser
    seen = []
    cls = rdrsa.SubspaceOptimizer
    orig_init, orig_run = cls.__init__, cls.run

    def rec_init(self, U, *a, **k):
        seen.append(U.detach().numpy().copy())
        orig_init(self, U, *a, **k)
    cls.__init__ = rec_init
    cls.run = lambda self, steps=2000: None
    try:
        A, C = drsa_inputs(64, 16, 5)
        with tempfile.TemporaryDirectory() as td:
            rdrsa.main(torch.from_numpy(A), torch.from_numpy(C), td, num_concepts=4,
                       steps=1, runs=3, seed=42, device=torch.device("cpu"))
    finally:
        cls.__init__, cls.run = orig_init, orig_run
    out["main_U_runs"] = np.stack(seen)
    return out


def _models(rcm, rmm):
    out = {}
    torch.manual_seed(0)
    gtzan = rcm.VGGType(n_filters=(32, 32, 64, 64, 128), n_dense=128,
                        pool_kernels=((2, 2),) * 5, dropout=0.4, input_size=(128, 128),
                        conv_bn=False, dense_bn=False, block_depth=1)
    gtzan.eval()
    names = [n for n, _ in gtzan.named_modules() if n.count(".") == 1]
    out["gtzan_names"] = np.array(names)
    out["gtzan_param_names"] = np.array([n for n, _ in gtzan.named_parameters()])
    out["gtzan_param_sums"] = np.array([float(p.double().sum()) for p in gtzan.parameters()])
    out["gtzan_param_abs"] = np.array([float(p.double().abs().sum()) for p in gtzan.parameters()])
    rng = np.random.default_rng(1)
    x = rng.standard_normal((2, 1, 128, 128)).astype(np.float32)
    out["gtzan_x"] = x
    with torch.no_grad():
        out["gtzan_logits"] = gtzan(torch.from_numpy(x)).numpy()
    np.random.seed(42)
    from scipy.stats import ortho_group
    U = torch.tensor(ortho_group.rvs(64), dtype=torch.float32)
    pm = rmm.ProjectionModel(gtzan, 7, U, 4, case="gtzan")
    pm.eval()
    out["proj_names"] = np.array([n for n, _ in pm.named_modules() if n.count(".") == 1])
    with torch.no_grad():
        out["proj_logits"] = pm(torch.from_numpy(x)).numpy()
        h = pm.features[:9](torch.from_numpy(x))           # ... relu7 -> projection
        out["proj_h"] = h[:, :64].numpy()               # first 64 positions only
    # toy (only runnable through ProjectionModel, defect D6)
    torch.manual_seed(0)
    toy = rcm.VGGType(n_filters=(8, 8, 16, 16, 16), n_dense=32, n_classes=2,
                      pool_kernels=((2, 2),) * 5, dropout=0.0, input_size=(64, 64),
                      conv_bn=False, dense_bn=False, block_depth=1)
    toy.eval()
    out["toy_names"] = np.array([n for n, _ in toy.named_modules() if n.count(".") == 1])
    out["toy_param_sums"] = np.array([float(p.double().sum()) for p in toy.parameters()])
    Ut = torch.eye(16)
    pmt = rmm.ProjectionModel(toy, 7, Ut, 1, case="toy")
    xt = rng.standard_normal((1, 1, 64, 64)).astype(np.float32)
    out["toy_x"] = xt
    with torch.no_grad():
        out["toy_logits"] = pmt(torch.from_numpy(xt)).numpy()
    # VGGish-BN shape contract (C5)
    torch.manual_seed(0)
    vgg = rcm.VGGType(n_filters=(64, 64, 100, 128, 128), n_dense=100,
                      pool_kernels=((2, 4), (2, 2), (2, 2), (2, 2), (2, 2)), dropout=0.3,
                      input_size=(128, 256), conv_bn=True, dense_bn=True)
    out["vggish_names"] = np.array([n for n, _ in vgg.named_modules() if n.count(".") == 1])
    out["vggish_param_sums"] = np.array([float(p.double().sum()) for p in vgg.parameters()])
    return out


def _preprocessing():
    """preprocessing.py imports zennit (absent), so its pure-torch helpers cannot be
    imported; they are evaluated here by exec'ing ONLY their function source text
    extracted from the reference file (no module import, nothing persisted)."""
    import ast
    src = pathlib.Path(REF, "cxai/xai/drsa/preprocessing.py").read_text()
    tree = ast.parse(src)
    keep = {"compute_context_vectors", "normalize_vectors", "get_vectors_from_maps"}
    ns = {"torch": torch, "np": np, "Tuple": tuple}
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name in keep:
            mod = ast.Module(body=[node], type_ignores=[])
            exec(compile(mod, "preprocessing.py", "exec"), ns)
    rng = np.random.default_rng(9)
    maps_a = np.maximum(rng.standard_normal((3, 8, 6, 6)), 0).astype(np.float32)
    maps_r = rng.standard_normal((3, 8, 6, 6)).astype(np.float32)
    idx = np.stack([rng.choice(36, 5, replace=False) for _ in range(3)])
    va = ns["get_vectors_from_maps"](torch.from_numpy(maps_a), idx)
    vr = ns["get_vectors_from_maps"](torch.from_numpy(maps_r), idx)
    ctx = ns["compute_context_vectors"](va, vr)
    return {"maps_a": maps_a, "maps_r": maps_r, "idx": idx, "vec_a": va.numpy(),
            "vec_r": vr.numpy(), "ctx": ctx.numpy(),
            "norm_a": ns["normalize_vectors"](va).numpy(),
            "norm_ctx": ns["normalize_vectors"](ctx).numpy()}


def _extract(relpath: str, names, ns):
    """exec ONLY the named top-level functions of a reference source file into ``ns`` (the
    module itself imports zennit, absent here).  Nothing is persisted."""
    import ast
    tree = ast.parse(pathlib.Path(REF, relpath).read_text())
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name in names:
            exec(compile(ast.Module(body=[node], type_ignores=[]), relpath, "exec"), ns)
    return ns


# compute_subspace_relevances cases: (b or 0 for a 2-D [N, d] input, N, d, K, seed)
SUBREL_CASES = [(1, 20000, 64, 4, 1), (3, 1000, 16, 1, 2), (3, 500, 64, 8, 3), (1, 3000, 128, 16, 4),
                (3, 777, 128, 4, 5), (2, 20, 100, 4, 6), (1, 5000, 100, 4, 7), (0, 300, 64, 4, 8),
                (3, 1, 16, 16, 9), (1, 20000, 128, 8, 10), (3, 4099, 32, 2, 11), (1, 2048, 100, 1, 12)]


def subrel_inputs(b: int, N: int, d: int, seed: int):
    """act = |N(0,1)| (post-ReLU), ctx = N(0,1) + 0.3, U = N(0,1)/sqrt(d) (any square matrix;
    orthogonality is not needed by the formula, and a LAPACK-free U regenerates bit-exactly)."""
    rng = np.random.default_rng(5000 + seed)
    shape = (b, N, d) if b else (N, d)
    act = np.abs(rng.standard_normal(shape)).astype(np.float32)
    ctx = (rng.standard_normal(shape) + 0.3).astype(np.float32)
    U = (rng.standard_normal((d, d)) / np.sqrt(d)).astype(np.float32)
    return act, ctx, U


def _subspace_relevances():
    """Reference compute_subspace_relevances (explainer.py:206-242) on SUBREL_CASES."""
    from typing import List, Tuple
    ns = _extract("cxai/xai/explain/explainer.py", {"compute_subspace_relevances"},
                  {"torch": torch, "np": np, "List": List, "Tuple": Tuple})
    out = {}
    for i, (b, N, d, K, seed) in enumerate(SUBREL_CASES):
        act, ctx, U = subrel_inputs(b, N, d, seed)
        r = ns["compute_subspace_relevances"](torch.from_numpy(act), torch.from_numpy(ctx),
                                              torch.from_numpy(U), K)
        out[f"case{i}_meta"] = np.array([b, N, d, K, seed])
        out[f"case{i}_rel"] = r.numpy()
        out[f"case{i}_checksum"] = np.array([act.sum(dtype=np.float64), ctx.sum(dtype=np.float64),
                                             U.sum(dtype=np.float64)])
    return out


# long-horizon reference runs: tag -> (N, d, K, data seed, U0 source, steps)
DRSA_LONG = {"c3": (20000, 64, 4, 3, "u64_seed42", 2000),     # SURVEY 8(d) C3, drsa.py:76 default
             "c4": (160000, 64, 8, 3, "u64_seed42", 10),      # C4 shape (8 x 20 000 rows)
             "d100": (20000, 100, 4, 13, "ortho100", 500)}    # VGGish j=19 (getdrsadata.py:119)


def _drsa_long(rdrsa):
    from scipy.stats import ortho_group
    out = {}
    for tag, (N, d, K, seed, usrc, steps) in DRSA_LONG.items():
        A, C = drsa_inputs(N, d, seed)
        if usrc == "u64_seed42":
            np.random.seed(42)
            U0 = ortho_group.rvs(64).astype(np.float32)
        else:
            np.random.seed(100)
            U0 = ortho_group.rvs(d).astype(np.float32)
        opt = rdrsa.SubspaceOptimizer(torch.from_numpy(U0), torch.from_numpy(A), torch.from_numpy(C), "/nonexistent",
                                      num_concepts=K, device=torch.device("cpu"))
        losses = []
        opt.save_train_stats = lambda arr: losses.extend(float(a) for a in arr)
        opt.save_model = lambda: None
        t0 = __import__("time").time()
        opt.run(steps=steps)
        print(f"[gen_fixtures] reference run {tag}: {steps} steps in {__import__('time').time() - t0:.1f} s")
        out[f"{tag}_meta"] = np.array([N, d, K, seed, steps])
        out[f"{tag}_U0"] = U0
        out[f"{tag}_A_checksum"] = np.array([A.sum(dtype=np.float64), C.sum(dtype=np.float64)])
        out[f"{tag}_traj"] = np.array(losses)
        out[f"{tag}_Ufinal"] = opt.U.detach().numpy().copy()
    return out


def _drsa_main(rdrsa):
    """drsa.main (drsa.py:241-301) end to end on a small problem: every run's trajectory and final
    U, captured by replacing the two save methods (no files are read back)."""
    runs = []
    cls = rdrsa.SubspaceOptimizer
    orig_stats, orig_model = cls.save_train_stats, cls.save_model

    def rec_stats(self, arr):
        runs.append({"traj": np.array([float(a) for a in arr])})

    def rec_model(self):
        runs.append({"U": self.U.detach().numpy().copy()})
    cls.save_train_stats, cls.save_model = rec_stats, rec_model
    try:
        A, C = drsa_inputs(3000, 32, 17)
        with tempfile.TemporaryDirectory() as td:
            rdrsa.main(torch.from_numpy(A), torch.from_numpy(C), td, num_concepts=4, steps=25, runs=3, seed=42,
                       device=torch.device("cpu"))
    finally:
        cls.save_train_stats, cls.save_model = orig_stats, orig_model
    # save_model is called before save_train_stats (drsa.py:119-120)
    Us = [r["U"] for r in runs if "U" in r]
    trajs = [r["traj"] for r in runs if "traj" in r]
    return {"main_meta": np.array([3000, 32, 4, 17, 25, 3, 42]), "main_Ufinal": np.stack(Us),
            "main_traj": np.stack(trajs)}


def main_round2():
    """Round-2 fixtures (separate files, so round-1 fixtures stay byte-identical)."""
    OUT.mkdir(parents=True, exist_ok=True)
    rdrsa, _, _ = _import_reference()
    np.savez_compressed(OUT / "subspace_rel_fixture.npz", **_subspace_relevances())
    long = _drsa_long(rdrsa)
    long.update(_drsa_main(rdrsa))
    np.savez_compressed(OUT / "drsa_long_fixture.npz", **long)
    print("round-2 fixtures written to", OUT)


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    rdrsa, rcm, rmm = _import_reference()
    np.savez_compressed(OUT / "drsa_fixture.npz", **_drsa(rdrsa))
    np.random.seed(42)
    from scipy.stats import ortho_group
    np.save(OUT / "u64_seed42.npy", ortho_group.rvs(64).astype(np.float32))
    np.savez_compressed(OUT / "model_fixture.npz", **_models(rcm, rmm))
    np.savez_compressed(OUT / "preprocessing_fixture.npz", **_preprocessing())
    with open(OUT / "VERSIONS.txt", "w") as fh:
        import scipy
        fh.write(f"torch {torch.__version__}\nnumpy {np.__version__}\nscipy {scipy.__version__}\n"
                 f"python {sys.version.split()[0]}\n")
    print("fixtures written to", OUT)


# ------------------------------------------------------------------ round 3: zennit-free LRP pins
# sort_subspaces cases (B, K, H, W, seed); the reference squeezes the batch dim away at B = 1 (D7)
SORT_CASES = [(3, 4, 128, 128, 1), (2, 4, 64, 64, 2), (2, 4, 128, 256, 3), (4, 8, 32, 32, 4), (3, 2, 36, 52, 5),
              (5, 4, 16, 16, 6), (2, 16, 8, 8, 7), (3, 4, 6, 6, 8), (2, 4, 2, 2, 9), (6, 3, 20, 20, 10)]


def sort_inputs(B: int, K: int, H: int, W: int, seed: int) -> np.ndarray:
    """Heatmaps [B, K+1, H, W] (standard first): signed, heavy-tailed values; in the first case
    sample 1 is all zeros (every concept ties) and sample 2's concept 3 duplicates concept 1."""
    rng = np.random.default_rng(7000 + seed)
    hm = (rng.standard_normal((B, K + 1, H, W)) * np.exp(rng.standard_normal((B, K + 1, 1, 1)))).astype(np.float32)
    if seed == 1:
        hm[1] = 0.0
        hm[2, 3] = hm[2, 1]
    return hm


def _lrp_pins():
    """Reference functions executed from their source text (zennit is only imported at module level):
    lrp_output_modifier (attribute.py:111-160), SubspaceHook.backward (attribute.py:42-60) and
    HeatmapGenerator.sort_subspaces (explainer.py:151-176), plus the standard relevance line
    (explainer.py:120, a numpy sum over the last two axes)."""
    import ast
    from typing import Tuple
    ns = _extract("cxai/xai/explain/attribute.py", {"lrp_output_modifier"}, {"torch": torch, "Tuple": Tuple})
    out = {}
    rng = np.random.default_rng(11)
    logits = (rng.standard_normal((20, 10)) * 3).astype(np.float32)
    out["seed_logits"] = logits
    for tag, kw in {"cls3": dict(class_idx=3), "cls0_onehot": dict(class_idx=0, one_hot_encoded=True),
                    "all10": dict(num_classes=10), "all10_onehot": dict(num_classes=10, one_hot_encoded=True),
                    "cls9": dict(class_idx=9)}.items():
        out[f"seed_{tag}"] = ns["lrp_output_modifier"](**kw)(torch.from_numpy(logits)).numpy()
    try:                                           # D8: the all-classes mask needs B % num_classes == 0
        ns["lrp_output_modifier"](num_classes=10)(torch.from_numpy(logits[:16]))
        out["seed_all10_b16_raises"] = np.array(0)
    except RuntimeError:
        out["seed_all10_b16_raises"] = np.array(1)

    # SubspaceHook.backward: the method body needs only self.num_concepts / self.device
    tree = ast.parse(pathlib.Path(REF, "cxai/xai/explain/attribute.py").read_text())
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "SubspaceHook")
    fn = next(n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name == "backward")
    hns = {"torch": torch, "Tuple": Tuple}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), "attribute.py", "exec"), hns)
    # n = 64 pixels (8 x 8, a shape the projection kernels take); small integers, exact under the
    # U = I identities the GPU test uses, and compressible
    for tag, (b, n, K, dk) in {"k4": (2, 64, 4, 4), "k2": (1, 64, 2, 8), "k8": (1, 64, 8, 4),
                               "k5": (1, 64, 5, 4)}.items():
        g = rng.integers(-64, 65, (b * (K + 1), n, K, dk)).astype(np.float32)
        self_ = types.SimpleNamespace(num_concepts=K, device=torch.device("cpu"))
        res, = hns["backward"](self_, None, None, (torch.from_numpy(g.copy()),))
        out[f"hook_{tag}_in"] = g
        out[f"hook_{tag}_out"] = res.numpy()

    # sort_subspaces (a method; self is unused by the body)
    ecls = next(n for n in ast.parse(pathlib.Path(REF, "cxai/xai/explain/explainer.py").read_text()).body
                if isinstance(n, ast.ClassDef) and n.name == "HeatmapGenerator")
    fn = next(n for n in ecls.body if isinstance(n, ast.FunctionDef) and n.name == "sort_subspaces")
    sns = {"np": np, "Tuple": Tuple}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), "explainer.py", "exec"), sns)
    for i, (B, K, H, W, seed) in enumerate(SORT_CASES):
        hm = sort_inputs(B, K, H, W, seed)
        std, sub = hm[:, 0:1], hm[:, 1:]                 # explainer.py:113-114 (views)
        s_hm, s_rel, mask = sns["sort_subspaces"](None, sub)
        assert np.array_equal(s_hm, sub[np.arange(B)[:, None], mask])
        out[f"sort{i}_meta"] = np.array([B, K, H, W, seed])
        out[f"sort{i}_checksum"] = np.array([hm.sum(dtype=np.float64)])
        out[f"sort{i}_rel"] = s_rel
        out[f"sort{i}_mask"] = mask
        out[f"sort{i}_std_rel"] = std.sum(axis=(-2, -1)).flatten()      # explainer.py:120
    try:
        hm = sort_inputs(1, 4, 8, 8, 3)
        sns["sort_subspaces"](None, hm[:, 1:])
        out["sort_b1_raises"] = np.array(0)
    except IndexError:
        out["sort_b1_raises"] = np.array(1)                               # D7
    return out


# C5 long horizon: two VGGish-width problems (layers 26 / 33: d = 128, K = 16), N = 20 000
DRSA_C5 = {"j26": (20000, 128, 16, 26, 126), "j33": (20000, 128, 16, 33, 133)}   # N, d, K, data seed, U seed
C5_STEPS = 5000                                                                 # optsubspaces.py:23


def _drsa_c5(rdrsa, steps=C5_STEPS):
    from scipy.stats import ortho_group
    out = {}
    for tag, (N, d, K, seed, useed) in DRSA_C5.items():
        A, C = drsa_inputs(N, d, seed)
        np.random.seed(useed)
        U0 = ortho_group.rvs(d).astype(np.float32)
        opt = rdrsa.SubspaceOptimizer(torch.from_numpy(U0), torch.from_numpy(A), torch.from_numpy(C), "/nonexistent",
                                      num_concepts=K, device=torch.device("cpu"))
        losses = []
        opt.save_train_stats = lambda arr: losses.extend(float(a) for a in arr)
        opt.save_model = lambda: None
        t0 = __import__("time").time()
        opt.run(steps=steps)
        print(f"[gen_fixtures] reference run C5 {tag}: {steps} steps in {__import__('time').time() - t0:.1f} s")
        out[f"{tag}_meta"] = np.array([N, d, K, seed, useed, steps])
        out[f"{tag}_U0"] = U0
        out[f"{tag}_A_checksum"] = np.array([A.sum(dtype=np.float64), C.sum(dtype=np.float64)])
        out[f"{tag}_traj"] = np.array(losses)
        out[f"{tag}_Ufinal"] = opt.U.detach().numpy().copy()
    return out


def main_round3():
    """Round-3 fixtures (new files; earlier fixtures stay byte-identical)."""
    OUT.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(OUT / "lrp_pins_fixture.npz", **_lrp_pins())
    print("lrp pins written")
    if "--no-c5" not in sys.argv:
        rdrsa, _, _ = _import_reference()
        np.savez_compressed(OUT / "drsa_c5_fixture.npz", **_drsa_c5(rdrsa))
    print("round-3 fixtures written to", OUT)


# C4 long horizon: the C4 shape (N = 160 000 = 8 x 20 000 rows, d = 64, K = 8) for the reference's
# default 2 000 steps (drsa.py:76); same data seed and U0 as DRSA_LONG["c4"]
DRSA_C4_LONG = {"c4long": (160000, 64, 8, 3, "u64_seed42", 2000)}


def main_round4():
    """Round-4 fixture (new file; earlier fixtures stay byte-identical)."""
    OUT.mkdir(parents=True, exist_ok=True)
    rdrsa, _, _ = _import_reference()
    saved = dict(DRSA_LONG)
    DRSA_LONG.clear()
    DRSA_LONG.update(DRSA_C4_LONG)
    try:
        out = _drsa_long(rdrsa)
    finally:
        DRSA_LONG.clear()
        DRSA_LONG.update(saved)
    np.savez_compressed(OUT / "drsa_c4_fixture.npz", **out)
    print("round-4 fixtures written to", OUT)


if __name__ == "__main__":
    if "--round4" in sys.argv:
        main_round4()
    elif "--round3" in sys.argv:
        main_round3()
    elif "--round2" in sys.argv:
        main_round2()
    else:
        main()
