"""Benchmark: explained samples/sec (LRP + DRSA subspace heatmaps, K=4) on MI355X.

Workload (BASELINE.json metric): GTZAN-128 VGG (random init, torch.manual_seed(0)),
HeatmapGenerator at layer j=7 (conv3 block, d=64) with K=4 subspaces, U = ortho_group.rvs(64)
(seed 42, committed fixture), synthetic 128x128 log-mel batches.  One step = one batch through
the whole hot path: forward, LRP backward with the K+1 relevance clones, split/sum/sort
(HeatmapGenerator.info semantics), inputs resident in HBM, outputs left in HBM.

  python bench.py [--gpus N --steps K --warmup W --batch B]
  (N>1: either under torchrun --nproc-per-node N, or bench.py spawns the N ranks itself
   (drsa_audio_amd/utils/launch.py) before any GPU call; each rank explains its own batch, no
   collective on the data path -> weak scaling; time = max over ranks.  The N>1 run adds the
   row-sharded DRSA leg (one RCCL all-reduce per step); every run has the task-parallel DRSA
   grid leg (the reference's 90 independent problems spread over the ranks, strong scaling).)

Also reported: per-kernel HIP-event timings of the dominant kernel (roofline), the standard
LRP rate at bs=64 (C2), the DRSA step rate at C3 (N=20000, d=64, K=4) with its objective
checked against the CPU oracle, and the CPU baseline (oracle's zennit-structured restatement,
K+1 batch replication like explainer.py:92) on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np
import torch

FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: dense fp32 MFMA (= vector) peak
BF16_MFMA_PEAK_TFLOPS = 2500.0     # MI355X_MICROARCH.md: dense bf16 MFMA peak (no sparsity)
HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synthetic_logmel(B, H=128, W=128, seed=1, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    e = torch.empty(B, 1, H, W).exponential_(generator=g)
    tilt = 10 ** (-3 * torch.arange(H).float() / (H - 1))
    return torch.clamp(torch.log10(e * tilt[None, None, :, None] + 1e-7), min=-4).to(device)


def gtzan128():
    from drsa_audio_amd.model.create_model import VGGType
    torch.manual_seed(0)
    return VGGType(n_filters=(32, 32, 64, 64, 128), n_dense=128, pool_kernels=((2, 2),) * 5, dropout=0.4,
                   input_size=(128, 128), conv_bn=False, dense_bn=False, block_depth=1).eval()


def load_u():
    return torch.from_numpy(np.load(os.path.join(ROOT, "tests", "golden", "u64_seed42.npy")))


# --------------------------------------------------------------------------- FLOP model
def kernel_macs(eng, B, K, standard="sum", launched=None):
    """Algorithmic multiply-accumulates per launch of each kernel tag for one batch of B
    explained samples ('Algorithmic work').  standard="sum": K relevance clones below
    the projection (the standard heatmap is their sum); "clone": K+1.

    `launched` (the tags one traced step actually ran) restricts the table to those kernels, so a
    whole-path sum counts exactly the work done (round 4's line also counted an unlaunched fused
    kernel: 1.224 instead of 0.884 GFLOP per sample)."""
    macs = {}
    rec = eng.last["stages"]
    clones_below = False
    for li in range(len(eng.stages) - 1, -1, -1):
        st = eng.stages[li]
        h, w = rec[li]["H"], rec[li]["W"]
        if st.proj is not None:
            d = st.cout
            macs["projection_fwd"] = B * h * w * d * d * 2
            # g1 U, [clone 0,] the K concept blocks (d_k x d each)
            macs["projection_bwd"] = B * h * w * (d * d + (d * d if standard == "clone" else 0) + d * d)
            clones_below = True
        nq = (K + (1 if standard == "clone" else 0)) if clones_below else 1
        macs[f"conv_fwd:{st.name}"] = B * h * w * st.cout * st.cin * 9 * st.ng_fwd
        tag = f"first_layer_bwd:{st.name}" if (li == 0 and st.w2_first is not None) else f"conv_bwd:{st.name}"
        macs[tag] = B * nq * h * w * st.cout * st.cin * 9 * st.ng_bwd
    for ds in eng.dense:
        N, Kd = ds.W.shape
        macs[f"linear_fwd:{ds.name}"] = B * N * Kd
        macs[f"linear_bwd:{ds.name}"] = B * N * Kd
    if launched is not None:
        launched = set(launched)
        macs = {k: v for k, v in macs.items() if k in launched}
    return macs


def whole_path_macs(macs, per, steps):
    """MACs of one traced step: each launched tag's per-launch MACs x its launches per step
    (`per`: tag -> list of event times over `steps` traced steps, as collected below)."""
    return sum(macs.get(tag, 0) * len(ts) for tag, ts in per.items()) / steps


# --------------------------------------------------------------------------- CPU baseline
def _cpu_model_name():
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return cpu


def _cgroup_cpus():
    """CPUs this process may actually use under a cgroup v2/v1 quota (None: no quota)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                return max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fq, open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fp:
            q, per = int(fq.read()), int(fp.read())
            if q > 0:
                return max(1, -(-q // per))
    except (OSError, ValueError):
        pass
    return None


def _cpu_threads():
    """torch.set_num_threads(len(os.sched_getaffinity(0))) -- capped at the cgroup CPU
    quota when one is set (the affinity mask can list the whole machine while the process is
    granted a share of it; threads beyond the share only contend).  Returns (threads, affinity,
    quota)."""
    aff = len(os.sched_getaffinity(0))
    quota = _cgroup_cpus()
    n = min(aff, quota) if quota else aff
    torch.set_num_threads(n)
    return n, aff, quota


def _median_timed(fn, warmup=2, reps=5):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


def cpu_baseline(chunk=8, reps=5):
    """The reference's CPU path, restated op for op (oracle zennit-structured mode: 5-pass Gamma +
    autograd like zennit.BasicHook, K+1 batch replication like explainer.py:92), timed per SURVEY
    8(d): all affinity cores, 2 warm-ups, median of >= 5 timed chunks of `chunk` samples."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import lrp_ref
    from drsa_audio_amd.model.modify_model import ProjectionModel
    threads, aff, quota = _cpu_threads()
    log(f"[bench] CPU baseline (LRP+DRSA explained samples): {threads} threads (affinity {aff}, cgroup quota {quota})")
    nm = {"features.0": ("wsquare", 1e-7), "features.3": ("gamma", 0.4, 1e-7), "features.6": ("gamma", 0.4, 1e-7),
          "features.9": ("gamma", 0.2, 1e-7), "features.12": ("gamma", 0.1, 1e-7),
          "classifier.0": ("epsilon", 1e-7), "classifier.3": ("epsilon", 1e-7), "classifier.6": ("epsilon", 1e-7)}
    pm = ProjectionModel(gtzan128(), 7, load_u(), 4).eval()
    x = synthetic_logmel(chunk, seed=100)
    med, ts = _median_timed(lambda: lrp_ref.subspace_heatmaps(pm, nm, 4, x, class_idx=3, mode="zennit"), 2, reps)
    return {"value": chunk / med, "unit": "explained samples/s", "cores": threads, "kind": "port",
            "sample": f"median of {reps} timed chunks ({', '.join(f'{t:.2f}' for t in ts)} s) after 2 warm-ups; "
                      f"chunk = {chunk} samples x (K+1=5 replicated rows), GTZAN-128 j=7 K=4, oracle "
                      f"zennit-structured mode, torch {torch.__version__} CPU, {threads} threads "
                      f"(len(sched_getaffinity) = {aff}, cgroup CPU quota = {quota}), {_cpu_model_name()}"}


def cpu_drsa_baseline(reps=7):
    """DRSA CPU leg at C3: oracle/drsa_ref.step (op for op drsa.py:84-106: fp32 obj + autograd, fp64
    eigh orthogonalize; pinned bit-exact to the reference's own fixtures), median of `reps` steps."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import drsa_ref
    from drsa_audio_amd.utils.synthetic import drsa_inputs
    threads, aff, quota = _cpu_threads()
    log(f"[bench] CPU baseline (DRSA C3 step): {threads} threads")
    A, C = (torch.from_numpy(v) for v in drsa_inputs(20000, 64, 3))
    U = torch.from_numpy(np.load(os.path.join(ROOT, "tests", "golden", "u64_seed42.npy")))
    med, _ = _median_timed(lambda: drsa_ref.step(A, C, U, 4), 2, reps)
    return {"config": "C3: N=20000, d=64, K=4", "ms_per_step": med * 1e3, "vector_steps_per_s": 20000 / med,
            "cores": threads, "kind": "port", "sample": f"median of {reps} steps after 2 warm-ups"}


# --------------------------------------------------------------------------- DRSA
def graph_replays(fn, device, steps, reps=7):
    """Steady-state timing of a whole fixed-step DRSA run (median of >= 20 steady-state
    steps): `fn` (one run of `steps` steps) runs once eagerly (library, side-stream
    pool, workspaces warm), is captured ONCE into a CUDA graph on a side stream (the C ABI records its
    plain sequence inside a caller's capture), and the graph is replayed `reps` times, each replay
    timed with HIP events on that stream.  Returns (per-step ms: median, min, max; fn's outputs as
    left by the last replay)."""
    s = torch.cuda.Stream(device)
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize(device)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out = fn()
    ts = []
    with torch.cuda.stream(s):
        g.replay()
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            g.replay()
            e1.record(s)
            torch.cuda.synchronize(device)
            ts.append(e0.elapsed_time(e1) / steps)
    return float(np.median(ts)), float(min(ts)), float(max(ts)), out


def _spread(med, lo, hi, reps=7):
    return {"median": med, "min": lo, "max": hi, "replays": reps}


def drsa_bench(device, steps=200):
    from drsa_audio_amd.utils.synthetic import drsa_inputs
    from drsa_audio_amd import _capi
    from drsa_audio_amd.xai.drsa.drsa import DrsaWorkspace, drsa_run
    N, d, K = 20000, 64, 4
    A, C = drsa_inputs(N, d, 3)
    U0 = np.load(os.path.join(ROOT, "tests", "golden", "u64_seed42.npy"))
    Ag, Cg, Ug = (torch.from_numpy(v).to(device) for v in (A, C, U0))
    ws = DrsaWorkspace(N, d, K, device)
    med, lo, hi, (U, traj) = graph_replays(lambda: drsa_run(Ag, Cg, Ug, K, steps, ws), device, steps)
    dt = med * 1e-3 * steps
    s = torch.cuda.Stream(device)
    with torch.cuda.stream(s):
        # the reference's 2000-step C3 run (tests/golden/drsa_long_fixture.npz): max deviation
        fx = np.load(os.path.join(ROOT, "tests", "golden", "drsa_long_fixture.npz"))
        _, t2000 = drsa_run(Ag, Cg, Ug, K, 2000, ws)
        torch.cuda.synchronize(device)
        ref = fx["c3_traj"]
        dev2000 = float(np.max(np.abs(t2000.cpu().numpy().astype(np.float64) - ref) / np.abs(ref)))
        # per-kernel HIP-event timings on this stream: partial (+ slab reduce) and finish (polar)
        st = s.cuda_stream
        Un = torch.empty_like(Ug)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tp, tf = [], []
        for _ in range(50):
            ev[0].record(s)
            _capi.call("drsa_amd_drsa_partial", Ag.data_ptr(), Cg.data_ptr(), N, d, K, Ug.data_ptr(), ws.gs.data_ptr(),
                       ws.ptr, ws.nbytes, st)
            ev[1].record(s)
            _capi.call("drsa_amd_drsa_finish", ws.gs.data_ptr(), N, d, K, Ug.data_ptr(), Un.data_ptr(),
                       ws.f.data_ptr(), 0, None, st)
            ev[2].record(s)
            torch.cuda.synchronize(device)
            tp.append(ev[0].elapsed_time(ev[1]))
            tf.append(ev[1].elapsed_time(ev[2]))
    traj = traj.cpu().numpy()
    flop = 8.0 * N * d * d
    ms = dt / steps * 1e3
    tflops = flop / (ms * 1e-3) / 1e12
    tp_ms = float(np.median(tp))
    return {"config": f"C3: N=20000, d=64, K=4 (synthetic normalised A=|N(0,1)|, C~N(0,1)), a {steps}-step run "
                      "captured once as a graph, replayed 7 times (HIP events); ms_per_step = median replay / steps",
            "ms_per_step": ms, "ms_per_step_spread": _spread(med, lo, hi), "vector_steps_per_s": N * steps / dt,
            "steps": steps, "objective_final": float(traj[-1]),
            "traj_dev_2000_vs_reference": dev2000,
            "roofline": {"bound": "mfma", "kernel": "drsa_partial (+ slab reduce)",
                         "achieved": flop / (tp_ms * 1e-3) / 1e12, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": flop / (tp_ms * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS,
                         "whole_step_tflops": tflops, "whole_step_frac": tflops / FP32_MFMA_PEAK_TFLOPS,
                         "algorithmic_flop_per_step": flop},
            "event_ms": {"partial_plus_reduce": tp_ms, "finish_polar": float(np.median(tf))}}


def frontend_bench(device, n_songs=64, iters=20):
    """R17 log-mel front end: n_songs synthetic 29.5 s songs x 8 chunks -> [512, 1, 128, 128] in one
    launch (get_slice + peak_normalizer + STFT + mel + log10 + clamp).  HBM roofline: the chunk's
    48 000 samples read once + the 128x128 log-mel written once = 257 KB per chunk."""
    from drsa_audio_amd.utils.dataloading import Loader
    from drsa_audio_amd.utils.synthetic import synthetic_songs
    songs = torch.from_numpy(synthetic_songs(n_songs, seed=3)).to(device)
    ld = Loader("gtzan", device=device)
    s = torch.cuda.current_stream(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        ld.load_songs(songs)
    e0.record(s)
    for _ in range(iters):
        ld.load_songs(songs)
    e1.record(s)
    torch.cuda.synchronize(device)
    ms = e0.elapsed_time(e1) / iters
    chunks = n_songs * 8
    byts = chunks * 4.0 * (48000 + 128 * 128)
    gbs = byts / (ms * 1e-3) / 1e9
    return {"config": f"GTZAN front end: {n_songs} songs x 8 chunks of 3 s @16 kHz -> 128x128 log-mel",
            "chunks_per_s": chunks / (ms * 1e-3), "ms_per_launch": ms, "algorithmic_bytes_per_launch": byts,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS},
            "parity": "tests/test_logmel_gpu.py (f64-anchored gates); not re-checked here"}


def drsa_joint_bench(device, steps=200):
    """C5 DRSA: layers j=26 and j=33 of VGGish (d=128, K=16 each, 20000 rows each) optimised
    together in one hipGraph (drsa_amd_drsa_run_multi)."""
    from drsa_audio_amd.utils.synthetic import drsa_inputs
    from drsa_audio_amd.xai.drsa.drsa import drsa_run, drsa_run_joint
    N, d, K = 20000, 128, 16
    probs = []
    for seed in (26, 33):
        A, C = drsa_inputs(N, d, seed)
        U0 = np.linalg.qr(np.random.default_rng(seed).standard_normal((d, d)))[0].astype(np.float32)
        probs.append(tuple(torch.from_numpy(v).to(device) for v in (A, C, U0)) + (K,))
    # every leg: one fixed-step run captured once, replayed 7 times (graph_replays)
    j = graph_replays(lambda: drsa_run_joint(probs, steps), device, steps)
    out = j[3]
    sq = graph_replays(lambda: [drsa_run(A, C, U0, K_, steps) for A, C, U0, K_ in probs], device, steps)
    # bf16 inputs + bf16 MFMA projection (C5; fp32 accumulate)
    probs16 = [(A.to(torch.bfloat16), C.to(torch.bfloat16), U0, K_) for A, C, U0, K_ in probs]
    b = graph_replays(lambda: drsa_run_joint(probs16, steps), device, steps)
    out16 = b[3]
    # fp16 inputs + fp16 MFMA projection (C5 "fp16 MFMA projection")
    probsh = [(A.to(torch.float16), C.to(torch.float16), U0, K_) for A, C, U0, K_ in probs]
    h = graph_replays(lambda: drsa_run_joint(probsh, steps), device, steps)
    outh = h[3]
    dt, dt_seq, dt16, dth = (x[0] * 1e-3 * steps for x in (j, sq, b, h))
    flop = 2 * 8.0 * N * d * d
    rel16 = max(abs(float(a[1][-1]) - float(b[1][-1])) / abs(float(b[1][-1])) for a, b in zip(out16, out))
    relh = max(abs(float(a[1][-1]) - float(b[1][-1])) / abs(float(b[1][-1])) for a, b in zip(outh, out))
    return {"config": f"C5 joint: 2 problems (VGGish j=26, j=33) x N=20000, d=128, K=16; each leg a {steps}-step "
                      "run captured once as a graph and replayed 7 times (HIP events), median / min / max per step",
            "ms_per_joint_step": dt / steps * 1e3, "ms_per_joint_step_spread": _spread(*j[:3]),
            "ms_per_step_sequential_runs": dt_seq / steps * 1e3, "sequential_spread": _spread(*sq[:3]),
            "bf16": {"ms_per_joint_step": dt16 / steps * 1e3, "spread": _spread(*b[:3]),
                     "objective_rel_diff_vs_fp32_after_steps": rel16, "tolerance": 1e-2},
            "fp16": {"ms_per_joint_step": dth / steps * 1e3, "spread": _spread(*h[:3]),
                     "objective_rel_diff_vs_fp32_after_steps": relh, "tolerance": 1e-2},
            "vector_steps_per_s": 2 * N * steps / dt, "tflops_algorithmic": flop * steps / dt / 1e12,
            "objective_final": [float(t[-1]) for _, t in out]}


def vggish_lrp_bench(device, B=32, iters=10):
    """C5 model: VGGish-BN, 128x256 log-mel.  Standard LRP (compute_relevances), the engine forward
    alone, and the C5 CNN leg (DRSA data capture at j = 26: forward + relevance backward to the
    layer), each on the fp32 plan, on the bf16 plan (model.bfloat16(): conv forwards on
    v_mfma_f32_32x32x16_bf16, relevance backward fp32; parity tests/test_bf16_gpu.py) and on the
    bf16 plan with the bf16 relevance backward (tests/test_bf16_bwd_gpu.py), with a roofline line
    for each standard-LRP pass's dominant kernel."""
    import copy
    from drsa_audio_amd.engine import get_engine
    from drsa_audio_amd.model.create_model import VGGType
    from drsa_audio_amd.utils.constants import LRP_NAME_MAP_VGGISH
    from drsa_audio_amd.zennit.canonizers import SequentialMergeBatchNorm
    from drsa_audio_amd.zennit.composites import NameMapComposite
    from drsa_audio_amd.xai.explain.attribute import compute_relevances
    from drsa_audio_amd.xai.drsa.preprocessing import get_intermediate
    torch.manual_seed(0)
    m32 = VGGType(n_filters=(64, 64, 100, 128, 128), n_dense=100, pool_kernels=((2, 4),) + ((2, 2),) * 4, dropout=0.3,
                  input_size=(128, 256), conv_bn=True, dense_bn=True).eval().to(device)
    comp = NameMapComposite(LRP_NAME_MAP_VGGISH, canonizers=[SequentialMergeBatchNorm()])
    x32 = synthetic_logmel(B, 128, 256, seed=5, device=device)

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize(device)
        return B * iters / (time.perf_counter() - t0)

    out = {"config": f"VGGish-BN (64,64,100,128,128), block_depth 2, 128x256, B={B}; samples/s",
           "legs": "fp32 plan; bf16 plan (bf16 conv forwards, fp32 relevance backward); bf16_bwd (bf16 plan "
                   "with the bf16 relevance backward, DRSA_AMD_BF16_BACKWARD=1)"}
    prev = os.environ.get("DRSA_AMD_BF16_BACKWARD")
    try:
        for prec, m, x in (("fp32", m32, x32), ("bf16", copy.deepcopy(m32).bfloat16(), x32.bfloat16()),
                           ("bf16_bwd", copy.deepcopy(m32).bfloat16(), x32.bfloat16())):
            os.environ["DRSA_AMD_BF16_BACKWARD"] = "1" if prec == "bf16_bwd" else "0"
            eng = get_engine(m, comp)
            out[prec] = {"standard_lrp": timed(lambda: compute_relevances(m, x, comp, class_idx=1)),
                         "forward": timed(lambda: eng.forward(x)),
                         "capture_j26": timed(lambda: get_intermediate(m, x, comp, 26, 1))}
            # roofline of the standard-LRP pass's dominant kernel (HIP events on the launch stream)
            eng.trace = []
            for _ in range(3):
                compute_relevances(m, x, comp, class_idx=1)
            torch.cuda.synchronize(device)
            per = {}
            for tag, e0, e1 in eng.trace:
                per.setdefault(tag, []).append(e0.elapsed_time(e1))
            eng.trace = None
            macs = kernel_macs(eng, B, 0, launched=per)
            top = max(per, key=lambda k: float(np.mean(per[k])))
            # the roofline line: the slowest MFMA conv kernel (the top kernel can be the VALU
            # first-layer backward, reported beside it)
            dom = max((k for k in per if k.startswith(("conv_fwd:", "conv_bwd:"))), key=lambda k: float(np.mean(per[k])))
            avg = float(np.mean(per[dom]))
            st = next((s_ for s_ in eng.stages if dom.endswith(":" + s_.name)), None)
            on_bf16 = st is not None and st.cin > 1 and (
                (dom.startswith("conv_fwd") and eng.bf16) or (dom.startswith("conv_bwd") and st.wts_bwd_bf is not None))
            peak = BF16_MFMA_PEAK_TFLOPS if on_bf16 else FP32_MFMA_PEAK_TFLOPS
            ach = 2.0 * macs.get(dom, 0) / (avg * 1e-3) / 1e12
            out[prec]["roofline"] = {"bound": "mfma", "kernel": dom, "operands": "bf16" if on_bf16 else "fp32",
                                     "avg_ms": avg, "achieved": ach, "peak": peak, "unit": "TFLOP/s", "frac": ach / peak}
            out[prec]["top_kernel"] = {"tag": top, "avg_ms": float(np.mean(per[top]))}
            out[prec]["kernels_ms"] = {k: float(np.mean(v)) for k, v in per.items()}
    finally:
        if prev is None:
            os.environ.pop("DRSA_AMD_BF16_BACKWARD", None)
        else:
            os.environ["DRSA_AMD_BF16_BACKWARD"] = prev
    out["samples_per_s"] = out["fp32"]["standard_lrp"]
    return out


def drsa_sharded_bench(device, world, rank, steps=100):
    """C4 row-sharded DRSA: 20000 rows per rank (weak; 160000 at 8 ranks), d=64, K=8; one RCCL
    all-reduce of the [d*d+K] partial per step (drsa_audio_amd/xai/drsa/distributed.py)."""
    import torch.distributed as dist
    from drsa_audio_amd.utils.synthetic import drsa_inputs
    from drsa_audio_amd.xai.drsa.distributed import sharded_run
    n, d, K = 20000, 64, 8
    A, C = drsa_inputs(n, d, 100 + rank)
    U0 = np.load(os.path.join(ROOT, "tests", "golden", "u64_seed42.npy"))
    Ag, Cg, Ug = (torch.from_numpy(v).to(device) for v in (A, C, U0))
    sharded_run(Ag, Cg, Ug, K, 3)
    torch.cuda.synchronize(device)
    dist.barrier()
    t0 = time.perf_counter()
    U, traj = sharded_run(Ag, Cg, Ug, K, steps)
    torch.cuda.synchronize(device)
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t)
    out = {"config": f"row-sharded DRSA: {n} rows/rank x {world} ranks, d={d}, K={K}, all-reduce {d*d+K} fp32/step",
           "ms_per_step": dt / steps * 1e3, "vector_steps_per_s": n * world * steps / dt, "steps": steps,
           "objective_final": float(traj[-1])}
    if rank == 0:
        # self-check (outside the timed region): every rank's seeded rows regenerated here, the
        # unsharded single-process run on their concatenation, max relative trajectory deviation
        from drsa_audio_amd.xai.drsa.drsa import drsa_run
        Aa, Ca = (torch.from_numpy(np.concatenate(v)).to(device)
                  for v in zip(*(drsa_inputs(n, d, 100 + r) for r in range(world))))
        _, tr1 = drsa_run(Aa, Ca, Ug, K, steps)
        tr1 = tr1.cpu().numpy().astype(np.float64)
        out["traj_dev_vs_unsharded"] = float(np.max(np.abs(np.asarray(traj, np.float64) - tr1) / np.abs(tr1)))
        del Aa, Ca
    dist.barrier()
    # C5 on N GPUs: the two VGGish layers (j = 26, 33; d = 128, K = 16) row-sharded, one packed
    # all-reduce of both partials per step (distributed.py::sharded_run_joint)
    from drsa_audio_amd.xai.drsa.distributed import sharded_run_joint
    d5, K5, s5 = 128, 16, 50
    g = torch.Generator().manual_seed(5)
    probs = []
    for p_ in range(2):
        A5, C5 = drsa_inputs(n, d5, 200 + 10 * rank + p_)
        U5 = torch.linalg.qr(torch.randn(d5, d5, generator=g, dtype=torch.float64))[0].float().contiguous()
        probs.append((torch.from_numpy(A5).to(device), torch.from_numpy(C5).to(device), U5.to(device), K5))
    sharded_run_joint(probs, 3)
    torch.cuda.synchronize(device)
    dist.barrier()
    t0 = time.perf_counter()
    res = sharded_run_joint(probs, s5)
    torch.cuda.synchronize(device)
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt5 = float(t)
    out["c5_joint"] = {"config": f"C5 joint, row-sharded: 2 problems x {n} rows/rank x {world} ranks, d={d5}, "
                                 f"K={K5}, one all-reduce of 2 x {d5 * d5 + K5} fp32/step",
                       "ms_per_joint_step": dt5 / s5 * 1e3, "steps": s5,
                       "objective_final": [float(tr[-1]) for _, tr in res]}
    if rank == 0:
        from drsa_audio_amd.xai.drsa.drsa import drsa_run
        devs = []
        for p_ in range(2):
            Aa, Ca = (torch.from_numpy(np.concatenate(v)).to(device)
                      for v in zip(*(drsa_inputs(n, d5, 200 + 10 * r + p_) for r in range(world))))
            _, tr1 = drsa_run(Aa, Ca, probs[p_][2], K5, s5)
            tr1 = tr1.cpu().numpy().astype(np.float64)
            devs.append(float(np.max(np.abs(np.asarray(res[p_][1], np.float64) - tr1) / np.abs(tr1))))
            del Aa, Ca
        out["c5_joint"]["traj_dev_vs_unsharded"] = max(devs)
    dist.barrier()
    return out


def drsa_pipeline_bench(device, world, rank, model, samples_per_rank=1000, steps=100, num_locations=20, K=8):
    """C4's rank-local chain (the reference: getdrsadata.py:119-137 preprocess_data
    -> :47-59 load_and_normalize_data -> drsa.main): every rank extracts DRSA rows from ITS slice of a
    seeded synthetic log-mel batch (drsa_training_data(group=): forward + LRP backward to j = 7, the
    locations drawn from the global numpy stream, normalisation over all ranks' rows), then
    main_sharded(local_rows=True) optimises K = 8 subspaces over the row shards (one all-reduce per
    step).  No rank holds the whole set.  Weak scaling: samples_per_rank x num_locations rows per rank
    (1000 x 20 = 20 000; 160 000 = C4's N at 8 ranks).  Rank 0 then rebuilds the whole batch, runs
    the single-process chain (drsa_training_data + drsa_run) and reports the trajectory deviation."""
    import tempfile
    import pandas as pd
    import torch.distributed as dist
    from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN
    from drsa_audio_amd.zennit.composites import NameMapComposite
    from drsa_audio_amd.xai.drsa.preprocessing import drsa_training_data
    from drsa_audio_amd.xai.drsa.distributed import main_sharded
    comp = NameMapComposite(LRP_NAME_MAP_GTZAN)
    group = dist.group.WORLD if world > 1 else None
    x = synthetic_logmel(samples_per_rank, seed=300 + rank, device=device)

    def barrier():
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()

    def max_over_ranks(v):
        if world == 1:
            return v
        t = torch.tensor([v], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t)

    np.random.seed(7)
    drsa_training_data(model, x[:8], comp, 7, 3, num_locations=num_locations, group=group)   # plan build / warm-up
    barrier()
    np.random.seed(7)
    t0 = time.perf_counter()
    A, C = drsa_training_data(model, x, comp, 7, 3, num_locations=num_locations, group=group)
    barrier()
    t_ext = max_over_ranks(time.perf_counter() - t0)
    with tempfile.TemporaryDirectory() as root:
        main_sharded(A, C, root, num_concepts=K, steps=3, runs=1, local_rows=True, group=group)   # warm-up
        barrier()
        t0 = time.perf_counter()
        main_sharded(A, C, root, num_concepts=K, steps=steps, runs=1, local_rows=True, group=group)
        barrier()
        t_opt = max_over_ranks(time.perf_counter() - t0)
        traj = None
        if rank == 0:
            traj = pd.read_csv(os.path.join(root, "run1", "train_stats.csv"))["loss"].to_numpy(np.float64)
    rows = A.size(0) * world
    out = {"config": f"rank-local C4 chain: {samples_per_rank} samples/rank x {world} rank(s), j=7 (d=64), "
                     f"{num_locations} locations/sample, K={K}: drsa_training_data(group=) -> "
                     f"main_sharded(local_rows=True), {steps} steps, 1 run",
           "scaling": "weak", "rows_total": rows,
           "extraction_rows_per_s": rows / t_ext, "extraction_s": t_ext,
           "optimisation_steps_per_s": steps / t_opt, "optimisation_vector_steps_per_s": rows * steps / t_opt}
    del A, C
    if rank == 0:
        from drsa_audio_amd.xai.drsa.drsa import drsa_run, initial_projections
        xa = torch.cat([synthetic_logmel(samples_per_rank, seed=300 + r, device=device) for r in range(world)])
        np.random.seed(7)
        A1, C1 = drsa_training_data(model, xa, comp, 7, 3, num_locations=num_locations)
        del xa
        U0 = torch.tensor(np.ascontiguousarray(initial_projections(A1.size(1), 1, 42)[0]), dtype=torch.float32,
                          device=device)
        _, t1 = drsa_run(A1, C1, U0, K, steps)
        t1 = t1.cpu().numpy().astype(np.float64)
        out["traj_dev_vs_unsharded"] = float(np.max(np.abs(traj - t1) / np.abs(t1)))
        del A1, C1
    if world > 1:
        dist.barrier()
    return out


def drsa_grid_bench(device, world, rank, steps=100, N=20000, classes=None):
    """Task-parallel DRSA over the reference's problem grid (optsubspaces.py:17-23): 10 classes x
    layers [19 (d=100), 26 (d=128), 33 (d=128)] x 3 runs = 90 independent problems, K=4, N rows
    each (synthetic normalised A=|N(0,1)|, C~N(0,1)); LPT-assigned over the ranks, each rank's
    problems batched (drsa_run_batched: one partial / reduce / finish launch per step for all of
    them, graph-replayed).  Strong scaling: the grid is fixed.
    The reference runs 5000 steps per problem; this leg times `steps` and projects."""
    import torch.distributed as dist
    from drsa_audio_amd.xai.drsa.cluster.optsubspaces import GTZAN_CLASSES, GTZAN_LAYERS, optimize_grid
    from drsa_audio_amd.xai.drsa.preprocessing import normalize_vectors
    classes = classes or GTZAN_CLASSES
    dims = {19: 100, 26: 128, 33: 128}
    g = torch.Generator(device=device).manual_seed(1234)
    data = {}
    for c in classes:
        for l in GTZAN_LAYERS:
            A = torch.randn(N, dims[l], device=device, generator=g).abs_()
            C = torch.randn(N, dims[l], device=device, generator=g)
            data[(c, l)] = (normalize_vectors(A, out=A), normalize_vectors(C, out=C))
    optimize_grid(data, None, num_concepts=4, steps=2, device=device)        # graph instantiate / warm-up
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    res = optimize_grid(data, None, num_concepts=4, steps=steps, device=device)
    torch.cuda.synchronize(device)
    dt_rank = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    dts = [dt_rank]
    if world > 1:
        t = torch.zeros(world, device=device, dtype=torch.float64)
        t[rank] = dt_rank
        dist.all_reduce(t)
        dts = t.tolist()
    dt = max(dts)
    P = len(res)
    per_rank = {}
    for k, v in res.items():
        per_rank[v["rank"]] = per_rank.get(v["rank"], 0) + 1
    return {"config": f"task-parallel DRSA grid: {len(classes)} classes x layers {list(GTZAN_LAYERS)} (d=100/128/128) "
                      f"x 3 runs = {P} problems, K=4, N={N} each, {world} rank(s), LPT assignment, "
                      "each rank's problems batched: one launch per phase for all (drsa_run_batched)",
            "scaling": "strong", "steps": steps, "problems": P, "problems_per_rank": [per_rank.get(r, 0) for r in range(world)],
            "problem_steps_per_s": P * steps / dt, "vector_steps_per_s": P * N * steps / dt,
            "rank_seconds": dts,
            "projected_full_grid_s": P * 5000 / (P * steps / dt),
            "objective_final_min_max": [min(v["objective"] for v in res.values()),
                                        max(v["objective"] for v in res.values())]}


# --------------------------------------------------------------------------- main
LEGS = ("c2", "drsa", "frontend", "joint", "vggish", "sharded", "pipeline", "grid", "to_host", "clone")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=512, help="explained samples per GPU per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-drsa", action="store_true")
    ap.add_argument("--tag-order", default=None,
                    help="write the per-step kernel tag order (JSON) for scripts/tag_profile.py")
    ap.add_argument("--grid-steps", type=int, default=100, help="steps of the task-parallel DRSA grid leg")
    ap.add_argument("--grid-classes", type=int, default=10, help="classes of the DRSA grid (10 = the reference's)")
    ap.add_argument("--pipeline-samples", type=int, default=1000, help="samples per rank of the rank-local C4 leg")
    ap.add_argument("--pipeline-steps", type=int, default=100, help="DRSA steps of the rank-local C4 leg")
    ap.add_argument("--legs", default="all",
                    help="secondary legs to run: all, none, or a comma list of " + ",".join(LEGS))
    args = ap.parse_args()
    legs = set(LEGS) if args.legs == "all" else set() if args.legs == "none" else set(args.legs.split(","))
    if not legs <= set(LEGS):
        ap.error(f"--legs: unknown {sorted(legs - set(LEGS))}")
    if args.no_drsa:
        legs -= {"drsa", "joint", "vggish", "sharded", "pipeline", "grid"}

    # rehearsal of the N > 1 path on a one-GPU box (tests only): every rank on cuda:0, usually gloo
    one_dev = os.environ.get("DRSA_BENCH_ONE_DEVICE") == "1"
    backend = os.environ.get("DRSA_BENCH_BACKEND", "nccl")   # nccl = RCCL on ROCm
    from drsa_audio_amd.utils.launch import init_distributed, maybe_launch
    # --gpus N without torchrun: fan out into N ranks here, before anything touches the GPU
    maybe_launch(args.gpus, one_device=one_dev)
    world, rank, device = init_distributed(backend, one_dev)
    if world > 1:
        import torch.distributed as dist
        if world != args.gpus:
            log(f"[bench] note: WORLD_SIZE={world} but --gpus {args.gpus}; measuring {world} ranks")

    from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN
    from drsa_audio_amd.xai.explain.explainer import HeatmapGenerator
    from drsa_audio_amd.engine import get_engine

    B, K = args.batch, 4
    model = gtzan128().to(device)
    # headline: the standard heatmap as the sum of the K concept heatmaps (exact reformulation, every
    # rule is linear in R; gated bit-exact vs the oracle in both modes); the reference's clone-0
    # form (HeatmapGenerator's default) is timed beside it in secondary.clone_mode
    hg = HeatmapGenerator(model, load_u(), LRP_NAME_MAP_GTZAN, "blues", num_concepts=K, layer_idx=7, device=device,
                          standard="sum")
    x = synthetic_logmel(B, seed=1 + rank, device=device)

    props = torch.cuda.get_device_properties(device)
    dev_info = {"name": props.name, "cus": props.multi_processor_count,
                "gcn_arch": getattr(props, "gcnArchName", ""), "clock_khz": getattr(props, "clock_rate", None)}
    log(f"[bench] device {dev_info}")
    log(f"[bench] rank {rank}/{world}: headline B={B}, {args.warmup} warm-up + {args.steps} timed steps")
    for _ in range(args.warmup):
        hg.generate_subspace_heatmaps(x, to_host=False)
    torch.cuda.synchronize(device)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hg.generate_subspace_heatmaps(x, to_host=False)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    rank_ms = [dt / args.steps * 1e3]
    if world > 1:
        t = torch.zeros(world, device=device, dtype=torch.float64)
        t[rank] = dt
        dist.all_reduce(t)                          # every rank's time; the job's time is the max
        rank_ms = [v / args.steps * 1e3 for v in t.tolist()]
        dt = max(t.tolist())
    ms = dt / args.steps * 1e3
    value = world * B * args.steps / dt

    # ---- per-kernel timing (HIP events on the launch stream), separate traced steps ----
    eng = get_engine(hg.projectionmodel, hg.composite)
    eng.trace = []
    for _ in range(3):
        hg.generate_subspace_heatmaps(x, to_host=False)
    torch.cuda.synchronize(device)
    per = {}
    for tag, e0, e1 in eng.trace:
        per.setdefault(tag, []).append(e0.elapsed_time(e1))
    tags = [t for t, _, _ in eng.trace]
    eng.trace = None
    if args.tag_order and rank == 0:
        L = len(tags) // 3
        with open(args.tag_order, "w") as fh:
            json.dump({"tags": tags[:L], "main_steps": args.warmup + args.steps + 3, "batch": B}, fh)
    macs = kernel_macs(eng, B, K, hg.standard, launched=per)
    kernels = {}
    for tag, ts in per.items():
        avg = float(np.mean(ts))
        m = macs.get(tag)
        kernels[tag] = {"avg_ms": avg, "launches": len(ts)}
        if m:
            kernels[tag]["tflops"] = 2.0 * m / (avg * 1e-3) / 1e12
    dom = max(kernels, key=lambda k: kernels[k]["avg_ms"])
    dom_ach = kernels[dom].get("tflops", 0.0)
    traffic = traffic_src = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as fh:
                pm = json.load(fh)
            traffic = pm.get("per_launch_bytes", {}).get(dom)
            # (no clock figure: GRBM_GUI_ACTIVE / 8 over a PMC-serialised dispatch read 2.4-6.7 GHz,
            # above the 2.4 GHz behind the peak, so it is not physical)
            # PMC counters cannot be read inside this process: the bytes come from the committed
            # rocprofv3 --pmc passes (scripts/pmc_run.sh) of the same kernel, named here
            traffic_src = f"profiles/pmc_traffic.json ({pm.get('profile', 'unlabelled')}), not measured in this run"
        except Exception:
            traffic = None
    total_macs = whole_path_macs(macs, per, 3)

    log(f"[bench] headline {value:.0f} explained samples/s ({ms:.3f} ms/step); secondaries next")
    # ---- secondary: standard LRP (C2, bs=64) ----
    c2 = bs64 = None
    if "c2" in legs:
        from drsa_audio_amd.zennit.composites import NameMapComposite
        from drsa_audio_amd.xai.explain.attribute import compute_relevances
        comp = NameMapComposite(LRP_NAME_MAP_GTZAN)
        x64 = synthetic_logmel(64, seed=7 + rank, device=device)
        for _ in range(3):
            compute_relevances(model, x64, comp, class_idx=3)
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        for _ in range(10):
            compute_relevances(model, x64, comp, class_idx=3)
        torch.cuda.synchronize(device)
        c2 = 64 * 10 / (time.perf_counter() - t1)
        # bs=64 explained samples (same path, C2 batch size)
        x64b = x64
        for _ in range(3):
            hg.generate_subspace_heatmaps(x64b, to_host=False)
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        for _ in range(10):
            hg.generate_subspace_heatmaps(x64b, to_host=False)
        torch.cuda.synchronize(device)
        bs64 = 64 * 10 / (time.perf_counter() - t1)
    drsa = None
    if "drsa" in legs and rank == 0:
        log("[bench] DRSA C3")
        drsa = drsa_bench(device)
    log("[bench] log-mel front end, DRSA C5 joint, VGGish")
    frontend = frontend_bench(device) if (rank == 0 and "frontend" in legs) else None
    joint = drsa_joint_bench(device) if (rank == 0 and "joint" in legs) else None
    vgg = vggish_lrp_bench(device) if (rank == 0 and "vggish" in legs) else None
    drsa_sharded = grid = pipeline = None
    if "sharded" in legs and world > 1:
        drsa_sharded = drsa_sharded_bench(device, world, rank)
    if "pipeline" in legs:
        log("[bench] rank-local DRSA pipeline (C4 chain)")
        pipeline = drsa_pipeline_bench(device, world, rank, model, samples_per_rank=args.pipeline_samples,
                                       steps=args.pipeline_steps)
    if "grid" in legs:
        log("[bench] task-parallel DRSA grid")
        from drsa_audio_amd.xai.drsa.cluster.optsubspaces import GTZAN_CLASSES
        grid = drsa_grid_bench(device, world, rank, steps=args.grid_steps,
                               classes=GTZAN_CLASSES[:max(1, args.grid_classes)])
    # the reference's clone-0 standard heatmap (K+1 clones below the projection, explainer.py:92)
    clone_mode = None
    if rank == 0 and "clone" in legs:
        log("[bench] clone-mode rate")
        hgc = HeatmapGenerator(model, load_u(), LRP_NAME_MAP_GTZAN, "blues", num_concepts=K, layer_idx=7,
                               device=device, standard="clone")
        for _ in range(2):
            hgc.generate_subspace_heatmaps(x, to_host=False)
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        nc = 10
        for _ in range(nc):
            hgc.generate_subspace_heatmaps(x, to_host=False)
        torch.cuda.synchronize(device)
        tc = (time.perf_counter() - t1) / nc
        clone_mode = {"explained_samples_per_s": B / tc, "ms_per_step": tc * 1e3,
                      "note": "HeatmapGenerator(standard='clone') (the default): the standard heatmap is clone 0 "
                              "of K+1 relevance clones, as the reference's replicated batch (explainer.py:92)"}
        del hgc
    # the reference API returns numpy (explainer.py:111): the same steps with the D2H copy of info
    to_host = None
    if rank == 0 and "to_host" in legs:
        log("[bench] to_host rate")
        for _ in range(2):
            hg.generate_subspace_heatmaps(x, to_host=True)
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        nh = 5
        for _ in range(nh):
            hg.generate_subspace_heatmaps(x, to_host=True)
        torch.cuda.synchronize(device)
        th = (time.perf_counter() - t1) / nh
        to_host = {"explained_samples_per_s": B / th, "ms_per_step": th * 1e3,
                   "note": "generate_subspace_heatmaps(to_host=True): info dict as numpy (input + heatmaps + "
                           "relevances + mask copied D2H each step, PCIe-inclusive)"}
    if world > 1:
        # the other ranks leave before rank 0 times the CPU baseline, so nothing competes for the cores
        dist.barrier()
        dist.destroy_process_group()
        if rank != 0:
            return
    cpu = cpu_drsa = None
    if not args.no_cpu_baseline and rank == 0:
        cpu = cpu_baseline()
        cpu_drsa = cpu_drsa_baseline()

    if rank == 0:
        out = {
            "metric": "explained samples/sec (LRP+DRSA k=4)",
            "value": value,
            "unit": "explained samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "rank_ms_per_step": rank_ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (seeded log-mel-like 128x128 batches; random-init GTZAN-128 weights, "
                    "torch.manual_seed(0); U = ortho_group.rvs(64) seed 42)",
            "config": {"workload": "GTZAN-128 HeatmapGenerator: LRP (WSquare/Gamma/Epsilon name map) + DRSA "
                                   "subspace heatmaps, K=4 at layer j=7 (conv3 block, d=64), sorted info dict",
                       "standard_heatmap": "sum of the K concept heatmaps (standard='sum'; exact reformulation, "
                                           "bit-exact vs the oracle); the reference's clone-0 form: "
                                           "secondary.clone_mode; with the numpy info D2H: secondary.to_host",
                       "global_batch": B * world, "per_gpu_batch": B, "input": "128x128 log-mel",
                       "parallelism": f"data-parallel x{world} (no collective on the data path)",
                       "launch": ("torchrun" if os.environ.get("TORCHELASTIC_RUN_ID") else
                                  "bench.py --gpus (own launcher)" if world > 1 else "single process"),
                       "one_device_rehearsal": one_dev, "backend": backend if world > 1 else None},
            "roofline": {"bound": "mfma", "kernel": dom, "achieved": dom_ach, "peak": FP32_MFMA_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": dom_ach / FP32_MFMA_PEAK_TFLOPS, "traffic": traffic,
                         "traffic_source": traffic_src},
            "whole_path": {"algorithmic_gflop_per_sample": 2.0 * total_macs / B / 1e9,
                           "achieved_tflops": 2.0 * total_macs * value / B / world / 1e12},
            "kernels": kernels,
            "secondary": {"standard_lrp_c2_bs64_samples_per_s": c2 and c2 * world,
                          "explained_samples_per_s_bs64": bs64 and bs64 * world, "drsa": drsa,
                          "drsa_sharded": drsa_sharded, "drsa_rank_local_pipeline": pipeline,
                          "drsa_joint_c5": joint, "vggish_lrp": vgg,
                          "drsa_grid_task_parallel": grid, "logmel_frontend": frontend, "to_host": to_host,
                          "clone_mode": clone_mode,
                          "cpu_baseline_drsa_c3": cpu_drsa},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
