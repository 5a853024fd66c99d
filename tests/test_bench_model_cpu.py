"""bench.py's FLOP model: the whole-path figure counts the kernels one traced
step launched, and nothing else.  The engine is faked with the GTZAN-128 j=7 K=4 plan's stage
geometry; the launched tags are the ones profiles/r04_s4/bench.json recorded."""
import json
import os
import types

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stage(name, cin, cout, ng_fwd, ng_bwd, proj=False, w2=False):
    return types.SimpleNamespace(name=name, cin=cin, cout=cout, ng_fwd=ng_fwd, ng_bwd=ng_bwd,
                                 proj=object() if proj else None, w2_first=object() if w2 else None)


def _gtzan_engine():
    stages = [_stage("features.0", 1, 32, 1, 1, w2=True), _stage("features.3", 32, 32, 2, 1),
              _stage("features.6", 32, 64, 2, 1, proj=True), _stage("features.9", 64, 64, 3, 2),
              _stage("features.12", 64, 128, 2, 1)]
    hw = [128, 64, 32, 16, 8]
    dense = [types.SimpleNamespace(name=n, W=types.SimpleNamespace(shape=s))
             for n, s in (("classifier.0", (128, 2048)), ("classifier.3", (128, 128)), ("classifier.6", (10, 128)))]
    return types.SimpleNamespace(stages=stages, dense=dense, last={"stages": [{"H": h, "W": h} for h in hw]})


def _recorded_tags():
    with open(os.path.join(ROOT, "profiles", "r04_s4", "bench.json")) as fh:
        return list(json.load(fh)["kernels"])


def test_kernel_macs_launched_only():
    eng, tags = _gtzan_engine(), _recorded_tags()
    full = bench.kernel_macs(eng, 512, 4, "sum")
    macs = bench.kernel_macs(eng, 512, 4, "sum", launched=tags)
    assert set(macs) <= set(tags) and set(macs) <= set(full)
    # a tag the step did not launch contributes nothing
    fewer = bench.kernel_macs(eng, 512, 4, "sum", launched=[t for t in tags if t != "conv_bwd:features.3"])
    assert "conv_bwd:features.3" not in fewer and len(fewer) == len(macs) - 1
    per = {t: [0.0] * 3 for t in tags}                     # three traced steps, one launch each
    gflop = 2.0 * bench.whole_path_macs(macs, per, 3) / 512 / 1e9
    assert gflop == pytest.approx(0.884020224, rel=1e-9)   # DESIGN.md section 4 / VERDICT r04
    # the dominant kernel: 4 clones x 37.75 M MAC per clone per sample
    assert macs["conv_bwd:features.3"] == 512 * 4 * 64 * 64 * 32 * 32 * 9


def test_whole_path_counts_repeat_launches():
    eng = _gtzan_engine()
    macs = bench.kernel_macs(eng, 8, 4, "sum", launched=["conv_fwd:features.3", "heatmap_sort"])
    per = {"conv_fwd:features.3": [0.0] * 4, "heatmap_sort": [0.0] * 2}   # 2 steps, conv twice per step
    assert bench.whole_path_macs(macs, per, 2) == 2 * macs["conv_fwd:features.3"]
