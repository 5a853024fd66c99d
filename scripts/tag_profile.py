"""Map rocprofv3 dispatch records of one bench.py run onto the engine's kernel tags.

bench.py --tag-order F writes the ordered tags of one hot-path step (every engine call is one
HIP launch) and how many main steps ran before the secondary workloads.  Our kernels' dispatches
(setup launches skipped) are then assigned to tags by position, the names checked to repeat per
step, and per-tag averages written:

  python scripts/tag_profile.py trace  <dir-with-kernel_trace.csv> F  -> avg duration per tag
  python scripts/tag_profile.py pmc    <root-with-pmc_*/> F [out.json] -> HBM bytes per launch per tag
                                        (2 x FETCH_SIZE + WRITE_SIZE, KB->B; gfx950 FETCH_SIZE
                                         counts half of wide reads: MI355X_MICROARCH.md "HBM")
    and, when <root>/pmc_CLOCK/ exists, per tag the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / the
    dispatch's wall time, MI355X_MICROARCH.md "DVFS give-back") and the MFMA-pipe occupancy
    (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x those cycles)
"""
import csv
import glob
import json
import sys
from collections import defaultdict

OURS = ("conv3x3_kernel", "linear_kernel", "linear_fwd_kernel", "linear_fwd_w1_kernel", "projection_fwd_kernel", "projection_bwd_kernel",
        "projection_bwd_rc_kernel", "first_conv_pool_kernel", "first_layer_bwd", "heatmap_sort_kernel",
        "heatmap_sort_cached_kernel")


def _ours(name):
    return any(k in name for k in OURS)


def _assign(rows, order):
    tags, steps = order["tags"], order["main_steps"]
    L = len(tags)
    rows = [r for r in rows if _ours(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    main = rows[:L * steps]
    if len(main) < L * steps:
        raise SystemExit(f"only {len(main)} of {L * steps} expected dispatches found")
    for i, r in enumerate(main):
        if r["Kernel_Name"] != main[i % L]["Kernel_Name"]:
            raise SystemExit(f"dispatch {i}: kernel name does not repeat per step")
    out = defaultdict(list)
    for i, r in enumerate(main):
        out[tags[i % L]].append(r)
    return out, {t: main[j]["Kernel_Name"] for j, t in enumerate(tags)}


def trace(d, order_path):
    order = json.load(open(order_path))
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    by, names = _assign(rows, order)
    res = {}
    for t, rs in by.items():
        ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rs]
        ds = ds[1:] if len(ds) > 1 else ds          # first launch includes code-object warm-up
        res[t] = {"avg_ms": sum(ds) / len(ds), "launches": len(ds), "kernel": names[t]}
    return res


def pmc(root, order_path):
    order = json.load(open(order_path))
    per = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = []
        for f in glob.glob(f"{root}/pmc_{counter}/**/*counter_collection.csv", recursive=True):
            rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
        by, names = _assign(rows, order)
        for t, rs in by.items():
            v = sum(float(r["Counter_Value"]) for r in rs) / len(rs) * 1024.0
            per.setdefault(t, {"kernel": names[t]})[counter.lower() + "_bytes"] = v
    for t, v in per.items():
        v["hbm_bytes"] = 2.0 * v["fetch_size_bytes"] + v["write_size_bytes"]
    # No clock figure: GRBM_GUI_ACTIVE / 8 XCDs over the kernel's own timestamps read 2.4-6.7 GHz on a
    # PMC-serialised dispatch (counter-window overhead), above the 2.4 GHz the peak is quoted at.
    return {"note": "per-launch HBM bytes at bench batch %d: 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE "
                    "counts half of 16-B/lane reads)" % order["batch"],
            "per_launch_bytes": {t: v["hbm_bytes"] for t, v in per.items()}, "detail": per}


if __name__ == "__main__":
    mode, path, order = sys.argv[1:4]
    res = trace(path, order) if mode == "trace" else pmc(path, order)
    txt = json.dumps(res, indent=1)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(txt)
    print(txt)
