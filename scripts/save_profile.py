"""Copy one GPU pass's judged artefacts from gpurun_out/<tag> into profiles/<name> (tracked).

  python scripts/save_profile.py gpurun_out/r01_s2a profiles/r01_s2 [--current]

--current also installs the PMC traffic table as profiles/pmc_traffic.json, which bench.py
reads to fill roofline.traffic for the dominant kernel.
"""
import json
import os
import shutil
import subprocess
import sys


def main(src, dst, current=False):
    os.makedirs(dst, exist_ok=True)
    pairs = [("bench.json", "bench.json"), ("prof/run_kernel_stats.csv", "kernel_stats.csv"),
             ("prof_tags_timing.json", "tag_timing.json"), ("pmc/pmc_traffic.json", "pmc_traffic.json"),
             ("pytest_gpu.log", "pytest_gpu.log"), ("smoke.log", "smoke.log")]
    for a, b in pairs:
        p = os.path.join(src, a)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, b))
    lines = []
    bj = os.path.join(src, "bench.json")
    if os.path.exists(bj):
        d = json.load(open(bj))
        lines += [f"# {os.path.basename(dst)}", "",
                  f"bench: **{d['value']:.0f} {d['unit']}** (B={d['config']['per_gpu_batch']}, "
                  f"{d['ms_per_step']:.2f} ms/step, {d['n_gpus']} GPU)", "",
                  f"roofline: `{d['roofline']['kernel']}` {d['roofline']['achieved']:.1f} "
                  f"{d['roofline']['unit']} = {d['roofline']['frac']:.3f} of {d['roofline']['peak']}", ""]
        tt = os.path.join(src, "prof_tags_timing.json")
        if os.path.exists(tt):
            t = json.load(open(tt))
            pm = {}
            pp = os.path.join(src, "pmc/pmc_traffic.json")
            if os.path.exists(pp):
                pm = json.load(open(pp)).get("per_launch_bytes", {})
            lines += ["| tag | bench HIP-event avg ms | rocprof avg ms | HBM MB/launch (PMC) |", "|---|---:|---:|---:|"]
            for k, v in t.items():
                be = d["kernels"].get(k, {}).get("avg_ms", float("nan"))
                hb = pm.get(k)
                lines.append(f"| {k} | {be:.3f} | {v['avg_ms']:.3f} | {'' if hb is None else f'{hb/1e6:.1f}'} |")
            lines.append("")
    ks = os.path.join(src, "prof/run_kernel_stats.csv")
    if os.path.exists(ks):
        lines += ["rocprofv3 --kernel-trace --stats (whole bench process: B=512 steps, bs=64 lines, DRSA):", ""]
        lines.append(subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "prof_summary.py"), ks, "16"],
                                    capture_output=True, text=True, check=True).stdout)
    with open(os.path.join(dst, "summary.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    if current and os.path.exists(os.path.join(dst, "pmc_traffic.json")):
        pm = json.load(open(os.path.join(dst, "pmc_traffic.json")))
        pm["profile"] = os.path.basename(os.path.normpath(dst))      # bench.py names it in traffic_source
        with open(os.path.join(os.path.dirname(dst), "pmc_traffic.json"), "w") as fh:
            json.dump(pm, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], "--current" in sys.argv)
