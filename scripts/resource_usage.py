"""Per-kernel VGPR/AGPR/occupancy table from hipcc -Rpass-analysis=kernel-resource-usage."""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]


def usage(src, defs=()):
    cmd = [*()] + ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
           "-I", f"{ROOT}/drsa_audio_amd/csrc", "-I", f"{ROOT}/include", "-c", src, "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage", *defs]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": subprocess.run(["c++filt"], input=t.split(":", 1)[1].strip(), capture_output=True,
                                          text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    return rows


if __name__ == "__main__":
    defs = [a for a in sys.argv[1:] if a.startswith("-D")]
    for src in [a for a in sys.argv[1:] if not a.startswith("-D")]:
        for r in usage(src, defs):
            name = r["name"].replace("(anonymous namespace)::", "")
            name = re.sub(r"\(.*", "", name)
            print(f"{name[:70]:70s} V{r.get('VGPRs'):>4} A{r.get('AGPRs'):>4} occ{r.get('Occupancy [waves/SIMD]'):>2} "
                  f"spill{r.get('VGPRs Spill')} sgpr{r.get('TotalSGPRs')}")
