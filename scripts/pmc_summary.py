"""Per-kernel averages of rocprofv3 --pmc counter_collection.csv files (one pass per directory)."""
import collections
import csv
import glob
import json
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    m = re.match(r"void drsa_conv::conv3x3_kernel<([^>]*)>", name)
    if m:
        return "conv<" + m.group(1).replace(" ", "") + ">"
    return re.sub(r"\(.*", "", name).replace("void ", "")


def load(root="gpurun_out"):
    data = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/pmc_*/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            data[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return data


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    d = load(root)
    rows = []
    for k, c in d.items():
        avg = {n: sum(v) / len(v) for n, v in c.items()}
        rows.append((k, avg))
    rows.sort(key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))
    keys = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
            "GRBM_GUI_ACTIVE", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
            "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VMEM", "FETCH_SIZE", "WRITE_SIZE"]
    print(json.dumps({k: {n: round(v, 1) for n, v in a.items()} for k, a in rows[:12]}, indent=1))
