"""Steady-state DRSA step times (bench.py's captured-graph replays): C3 and the C5 joint run.
Prints {"ms": C3 ms/step, "joint_ms": C5 joint ms/step}; used with scripts/ab_lib.sh.
python scripts/bench_drsa_steady.py [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import torch  # noqa: E402

import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda", 0)
c3 = bench.drsa_bench(dev, steps=steps)
j = bench.drsa_joint_bench(dev, steps=steps)
print(json.dumps({"ms": c3["ms_per_step"], "c3_spread": c3["ms_per_step_spread"], "joint_ms": j["ms_per_joint_step"],
                  "joint_spread": j["ms_per_joint_step_spread"], "event_ms": c3["event_ms"]}))
