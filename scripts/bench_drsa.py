"""DRSA-only timing: C3 (N=20000, d=64, K=4) drsa_run and the C5 joint run (2 x d=128, K=16),
via bench.py's helpers.  python scripts/bench_drsa.py [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda", 0)
out = {"drsa_c3": bench.drsa_bench(dev, steps=steps), "drsa_joint_c5": bench.drsa_joint_bench(dev, steps=steps)}
print(json.dumps(out, indent=1))
