"""Micro-benchmark of the log-mel front end (bench.frontend_bench) for kernel A/B runs."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench

print(json.dumps(bench.frontend_bench(torch.device("cuda"))))
