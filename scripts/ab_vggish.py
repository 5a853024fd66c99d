"""Micro-bench: VGGish-BN fp32 standard LRP (B = 32, 128 x 256): samples/s and per-tag ms (JSON)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from drsa_audio_amd.engine import get_engine  # noqa: E402
from drsa_audio_amd.model.create_model import VGGType  # noqa: E402
from drsa_audio_amd.utils.constants import LRP_NAME_MAP_VGGISH  # noqa: E402
from drsa_audio_amd.xai.explain.attribute import compute_relevances  # noqa: E402
from drsa_audio_amd.zennit.canonizers import SequentialMergeBatchNorm  # noqa: E402
from drsa_audio_amd.zennit.composites import NameMapComposite  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = VGGType(n_filters=(64, 64, 100, 128, 128), n_dense=100, pool_kernels=((2, 4),) + ((2, 2),) * 4, dropout=0.3,
            input_size=(128, 256), conv_bn=True, dense_bn=True).eval().to(dev)
if len(sys.argv) > 1 and sys.argv[1] == "bf16":
    m = m.bfloat16()
comp = NameMapComposite(LRP_NAME_MAP_VGGISH, canonizers=[SequentialMergeBatchNorm()])
x = bench.synthetic_logmel(32, 128, 256, seed=5, device=dev)
if m.features[0].weight.dtype == torch.bfloat16:
    x = x.bfloat16()
for _ in range(3):
    compute_relevances(m, x, comp, class_idx=1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    compute_relevances(m, x, comp, class_idx=1)
torch.cuda.synchronize()
sps = 32 * 20 / (time.perf_counter() - t0)
eng = get_engine(m, comp)
eng.trace = []
for _ in range(5):
    compute_relevances(m, x, comp, class_idx=1)
torch.cuda.synchronize()
per = {}
for tag, e0, e1 in eng.trace:
    per.setdefault(tag, []).append(e0.elapsed_time(e1))
print(json.dumps({"samples_per_s": sps, "ms": 32 / sps * 1e3,
                  "kernels": {k: round(sum(v) / len(v), 4) for k, v in per.items()}}))
