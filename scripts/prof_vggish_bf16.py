"""VGGish-BN forward on the fp32 and bf16 plans (B = 32, 128x256), for rocprofv3 --kernel-trace."""
import copy
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from drsa_audio_amd.engine import get_engine  # noqa: E402
from drsa_audio_amd.model.create_model import VGGType  # noqa: E402
from drsa_audio_amd.utils.constants import LRP_NAME_MAP_VGGISH  # noqa: E402
from drsa_audio_amd.zennit.canonizers import SequentialMergeBatchNorm  # noqa: E402
from drsa_audio_amd.zennit.composites import NameMapComposite  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
m32 = VGGType(n_filters=(64, 64, 100, 128, 128), n_dense=100, pool_kernels=((2, 4),) + ((2, 2),) * 4, dropout=0.3,
              input_size=(128, 256), conv_bn=True, dense_bn=True).eval().to(dev)
comp = NameMapComposite(LRP_NAME_MAP_VGGISH, canonizers=[SequentialMergeBatchNorm()])
x = bench.synthetic_logmel(32, 128, 256, seed=5, device=dev)
which = sys.argv[1] if len(sys.argv) > 1 else "bf16"
m = copy.deepcopy(m32).bfloat16() if which == "bf16" else m32
eng = get_engine(m, comp)
for _ in range(10):
    eng.forward(x)
torch.cuda.synchronize()
eng.trace = []
eng.forward(x)
torch.cuda.synchronize()
for tag, e0, e1 in eng.trace:
    print(f"{tag:28s} {e0.elapsed_time(e1):8.3f} ms")
