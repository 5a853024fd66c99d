"""Diagnostic: VGGish bf16 plan capture relevances vs the teacher-forced bf16 oracle, per layer."""
import copy
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "oracle")
sys.path.insert(0, "tests")
import lrp_ref  # noqa: E402
from lrp_common import logmel, spec, vggish  # noqa: E402
from drsa_audio_amd.engine import get_engine  # noqa: E402
from drsa_audio_amd.utils.constants import LRP_NAME_MAP_VGGISH  # noqa: E402
from drsa_audio_amd.xai.drsa.preprocessing import get_intermediate  # noqa: E402
from drsa_audio_amd.zennit.canonizers import SequentialMergeBatchNorm  # noqa: E402
from drsa_audio_amd.zennit.composites import NameMapComposite  # noqa: E402

DEV = torch.device("cuda")
size = (64, 128) if len(sys.argv) > 1 else (128, 256)
net = vggish(input_size=size).bfloat16()
x = logmel(2, *size, seed=26).bfloat16()
comp = NameMapComposite(LRP_NAME_MAP_VGGISH, canonizers=[SequentialMergeBatchNorm()])
merged = lrp_ref.merge_batch_norm(copy.deepcopy(net).float())
print({k: v for k, v in spec(LRP_NAME_MAP_VGGISH).items()})
mg = copy.deepcopy(net).to(DEV)
for j in (33, 30, 27, 26, 23):
    a, r = get_intermediate(mg, x.to(DEV), comp, j, 1)
    a, r = a.cpu(), r.cpu()
    eng = get_engine(mg, comp)
    forced = {st.name: rec["in"].cpu() for st, rec in zip(eng.stages, eng.last["stages"])}
    _, _, (act, rel) = lrp_ref.lrp(merged, spec(LRP_NAME_MAP_VGGISH), x.float(), class_idx=1, mode="bf16",
                                   capture=f"features.{j}", forced_inputs=forced)
    print(j, [(float((a[b].double() - act[b]).norm() / act[b].norm()),
               float((r[b].double() - rel[b]).norm() / rel[b].norm())) for b in range(2)], flush=True)
