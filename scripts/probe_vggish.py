"""Diagnostic: where does the VGGish engine path leave the exact oracle?  (GPU box)"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch

import lrp_ref
from lrp_common import logmel, spec, vggish
from drsa_audio_amd.engine import get_engine
from drsa_audio_amd.utils.constants import LRP_NAME_MAP_VGGISH
from drsa_audio_amd.zennit.canonizers import SequentialMergeBatchNorm
from drsa_audio_amd.zennit.composites import NameMapComposite
from drsa_audio_amd.xai.drsa.preprocessing import get_intermediate

DEV = torch.device("cuda")
net = vggish(input_size=(64, 128))
merged = lrp_ref.merge_batch_norm(net)
comp = NameMapComposite(LRP_NAME_MAP_VGGISH, canonizers=[SequentialMergeBatchNorm()])
m = copy.deepcopy(net).to(DEV)
eng = get_engine(m, comp)
for st in eng.stages:
    i = int(st.name.split(".")[1])
    wref = merged.features[i].weight
    print(st.name, "W fold eq", torch.equal(st.W.cpu(), wref), "b eq", torch.equal(st.b.cpu(), merged.features[i].bias),
          "pool", st.pool_k if st.pool else None, "kind", st.rule_kind, "nonneg", st.input_nonneg)
for ds in eng.dense:
    i = int(ds.name.split(".")[1])
    print(ds.name, "W eq", torch.equal(ds.W.cpu(), merged.classifier[i].weight), "b eq",
          torch.equal(ds.b.cpu(), merged.classifier[i].bias))
x = logmel(3, 64, 128, seed=3)
lg_ref, _ = lrp_ref.lrp(merged, spec(LRP_NAME_MAP_VGGISH), x, class_idx=4, mode="exact")
lg = eng.forward(x.to(DEV))
print("logits eq", torch.equal(lg.cpu(), lg_ref), float((lg.cpu() - lg_ref).abs().max()))
for li in [33, 30, 26, 23, 19, 16, 12, 9, 5, 2]:
    _, _, (act, rel) = lrp_ref.lrp(merged, spec(LRP_NAME_MAP_VGGISH), x, class_idx=4, mode="exact",
                                   capture=f"features.{li}")
    a, r = get_intermediate(m, x.to(DEV), comp, li, 4)
    print(f"features.{li}: act eq {torch.equal(a.cpu(), act)} d={float((a.cpu() - act).abs().max()):.3g}  "
          f"rel eq {torch.equal(r.cpu(), rel)} d={float((r.cpu() - rel).abs().max()):.3g} |rel|={float(rel.abs().max()):.3g}")
