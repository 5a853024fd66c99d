"""Debug probe: HIP LRP engine vs the exact (pinned-order) oracle."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "scripts")]
import numpy as np, torch
import lrp_ref
from probe_lrp import spec, logmel, err
from drsa_audio_amd.model.create_model import VGGType
from drsa_audio_amd.model.modify_model import ProjectionModel
from drsa_audio_amd.utils.constants import LRP_NAME_MAP_GTZAN, LRP_NAME_MAP_TOY
from drsa_audio_amd.zennit.composites import NameMapComposite
from drsa_audio_amd.xai.explain.attribute import compute_relevances
from drsa_audio_amd.xai.explain.explainer import HeatmapGenerator
dev = torch.device("cuda")
torch.manual_seed(0)
m = VGGType(n_filters=(32, 32, 64, 64, 128), n_dense=128, pool_kernels=((2, 2),) * 5, dropout=0.4,
            input_size=(128, 128), conv_bn=False, dense_bn=False, block_depth=1).eval()
x = logmel(2, 128, 128, 1)
lg_ref, Rref = lrp_ref.lrp(m, spec(LRP_NAME_MAP_GTZAN), x, class_idx=3, mode="exact")
from drsa_audio_amd.engine import get_engine
mg = m.to(dev)
comp = NameMapComposite(LRP_NAME_MAP_GTZAN)
eng = get_engine(mg, comp)
lg = eng.forward(x.to(dev))
print("logits exact diff", float((lg.cpu() - lg_ref).abs().max()))
Rg = compute_relevances(mg, x.to(dev), comp, class_idx=3)
print("C2 exact: maxabs", float((Rg.cpu() - Rref).abs().max()), "maxnorm/relL2", err(Rg.cpu(), Rref),
      "n_diff", int((Rg.cpu() != Rref).sum()), "/", Rref.numel())
U = torch.from_numpy(np.load(os.path.join(ROOT, "tests/golden/u64_seed42.npy")))
pm = ProjectionModel(m.cpu(), 7, U, 4).eval()
ref = lrp_ref.subspace_heatmaps(pm, spec(LRP_NAME_MAP_GTZAN), 4, x, class_idx=3, mode="exact")
hg = HeatmapGenerator(m.to(dev), U, LRP_NAME_MAP_GTZAN, "blues", num_concepts=4, layer_idx=7, device="cuda")
hg.generate_subspace_heatmaps(x)
for k in ["standard_heatmaps", "subspace_heatmaps", "standard_relevance", "subspace_relevances", "mask"]:
    a, b = hg.info[k], ref[k]
    print(k, "max abs diff", float(np.abs(a.astype(np.float64) - b.astype(np.float64)).max()),
          "n_diff", int((a != b).sum()), "/", a.size)
# toy C1
torch.manual_seed(0)
toy = VGGType(n_filters=(8, 8, 16, 16, 16), n_dense=32, n_classes=2, pool_kernels=((2, 2),) * 5, dropout=0.0,
              input_size=(64, 64), conv_bn=False, dense_bn=False, block_depth=1).eval()
xt = logmel(1, 64, 64, 5)
_, Rt = lrp_ref.lrp(toy, spec(LRP_NAME_MAP_TOY), xt, class_idx=1, mode="exact")
Rtg = compute_relevances(toy.to(dev), xt.to(dev), NameMapComposite(LRP_NAME_MAP_TOY), class_idx=1)
print("toy exact: maxabs", float((Rtg.cpu() - Rt).abs().max()), "n_diff", int((Rtg.cpu() != Rt).sum()))
