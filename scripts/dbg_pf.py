import sys, os
R0=os.environ.get("GRAFT_REPO_ROOT","."); sys.path[:0]=[R0]+[os.path.join(R0,d) for d in ("tests","oracle")]
import torch
import lrp_ref
from lrp_common import gtzan128, logmel
from drsa_audio_amd.xai.pixelflipping.pf import PixelFlipping
from drsa_audio_amd.xai.explain.attribute import compute_relevances
from drsa_audio_amd.zennit.composites import NameMapComposite
net=gtzan128(); x=logmel(1, seed=60)
conf={"convolutional": ("gamma", 0.25), "dense": ("epsilon", 1e-7), "first_layer": ("wsquare",)}
pf=PixelFlipping(net, torch.zeros(10,1,128,128), num_classes=10, device='cuda'); pf.canonizer=None; pf.stabilizers=None
comp=pf._get_composite(conf)
robj=comp.rules(net)
def sp(r):
    k=r.kind
    return {"epsilon":("epsilon",getattr(r,'epsilon',None)),"gamma":("gamma",getattr(r,'gamma',None),getattr(r,'stabilizer',None)),"wsquare":("wsquare",getattr(r,'stabilizer',None)),"pass":("pass",)}[k]
rules={n:sp(r) for n,r in robj.items()}
nm=NameMapComposite([([n],r) for n,r in robj.items() if r.kind!='pass'])
Ra=compute_relevances(net, x.cuda(), comp, class_idx=0).cpu()
Rb=compute_relevances(net, x.cuda(), nm, class_idx=0).cpu()
_,Rc=lrp_ref.lrp(net.cpu(),rules,x,class_idx=0,mode="exact")
print("a==b",torch.equal(Ra,Rb),"b==c",torch.equal(Rb,Rc),"a==c",torch.equal(Ra,Rc))
print((Ra-Rc).abs().max(), (Rb-Rc).abs().max(), Rc.abs().max())
d=(Ra-Rc).abs()
print("n diff", (d>0).sum().item(), "of", d.numel())
