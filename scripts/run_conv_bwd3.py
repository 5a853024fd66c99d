"""Times drsa_amd_conv_bwd at the GTZAN-128 features.3 bench shape (B=512 x 5 clones); used
under rocprofv3 --pmc by scripts/pmc_kernel.sh."""
import os, sys, torch, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drsa_audio_amd import _capi
dev = torch.device("cuda")
Bs, clones = 512, 4
Bq = Bs * clones
g = torch.randn(Bq, 32, 32, 32, device=dev)
amax = torch.randint(0, 4, (Bs, 32, 32, 32), device=dev, dtype=torch.uint8)
w = torch.randn(1, 9 * 32, 32, device=dev)
x = torch.rand(Bs, 32, 64, 64, device=dev)
den = torch.rand(Bs, 32, 64, 64, device=dev) + 0.5
out = torch.empty(Bq, 32, 64, 64, device=dev)
s = _capi.stream_ptr()
def run():
    _capi.call("drsa_amd_conv_bwd", g.data_ptr(), amax.data_ptr(), w.data_ptr(), x.data_ptr(), den.data_ptr(), out.data_ptr(), Bq, clones, 32, 32, 64, 64, 1, 1, 1, 1e-7, s)
for _ in range(3): run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10): run()
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
print(json.dumps({"ms": ms, "tflops": 2 * 37748736 * Bq / ms / 1e9}))
