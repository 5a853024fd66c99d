"""Micro-benchmark of drsa_amd_heatmap_sort at the bench shape (B=512, K=4, 128x128).
DRSA_AMD_SORT_GENERIC=1 selects the generic (two-read) kernel."""
import sys
import torch
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from drsa_audio_amd import ops

B, K, H, W = 512, 4, 128, 128
hm = torch.randn(B * (K + 1), 1, H, W, device="cuda")
for _ in range(3):
    ops.heatmap_sort(hm, K)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    ops.heatmap_sort(hm, K)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(f"heatmap_sort B={B} K={K} {H}x{W}: {ms:.4f} ms, {2 * hm.numel() * 4 / ms / 1e6:.0f} GB/s")
