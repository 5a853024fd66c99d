"""A/B of the batched DRSA grid partial: workgroups per problem (the result is the same bits for any)."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from drsa_audio_amd.xai.drsa.drsa import drsa_run_batched  # noqa: E402
from drsa_audio_amd.xai.drsa.preprocessing import normalize_vectors  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(1234)
probs = []
for i in range(90):
    d = (100, 128, 128)[i % 3]
    A = torch.randn(20000, d, device=dev, generator=g).abs_()
    C = torch.randn(20000, d, device=dev, generator=g)
    U0 = torch.linalg.qr(torch.randn(d, d, device=dev, generator=g))[0].contiguous()
    probs.append((normalize_vectors(A, out=A), normalize_vectors(C, out=C), U0, 4))
s = torch.cuda.Stream(dev)
steps = 60
ref = None
with torch.cuda.stream(s):
    for blocks in [int(b) for b in sys.argv[1:]] or [0, 8, 11, 16, 32]:
        drsa_run_batched(probs, 2, blocks=blocks)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = drsa_run_batched(probs, steps, blocks=blocks)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        same = ref is None or all(torch.equal(a[1], b[1]) for a, b in zip(out, ref))
        ref = ref or out
        print(f"blocks {blocks:4d}: {90 * steps / dt:9.0f} problem-steps/s  same={same}", flush=True)
