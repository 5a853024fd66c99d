"""Micro-benchmark of the log-mel front end (bench.frontend_bench) for kernel A/B runs, plus a bit
checksum of one launch's output (variants that claim the same bits must print the same one)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench


def checksum(device):
    from drsa_audio_amd.utils.dataloading import Loader
    from drsa_audio_amd.utils.synthetic import synthetic_songs
    songs = torch.from_numpy(synthetic_songs(8, seed=3)).to(device)
    out = Loader("gtzan", device=device).load_songs(songs)
    x = out[0] if isinstance(out, (tuple, list)) else out
    xi = x.contiguous().view(torch.int32).to(torch.int64)
    return int((xi * (torch.arange(xi.numel(), device=device, dtype=torch.int64).view_as(xi) % 1000003 + 1)).sum())


dev = torch.device("cuda")
r = bench.frontend_bench(dev)
r["lib"] = os.environ.get("DRSA_AMD_LIB", "default")
r["bits_checksum"] = checksum(dev)
print(json.dumps(r))
