"""A/B of the conv3 backward shape (GTZAN-128 features.3, K+1=5 clones of B=512) across variant
libraries (scripts/build_variant.py): python scripts/ab_conv3.py lib1.so lib2.so ...
One child process per library (DRSA_AMD_LIB), HIP-event time of 20 launches, 3 rounds interleaved."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ablate_conv import CHILD  # noqa: E402  (same workload as the ablation script)
CHILD = CHILD.replace("range(10)", "range(20)").replace("/ 10", "/ 20")
res = {}
for rnd in range(3):
    for lib in sys.argv[1:]:
        env = dict(os.environ, DRSA_AMD_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        v = json.loads(line[0])["ms"] if line else None
        res.setdefault(os.path.basename(lib), []).append(v)
        print(rnd, os.path.basename(lib), v if v is not None else r.stderr[-500:], flush=True)
print(json.dumps({k: min(x for x in v if x is not None) for k, v in res.items()}))
