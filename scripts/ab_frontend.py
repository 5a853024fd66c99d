"""A/B of the log-mel front end (bench.frontend_bench) across variant libraries
(scripts/build_variant.py): python scripts/ab_frontend.py lib1.so lib2.so ..."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for rnd in range(2):
    for lib in sys.argv[1:]:
        env = dict(os.environ, DRSA_AMD_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "bench_frontend.py")], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if line:
            d = json.loads(line[-1])
            print(rnd, os.path.basename(lib), round(d["ms_per_launch"], 4), "ms", round(d["roofline"]["frac"], 3),
                  "err", d.get("max_abs_logmel_err_vs_f64_oracle_song0"), flush=True)
        else:
            print(rnd, os.path.basename(lib), r.stderr[-600:], flush=True)
