"""Experiment helper: rebuild csrc files with extra -D defines and link a variant library
drsa_audio_amd/lib/exp/<name>.so (select it at run time with DRSA_AMD_LIB=<path>).

  python scripts/build_variant.py <name> <file.hip>[,<file.hip>...|all] [-DNAME=VAL ...]
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drsa_audio_amd import build as B


def main(name, srcs, *defs):
    B.build(verbose=False)
    exp = os.path.join(B.LIBDIR, "exp")
    os.makedirs(exp, exist_ok=True)
    allsrc = sorted(f for f in os.listdir(B.CSRC) if f.endswith(".hip"))
    sel = allsrc if srcs == "all" else [os.path.basename(s) for s in srcs.split(",")]
    paths = {s: (s if os.path.isabs(s) else os.path.join(B.CSRC, s)) for s in srcs.split(",")} if srcs != "all" else {}

    def one(src):
        obj = os.path.join(exp, f"{name}_{src.replace('.hip', '.o')}")
        srcp = paths.get(src, os.path.join(B.CSRC, src))   # an absolute path replaces its namesake
        subprocess.run([B._hipcc(), *B.CXXFLAGS, *defs, "-c", srcp, "-o", obj], check=True)
        return obj

    with ThreadPoolExecutor(8) as ex:
        new = list(ex.map(one, sel))
    objs = [os.path.join(B.OBJDIR, f.replace(".hip", ".o")) for f in allsrc if f not in sel] + new
    out = os.path.join(exp, f"{name}.so")
    subprocess.run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out, *objs], check=True)
    for o in new:
        os.remove(o)
    print(out)


if __name__ == "__main__":
    main(*sys.argv[1:])
