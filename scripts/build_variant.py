"""Experiment helper: rebuild ONE csrc file with extra -D defines and link a variant library
drsa_audio_amd/lib/exp/<name>.so (select it at run time with DRSA_AMD_LIB=<path>).

  python scripts/build_variant.py <name> <file.hip> [-DNAME=VAL ...]
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drsa_audio_amd import build as B


def main(name, src, *defs):
    B.build(verbose=False)
    exp = os.path.join(B.LIBDIR, "exp")
    os.makedirs(exp, exist_ok=True)
    srcp = src if os.path.isabs(src) else os.path.join(B.CSRC, src)   # an absolute path replaces its namesake
    src = os.path.basename(src)
    obj = os.path.join(exp, f"{name}_{src.replace('.hip', '.o')}")
    subprocess.run([B._hipcc(), *B.CXXFLAGS, *defs, "-c", srcp, "-o", obj], check=True)
    objs = [os.path.join(B.OBJDIR, f.replace(".hip", ".o")) for f in sorted(os.listdir(B.CSRC)) if f.endswith(".hip")
            and f != src] + [obj]
    out = os.path.join(exp, f"{name}.so")
    subprocess.run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out, *objs], check=True)
    print(out)


if __name__ == "__main__":
    main(*sys.argv[1:])
