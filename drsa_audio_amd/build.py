"""Build the in-tree HIP library ``drsa_audio_amd/lib/libdrsa_amd.so`` for gfx950.

``python -m drsa_audio_amd.build`` (or ``__graft_entry__.build()``).  Each
``csrc/*.hip`` is compiled to an object with ``hipcc --offload-arch=gfx950`` (in
parallel, skipped when up to date) and linked into one shared library exposing the
C ABI declared in ``include/drsa_amd.h``.  The library is git-ignored but travels
to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(HERE, "lib", "obj")
LIB = os.path.join(LIBDIR, "libdrsa_amd.so")
ROOT = os.path.dirname(HERE)
ARCH = os.environ.get("DRSA_AMD_ARCH", "gfx950")

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off", "-Wall",
            "-Wno-unused-result", "-Wno-unused-variable", "-Wno-unused-function",
            "-I", CSRC, "-I", os.path.join(ROOT, "include")]


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build drsa_amd)")


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers_mtime() -> float:
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs += [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))]
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _compile(src: str, hipcc: str, hdr_t: float) -> str:
    obj = os.path.join(OBJDIR, os.path.basename(src).replace(".hip", ".o"))
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_t):
        return obj
    cmd = [hipcc, *CXXFLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    return obj


def build(verbose: bool = True, jobs: int | None = None) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    hipcc = _hipcc()
    hdr_t = _headers_mtime()
    srcs = _sources()
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4)), 8)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hipcc, hdr_t), srcs))
    if (not os.path.exists(LIB)) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB + ".tmp", *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        os.replace(LIB + ".tmp", LIB)
    build_torch_ops(hipcc)
    if verbose:
        print(f"[drsa_amd] built {LIB} from {len(srcs)} sources (+ {os.path.basename(TORCH_LIB)})")
    return LIB


TORCH_SRC = os.path.join(HERE, "csrc_torch", "ops_torch.cpp")
TORCH_LIB = os.path.join(LIBDIR, "libdrsa_amd_torch.so")


def build_torch_ops(hipcc: str) -> str:
    """The C++ TORCH_LIBRARY(drsa_amd) registration (csrc_torch/ops_torch.cpp): host code compiled
    against the installed torch and linked to libdrsa_amd.so (rpath $ORIGIN)."""
    deps = [TORCH_SRC, LIB, os.path.join(ROOT, "include", "drsa_amd.h")]
    if os.path.exists(TORCH_LIB) and os.path.getmtime(TORCH_LIB) >= max(os.path.getmtime(d) for d in deps):
        return TORCH_LIB
    import torch
    tdir = os.path.dirname(torch.__file__)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = [hipcc, "-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", os.path.join(tdir, "include"),
           "-I", os.path.join(tdir, "include", "torch", "csrc", "api", "include"), "-I", os.path.join(ROOT, "include"),
           "-Wno-deprecated-declarations", TORCH_SRC, "-o", TORCH_LIB + ".tmp", "-L", LIBDIR, "-ldrsa_amd",
           "-L", os.path.join(tdir, "lib"), "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
           "-Wl,-rpath,$ORIGIN"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"torch op library build failed:\n{r.stderr[-6000:]}")
    os.replace(TORCH_LIB + ".tmp", TORCH_LIB)
    return TORCH_LIB


if __name__ == "__main__":
    build()
    sys.exit(0)
