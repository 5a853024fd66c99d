"""C-ABI boundary: the library builds, loads and exports every symbol include/drsa_amd.h declares.
Runs on CPU (no compute calls)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "drsa_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(drsa_amd_\w+)\s*\(", src)))


def test_header_declares_entry_points():
    names = _declared()
    assert "drsa_amd_drsa_step" in names and "drsa_amd_last_error" in names


def test_library_exports_all_declared_symbols():
    from drsa_audio_amd import _capi
    if not os.path.exists(_capi.LIB_PATH):
        from drsa_audio_amd import build
        build.build(verbose=False)
    lib = ctypes.CDLL(_capi.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, f"symbols declared in include/drsa_amd.h but not exported: {missing}"


def test_python_signatures_cover_header():
    from drsa_audio_amd import _capi
    assert set(_declared()) <= set(_capi.SIGNATURES), set(_declared()) - set(_capi.SIGNATURES)


def test_version_and_error_calls_without_gpu():
    from drsa_audio_amd import _capi
    lib = _capi.load()
    assert lib.drsa_amd_version() >= 1
    assert isinstance(lib.drsa_amd_last_error(), bytes)
    # argument validation happens before any device work
    assert lib.drsa_amd_drsa_workspace_bytes(100, 63, 4) == 0
    assert lib.drsa_amd_drsa_workspace_bytes(100, 64, 4) > 0


def test_bf16_weight_layout_host_logic():
    """plan._bf16_layout: [ng][9*cin_p][cout_p] (k = ci*9 + tap) -> [ng][cin_p/16][9][2][cout_p][8],
    ci = 16*chunk + 8*half + j (the layout drsa_amd_conv_fwd_bf16 stages, include/drsa_amd.h)."""
    import torch
    from drsa_audio_amd.engine.plan import _bf16_layout
    ng, cin_p, cout_p = 2, 32, 64
    wf = torch.arange(ng * 9 * cin_p * cout_p, dtype=torch.float32).reshape(ng, 9 * cin_p, cout_p) % 251
    t = _bf16_layout(wf, cin_p, cout_p)
    assert t.dtype == torch.bfloat16 and tuple(t.shape) == (ng, cin_p // 16, 9, 2, cout_p, 8)
    for g, ci, tap, co in [(0, 0, 0, 0), (1, 31, 8, 63), (0, 17, 4, 5), (1, 8, 3, 40)]:
        assert float(t[g, ci // 16, tap, (ci % 16) // 8, co, ci % 8]) == float(wf[g, ci * 9 + tap, co])
