"""Custom-op registration (drsa_audio_amd/ops.py) on CPU: every op is in torch.ops.drsa_amd, the
fake (meta) kernels give the output shapes without a GPU, and CPU tensors are refused (no CPU
kernel, no fallback)."""
import pytest
import torch

import drsa_audio_amd.ops as dops
from drsa_audio_amd import _capi

M = "meta"


def test_all_ops_registered():
    for name in dops.__all__:
        assert hasattr(torch.ops.drsa_amd, name), name


def test_meta_shapes():
    o = torch.ops.drsa_amd
    A, U = torch.empty(10, 100, device=M), torch.empty(100, 100, device=M)
    Un, f = o.drsa_step(A, A, U, 4)
    assert Un.shape == (100, 100) and f.shape == ()
    Ur, tr = o.drsa_run(A, A, U, 4, 7)
    assert tr.shape == (8,)
    assert o.subspace_relevances(torch.empty(3, 10, 100, device=M), torch.empty(3, 10, 100, device=M), U, 4).shape == (3, 4)
    y, am, den = o.lrp_conv_fwd(torch.empty(2, 32, 64, 64, device=M), torch.empty(2, 288, 32, device=M),
                                torch.empty(3, 32, device=M), None, 32, 2, True)
    assert y.shape == (2, 32, 32, 32) and am.dtype == torch.uint8
    G = o.projection_bwd(torch.empty(2, 64, 16, 16, device=M), None, torch.empty(2, 64, 32, 32, device=M), None,
                         torch.empty(64, 64, device=M), 4, 1e-6, 1e-7, True)
    assert G.shape == (10, 64, 32, 32)
    std, srel, sub, rel, mask = o.heatmap_sort(torch.empty(10, 1, 128, 128, device=M), 4)
    assert sub.shape == (2, 4, 128, 128) and mask.dtype == torch.int64
    assert o.logmel(torch.empty(8, 48000, device=M), 800, 360, 128, 128, True).shape == (8, 1, 128, 128)


def test_cpu_tensors_refused():
    # no CPU kernel is registered: the dispatcher refuses (NotImplementedError is a RuntimeError)
    with pytest.raises(RuntimeError):
        torch.ops.drsa_amd.drsa_step(torch.rand(10, 64), torch.rand(10, 64), torch.eye(64), 4)
    with pytest.raises(RuntimeError):
        torch.ops.drsa_amd.polar(torch.eye(8))


def test_ops_are_registered_from_cpp():
    """The stage ops come from the C++ TORCH_LIBRARY(drsa_amd) of libdrsa_amd_torch.so (visible to
    TorchScript / C++ callers), with a CUDA (HIP) kernel and no CPU kernel."""
    for name in dops.__all__:
        if name == "logmel":
            continue
        dump = torch._C._dispatch_dump(f"drsa_amd::{name}")
        assert "ops_torch.cpp" in dump, (name, dump)
        assert torch._C._dispatch_has_kernel_for_dispatch_key(f"drsa_amd::{name}", "CUDA"), name
        assert not torch._C._dispatch_has_kernel_for_dispatch_key(f"drsa_amd::{name}", "CPU"), name


def test_torchscript_sees_the_ops():
    @torch.jit.script
    def f(V: torch.Tensor) -> torch.Tensor:
        return torch.ops.drsa_amd.polar(V)
    assert "drsa_amd::polar" in str(f.graph)
