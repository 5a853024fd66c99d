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
