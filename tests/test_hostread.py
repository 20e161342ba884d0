"""utils.hostread: early read-backs polled on their data, the event only as the fallback."""
import numpy as np
import torch

from hfens.utils import hostread


class _Ev:
    def __init__(self, on_sync=None):
        self.calls = 0
        self.on_sync = on_sync

    def synchronize(self):
        self.calls += 1
        if self.on_sync is not None:
            self.on_sync()


def test_landed_returns_written_data_without_the_event():
    h = torch.tensor([1.5, -2.0, 0.0], dtype=torch.float64)
    ev = _Ev()
    assert np.array_equal(hostread.landed(h, ev), [1.5, -2.0, 0.0]) and ev.calls == 0
    hi = torch.tensor([0, 3, 7], dtype=torch.int64)
    assert np.array_equal(hostread.landed(hi, ev), [0, 3, 7]) and ev.calls == 0


def test_landed_falls_back_to_the_event_on_a_remaining_sentinel():
    h = torch.tensor([1.0, float("nan")], dtype=torch.float64)
    ev = _Ev(on_sync=lambda: h.__setitem__(1, 2.0))
    assert np.array_equal(hostread.landed(h, ev, budget_s=0.001), [1.0, 2.0]) and ev.calls == 1
    hi = torch.tensor([4, hostread.SENTINEL], dtype=torch.int64)
    ev2 = _Ev()
    out = hostread.landed(hi, ev2, budget_s=0.001)
    assert ev2.calls == 1 and out[1] == hostread.SENTINEL   # (a value equal to the sentinel: event path)
