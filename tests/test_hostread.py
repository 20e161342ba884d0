"""utils.hostread: early read-backs polled on their data, the event only as the fallback."""
import numpy as np
import pytest
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


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", [False, True])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32, torch.int32, torch.int64, torch.bool])
def test_stage_lands_the_device_values(monkeypatch, kernel, dtype):
    """stage() → landed() returns the device tensor's values, through the host_store kernel
    (ops/csrc/hostread.hip: system-scope stores into the pinned buffer) and through the async copy;
    the kernel's buffers stay referenced until their event completes."""
    from hfens import ops
    monkeypatch.setattr(hostread, "KERNEL_STORE", kernel)
    g = torch.Generator().manual_seed(3)
    for n in (1, 7, 300, 70000):
        ref = (torch.randn(n, generator=g, dtype=torch.float64) * 100).to(dtype)
        dev = ref.cuda()
        dev2 = dev * 1 if dtype != torch.bool else dev.clone()      # (a kernel right before the read)
        host, ev = hostread.stage(dev2)
        out = hostread.landed(host, ev, budget_s=5.0)
        exp = ref.to(torch.int32) if dtype == torch.bool else ref
        assert np.array_equal(out, exp.numpy())
        if kernel:
            assert any(h is host for h, _ in hostread._INFLIGHT)
            assert hasattr(ops.ext(), "host_store")
    torch.cuda.synchronize()
