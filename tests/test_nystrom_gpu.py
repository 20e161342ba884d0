"""ops/csrc/nystrom.hip rbf_f64 (the Nyström map's RBF matrices, one pass) against a plain fp64
PyTorch reference of the same op, and the map it feeds (Φ Φᵀ, invariant to the eigenbasis) against
the library-form map."""
import pytest
import torch

from hfens import ops
from hfens.models import svc_lowrank

pytestmark = pytest.mark.gpu


def _ref(A, B, gamma):
    return torch.exp(-gamma * ((A[:, None, :] - B[None, :, :]) ** 2).sum(-1))


@pytest.mark.parametrize("l,m,F", [(1037, 300, 17), (64, 64, 1), (130, 513, 32), (5, 1, 3)])
def test_rbf_f64_matches_fp64_reference(l, m, F):
    g = torch.Generator().manual_seed(l + m + F)
    A = torch.randn(l, F, generator=g, dtype=torch.float64)
    B = torch.randn(m, F, generator=g, dtype=torch.float64)
    gamma = 1.0 / F
    assert svc_lowrank.NATIVE_RBF and ops.has_ext()
    out = svc_lowrank._rbf(A.cuda(), B.cuda(), gamma).cpu()
    ref = _ref(A, B, gamma)
    assert out.shape == (l, m)
    assert torch.allclose(out, ref, rtol=1e-13, atol=1e-300)


def test_rbf_wide_features_fall_back_to_the_library_form():
    A = torch.randn(50, 40, dtype=torch.float64)
    B = torch.randn(20, 40, dtype=torch.float64)
    out = svc_lowrank._rbf(A.cuda(), B.cuda(), 0.02).cpu()
    assert torch.allclose(out, _ref(A, B, 0.02), rtol=1e-10, atol=1e-14)


def test_nystrom_map_native_matches_library_form(monkeypatch):
    g = torch.Generator().manual_seed(7)
    Z = torch.randn(3000, 17, generator=g, dtype=torch.float64).cuda()
    idx = torch.randperm(3000, generator=g)[:256].cuda()
    phis = []
    for native in (True, False):
        monkeypatch.setattr(svc_lowrank, "NATIVE_RBF", native)
        Phi, T = svc_lowrank.nystrom_map(Z, idx, 1.0 / 17)
        phis.append(Phi[:400])
    G0, G1 = phis[0] @ phis[0].T, phis[1] @ phis[1].T
    assert torch.allclose(G0, G1, rtol=1e-8, atol=1e-10)
