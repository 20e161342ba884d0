"""Numerics of the inference HIP kernels vs the plain-PyTorch fp64 references."""
import numpy as np
import pytest
import torch

from hfens import ops
from hfens.ops import reference as ref
from hfens.io.checkpoint import load_checkpoint
from hfens.cli.predict_hf import PATIENT_PARAMS

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,m,F", [(1, 434, 17), (1000, 434, 17), (777, 100, 40), (64, 33, 3), (300, 5000, 17), (200, 3000, 40)])
def test_rbf_decision(dev, n, m, F):
    g = torch.Generator().manual_seed(n + m + F)
    z = torch.randn(n, F, generator=g, dtype=torch.float64)
    sv = torch.randn(m, F, generator=g, dtype=torch.float64)
    coef = torch.randn(m, generator=g, dtype=torch.float64)
    gamma = 1.0 / F
    want = ref.rbf_decision(z, sv, coef, gamma, 0.25)
    got = ops.rbf_decision(z.to(dev), sv.to(dev), coef.to(dev), gamma, 0.25).cpu().double()
    scale = coef.abs().sum().item()
    assert torch.allclose(got, want, atol=2e-6 * scale, rtol=0)


def test_svc_proba1(dev):
    dec = torch.linspace(-8, 8, 4097, dtype=torch.float64)
    want = ref.svc_proba1(dec, -1.25857732, -1.18972403)
    got = ops.svc_proba1(dec.to(dev), -1.25857732, -1.18972403).cpu().double()
    assert torch.allclose(got, want, atol=1e-6)


def _random_forest(T, depth, F, seed):
    rng = np.random.default_rng(seed)
    K = 2 ** (depth + 1) - 1
    feat = np.full((T, K), -2)
    thr = np.full((T, K), -2.0)
    left = np.full((T, K), -1)
    right = np.full((T, K), -1)
    val = rng.normal(size=(T, K))
    for t in range(T):
        for i in range(2 ** depth - 1):
            feat[t, i] = rng.integers(0, F)
            thr[t, i] = rng.normal()
            left[t, i] = 2 * i + 1
            right[t, i] = 2 * i + 2
    return [torch.as_tensor(a) for a in (feat, thr, left, right, val)]


@pytest.mark.parametrize("T,depth,F", [(100, 1, 17), (50, 4, 40)])
def test_forest_raw(dev, T, depth, F):
    feat, thr, left, right, val = _random_forest(T, depth, F, T + depth)
    x = torch.randn(2000, F, dtype=torch.float64)
    want = ref.tree_raw(x, feat, thr, left, right, val, -1.3, 0.1)
    got = ops.tree_raw(x.to(dev), feat, thr, left, right, val, -1.3, 0.1).cpu().double()
    assert torch.allclose(got, want, atol=1e-5)


def test_checkpoint_stack_on_gpu(dev, ckpt_path):
    clf_cpu = load_checkpoint(ckpt_path)
    clf_gpu = load_checkpoint(ckpt_path, device=dev)
    rng = np.random.default_rng(1)
    X = rng.integers(0, 2, size=(5000, 17)).astype(np.float64)
    X[:, 6] += 1
    X[:, 13] = rng.normal(18.6, 4.4, 5000).round()
    X[:, 15] = rng.integers(0, 5, 5000)
    X[:, 16] = rng.normal(63, 5, 5000).round()
    X[0] = list(PATIENT_PARAMS.values())
    Xt = torch.as_tensor(X)
    want = clf_cpu.predict_proba(Xt)[:, 1]
    got = clf_gpu.predict_proba(Xt.to(dev))[:, 1].cpu()
    assert torch.allclose(got, want, atol=2e-6)
    assert f"{100 * float(got[0]):.2f}" == "27.09"
