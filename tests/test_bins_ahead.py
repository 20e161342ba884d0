"""Pieces of the host-synchronisation-free stacking fit that run on the CPU: the host-array bin fit
and the column-subset bin map (pipeline.develop bins every candidate column under the LassoCV path,
the GBC keeps the selected ones), and the deferred guard collector."""
import numpy as np
import pytest
import torch

from hfens.io.synth import make_hf_cohort
from hfens.models.binning import fit_bins, fit_bins_host
from hfens.utils.guards import Deferred, NonFiniteError, binary_flag, finite_flag


def _same(a, b):
    assert np.array_equal(a.nb_host, b.nb_host)
    assert torch.equal(a.nbins.cpu(), b.nbins.cpu())
    assert torch.equal(a.lo_val.cpu(), b.lo_val.cpu())
    assert torch.equal(a.hi_val.cpu(), b.hi_val.cpu())
    assert torch.equal(a.edges.cpu(), b.edges.cpu())
    assert len(a.uppers) == len(b.uppers)
    for u, v in zip(a.uppers, b.uppers):
        assert torch.equal(u.cpu(), v.cpu())


@pytest.mark.parametrize("max_bins", [256, 32])
def test_fit_bins_host_array_equals_fit_bins(max_bins):
    X, _, _ = make_hf_cohort(3000, 40, seed=5, nan_frac=0.0)
    X[:, 7] = np.random.default_rng(1).normal(size=3000)        # > 256 distinct: quantile groups
    Xt = torch.as_tensor(X)
    _same(fit_bins(Xt, max_bins), fit_bins_host(Xt.to(torch.float32).numpy(), max_bins, "cpu"))


def test_bin_map_select_equals_fit_on_columns():
    X, _, _ = make_hf_cohort(2500, 40, seed=6, nan_frac=0.0)
    X[:, 3] = np.random.default_rng(2).normal(size=2500)
    Xt = torch.as_tensor(X)
    cols = np.array([0, 3, 4, 9, 17, 22, 39])
    full = fit_bins_host(Xt.to(torch.float32).numpy(), 256, "cpu")
    _same(full.select(cols), fit_bins(Xt[:, torch.as_tensor(cols)], 256))
    sub = full.select(cols)
    assert torch.equal(sub.transform(Xt[:, torch.as_tensor(cols)]),
                       fit_bins(Xt[:, torch.as_tensor(cols)], 256).transform(Xt[:, torch.as_tensor(cols)]))


def test_deferred_guards_raise_and_call_fallbacks():
    d = Deferred()
    d.flag(finite_flag(torch.ones(3)), "finite", "a")
    d.flag(binary_flag(torch.tensor([0.0, 1.0])), "binary", "b")
    hit = []
    d.word(torch.tensor([0], dtype=torch.int32), lambda v: hit.append(v))
    d.resolve()
    assert hit == [] and len(d) == 0
    d.word(torch.tensor([3], dtype=torch.int32), lambda v: hit.append(v))
    d.flag(finite_flag(torch.tensor([1.0, float("nan")])), "finite", "leaf values")
    with pytest.raises(NonFiniteError, match="leaf values"):
        d.resolve()
    assert hit == [3]
    d.flag(binary_flag(torch.tensor([0.0, 2.0])), "binary", "labels")
    with pytest.raises(ValueError, match="labels"):
        d.resolve()
