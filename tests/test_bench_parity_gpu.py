"""Bench-shape parity (BASELINE.md target): the headline configuration — 10k development rows
× 40 candidate features, 2 % NaN, held-out independent draw (``bench.py``'s exact data) — run
through the reference pipeline on the installed scikit-learn 1.7.2 and through ``develop()`` on
the MI355X; held-out AUROC must agree within 0.005 (reference ``train_ensemble_public.py:37-64``)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_bench_shape_auroc_matches_sklearn(dev):
    from hfens.io.synth import make_hf_cohort
    from hfens.pipeline import develop
    from test_pipeline import _sklearn_reference
    Xd, yd, names = make_hf_cohort(10000, 40, seed=2020, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(10000, 40, seed=2021, nan_frac=0.02)
    res = develop(torch.as_tensor(Xd, device=dev), torch.as_tensor(yd, device=dev),
                  torch.as_tensor(Xs, device=dev), torch.as_tensor(ys, device=dev), names, device=dev)
    mask, p, auc = _sklearn_reference(np.array(Xd), np.asarray(yd), np.array(Xs), np.asarray(ys))
    assert np.array_equal(res.selected, mask)
    assert abs(res.scores["auroc"] - auc) < 0.005
    ours = res.proba_sel.double().cpu().numpy()
    assert np.corrcoef(ours, p)[0, 1] > 0.99
