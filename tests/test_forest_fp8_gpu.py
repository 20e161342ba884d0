"""fp8 leaf-value GEMV on the MFMA (ops/csrc/forest_fp8.hip, BASELINE config 5) vs a PyTorch
reference of the same quantised operands, and the fp8 model vs the exact f64 ensemble."""
import numpy as np
import pytest
import torch

from hfens.io.synth import make_hf_cohort
from hfens.models.forest_infer import Fp8Forest
from hfens.models.gbdt import GradientBoostingClassifier
from hfens.models.hist_gbdt import fit_gbdt_batch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("depth,S,n", [(1, 5, 10007), (2, 3, 4099), (3, 2, 2053), (5, 1, 1500)])
def test_fp8_kernel_matches_reference(dev, depth, S, n):
    X, y, _ = make_hf_cohort(4000, 17, seed=61, nan_frac=0.0)
    X, y = torch.as_tensor(X), torch.as_tensor(y)
    ms = [GradientBoostingClassifier(n_estimators=40, max_depth=depth, subsample=0.8, random_state=s)
          for s in range(S)]
    fit_gbdt_batch(ms, X.to(dev), y.to(dev))
    Xt, _, _ = make_hf_cohort(n, 17, seed=62, nan_frac=0.0)
    bins = ms[0]._bin_mapper.transform(torch.as_tensor(Xt).to(dev))
    f8 = Fp8Forest(ms)
    got = f8.raw(bins).double().cpu()
    ref = f8.reference_raw(bins.cpu())
    # identical quantised operands; only the f32 accumulation order differs
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-5)
    # two-term fp8 vs the unquantised binned model
    exact = f8.reference_raw(bins.cpu(), exact=True)
    assert float((got - exact).abs().max()) < 5e-3
    # without bagging, on the training rows the binned model IS the threshold model: every row of a
    # node lies in a non-empty bin of that node, so "bin ≤ blo" and "x ≤ threshold" agree (rows in
    # a bin the node's bag left empty — out-of-bag rows, unseen values — may not: the fp8 forest
    # implements the binned semantics, see Fp8Forest.reference_raw)
    full = [GradientBoostingClassifier(n_estimators=40, max_depth=depth, random_state=s) for s in range(S)]
    fit_gbdt_batch(full, X.to(dev), y.to(dev))
    bt = full[0]._bin_mapper.transform(X.to(dev))
    thr = torch.stack([m.decision_function(X.to(dev)).double().cpu() for m in full])
    assert float((Fp8Forest(full).raw(bt).double().cpu() - thr).abs().max()) < 5e-3


def test_fp8_deep_ensemble_auroc_guard(dev):
    """1000 stumps × 5 seeds: fp8 two-term leaf values keep held-out AUROC within 0.001 of the
    fp32 folded-table inference (BASELINE config 5 guard)."""
    from hfens.io.synth import make_hf_cohort_device
    from hfens.models.forest_infer import ensemble_raw_binned, stump_bin_tables
    from hfens.utils import metrics
    X, y = make_hf_cohort_device(60000, 40, seed=2020, rows=(0, 60000), device=dev)
    Xh, yh = make_hf_cohort_device(20000, 40, seed=2021, rows=(0, 20000), device=dev)
    ms = [GradientBoostingClassifier(n_estimators=1000, max_depth=1, subsample=0.8, random_state=s) for s in range(5)]
    fit_gbdt_batch(ms, X, y)
    bins = ms[0]._bin_mapper.transform(Xh)
    T, init = stump_bin_tables(ms)
    raw32 = ensemble_raw_binned(T, init, bins)
    raw8 = Fp8Forest(ms).raw(bins)
    p32 = torch.sigmoid(raw32.double()).mean(0)
    p8 = torch.sigmoid(raw8.double()).mean(0)
    a32 = metrics.roc_auc(yh.double(), p32)
    a8 = metrics.roc_auc(yh.double(), p8)
    assert abs(a8 - a32) <= 1e-3
    assert float((raw8 - raw32).abs().max()) < 2e-2
