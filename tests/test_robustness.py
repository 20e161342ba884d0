"""Robustness subsystems: fail-fast numeric guards, host-code
sanitizer self-test, and bitwise run-to-run determinism of the device training path."""
import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

from hfens.models.gbdt import GradientBoostingClassifier
from hfens.models.linear import LogisticRegression
from hfens.utils.guards import NonFiniteError

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_guards_reject_nonfinite_and_bad_labels():
    X = torch.randn(50, 4, dtype=torch.float64)
    y = (torch.arange(50) % 2).to(torch.float64)
    Xbad = X.clone()
    Xbad[3, 1] = float("inf")
    with pytest.raises(NonFiniteError):
        GradientBoostingClassifier(n_estimators=2).fit(Xbad, y)
    with pytest.raises(NonFiniteError):
        LogisticRegression(penalty="l1", solver="liblinear").fit(Xbad, y)
    with pytest.raises(ValueError):
        GradientBoostingClassifier(n_estimators=2).fit(X, y * 2)


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_host_code_asan_ubsan_selftest():
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "host_asan_selftest.sh")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_selftest: ok" in r.stdout


@pytest.mark.gpu
def test_device_training_is_bitwise_deterministic(dev):
    from hfens.io.synth import make_dev_select
    from hfens.pipeline import develop
    Xd, yd, Xs, ys, names = make_dev_select(3000, 30, seed=11)
    t = [torch.as_tensor(a, device=dev) for a in (Xd, yd, Xs, ys)]
    a = develop(*t, names, device=dev)
    b = develop(*t, names, device=dev)
    assert np.array_equal(a.selected, b.selected)
    assert torch.equal(a.proba_sel, b.proba_sel)
    assert torch.equal(a.model.final_estimator_.coef_, b.model.final_estimator_.coef_)
