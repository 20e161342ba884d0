"""SVC.set_platt (finish_svc_batch installs the Platt pair after a set_fitted that ran before the
pair was read back) leaves the same model as set_fitted with the pair (CPU)."""
import torch

from hfens.models.svc import SVC


def _kw():
    return dict(support=torch.tensor([0, 3, 5]), support_vectors=torch.linspace(-1, 1, 12, dtype=torch.float64).reshape(3, 4),
                n_support=[1, 2], dual_coef_libsvm=torch.tensor([0.5, -0.25, -0.25], dtype=torch.float64),
                rho=0.125, gamma=0.3, class_weight=torch.tensor([1.0, 2.0]), shape_fit=(10, 4), n_features=4)


def test_set_platt_matches_set_fitted():
    a = SVC(probability=True).set_fitted(probA=-1.5, probB=0.25, **_kw())
    b = SVC(probability=True).set_fitted(probA=0.0, probB=0.0, **_kw())
    b.set_platt(-1.5, 0.25)
    assert a._hs == b._hs
    assert torch.equal(a._probA, b._probA) and torch.equal(a._probB, b._probB)
    X = torch.randn(7, 4, dtype=torch.float64)
    assert torch.equal(a.predict_proba(X), b.predict_proba(X))
    c = SVC(probability=True).set_fitted(probA=0.0, probB=0.0, **_kw())
    c.set_platt(-1.5, 0.25, torch.tensor([-1.5, 0.25], dtype=torch.float64))
    assert torch.equal(a.predict_proba(X), c.predict_proba(X))
