"""Host-side bookkeeping of the working-set SMO (models/smo.py) that needs no GPU."""
import numpy as np
import pytest


@pytest.mark.parametrize("l,npos", [(10000, 2300), (8000, 1841), (6400, 3200), (4096, 5), (4500, 4000)])
def test_cascade_parts_partition_the_problem(l, npos):
    """smo.cascade_parts: disjoint parts covering every point once, each class-stratified (its
    positives first, as a problem's layout requires) — so the concatenated part solutions are a
    feasible point of the full problem (same C, Σ yα = 0 per part)."""
    from hfens.models import smo
    p = smo._Prob(0, -1, np.arange(l), npos, 1.0, 1.0, 0.1)
    parts = smo.cascade_parts(p)
    P = smo.cascade_split(l, npos)
    assert len(parts) == P
    if P == 0:
        return
    allpos = np.concatenate(parts)
    assert np.array_equal(np.sort(allpos), np.arange(l))
    for pos in parts:
        cp = int((pos < npos).sum())
        assert np.all(pos[:cp] < npos) and np.all(pos[cp:] >= npos)
        assert abs(cp - npos / P) <= 1 and abs((pos.shape[0] - cp) - (l - npos) / P) <= 1
