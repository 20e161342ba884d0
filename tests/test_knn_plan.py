"""The native KNN work-list planner (ops/csrc/host.hip knn_plan_host) against the numpy planning it
replaced (models/imputer.py): same receivers, slot columns, cell order and flat slot indices."""
import numpy as np
import pytest

from hfens import ops

pytestmark = pytest.mark.skipif(not ops.has_ext(), reason="needs the built extension")


def _numpy_plan(bits, F, slots):
    rows = np.nonzero(bits)[0]
    if rows.size == 0:
        return rows, None
    Rm = ((bits[rows, None] >> np.arange(F, dtype=np.uint64)) & np.uint64(1)).astype(bool)
    rl, cc = np.nonzero(Rm)
    nm = Rm.sum(1)
    start = np.concatenate([[0], np.cumsum(nm)[:-1]])
    kk = np.arange(rl.shape[0]) - start[rl]
    nslot = -(-int(nm.max()) // slots) * slots
    slot_all = np.full((rows.shape[0], nslot), -1, dtype=np.int64)
    slot_all[rl, kk] = cc
    return rows, (bits[rows].view(np.int64), slot_all, rl * nslot + kk, rows[rl], cc, nslot)


@pytest.mark.parametrize("n,F,p", [(1000, 40, 0.02), (500, 64, 0.3), (300, 17, 0.0), (257, 9, 0.9)])
def test_knn_plan_host_matches_numpy(n, F, p):
    rng = np.random.default_rng(n + F)
    miss = rng.random((n, F)) < p
    bits = (miss.astype(np.uint64) << np.arange(F, dtype=np.uint64)).sum(1).astype(np.uint64)
    nslot_max = -(-F // 8) * 8
    cap = 2 * n + n * nslot_max + 3 * n * F
    out = np.zeros(cap, dtype=np.int64)
    dims = np.zeros(4, dtype=np.int64)
    ops.ext().knn_plan_host(bits.ctypes.data, n, F, 8, out.ctypes.data, cap, dims.ctypes.data)
    assert int(dims[3]) == 0
    rows, ref = _numpy_plan(bits, F, 8)
    nr, nc, nslot = (int(v) for v in dims[:3])
    # a counting call (cap 0) gives the same sizes and writes nothing
    d0 = np.zeros(4, dtype=np.int64)
    ops.ext().knn_plan_host(bits.ctypes.data, n, F, 8, 0, 0, d0.ctypes.data)
    assert d0[:3].tolist() == dims[:3].tolist() and (int(d0[3]) == -1 or nr == 0)
    assert nr == rows.shape[0]
    if nr == 0:
        return
    rb, slot_all, flat, ri, ci, nslot_ref = ref
    assert nslot == nslot_ref and nc == ci.shape[0]
    o = np.cumsum([0, nr, nr, nr * nslot, nc, nc, nc])
    assert np.array_equal(out[o[0]:o[1]], rows)
    assert np.array_equal(out[o[1]:o[2]], rb)
    assert np.array_equal(out[o[2]:o[3]].reshape(nr, nslot), slot_all)
    assert np.array_equal(out[o[3]:o[4]], flat)
    assert np.array_equal(out[o[4]:o[5]], ri)
    assert np.array_equal(out[o[5]:o[6]], ci)
