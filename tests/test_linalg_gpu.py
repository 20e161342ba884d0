"""Native single-workgroup SPD factor / solve (ops/csrc/linalg.hip) vs torch.linalg in f64: the
interior-point SVC's r × r Woodbury systems (equilibrated, jitter retries on the device)."""
import numpy as np
import pytest
import torch

from hfens import ops

pytestmark = pytest.mark.gpu


def _spd(r, cond_decades, seed):
    g = torch.Generator().manual_seed(seed)
    Q, _ = torch.linalg.qr(torch.randn(r, r, generator=g, dtype=torch.float64))
    ev = torch.logspace(0, cond_decades, r, dtype=torch.float64)
    S = (Q * ev) @ Q.T
    # badly scaled rows/columns, as I + ΦᵀD⁻¹Φ near the end of the interior-point solve
    dsc = torch.logspace(-4, 4, r, dtype=torch.float64)[torch.randperm(r, generator=g)]
    return dsc[:, None] * S * dsc[None, :]


@pytest.mark.parametrize("r", [1, 17, 33, 64, 65, 200, 512, 600, 1024])
def test_chol_spd_and_solve_match_torch(dev, r):
    E = ops.ext()
    S = _spd(r, 8, r).to(dev)
    L = torch.empty(r, r, dtype=torch.float64, device=dev)
    sc = torch.empty(r, dtype=torch.float64, device=dev)
    info = torch.full((1,), 99, dtype=torch.int32, device=dev)
    E.chol_spd(S.data_ptr(), r, L.data_ptr(), sc.data_ptr(), info.data_ptr(), ops.stream_ptr(dev))
    assert int(info) == 0
    # L is the Cholesky factor of the equilibrated matrix
    Ss = S * sc[:, None] * sc[None, :]
    assert torch.allclose(L @ L.T, Ss, atol=1e-10, rtol=0)
    assert torch.equal(torch.triu(L, 1), torch.zeros_like(L))
    for k in (1, 2, 3):
        B = torch.randn(r, k, dtype=torch.float64, device=dev)
        X = B.clone()
        E.chol_solve(L.data_ptr(), sc.data_ptr(), r, k, X.data_ptr(), ops.stream_ptr(dev))
        # the same factor through torch's triangular solves
        want = sc[:, None] * torch.cholesky_solve(sc[:, None] * B, L)
        assert float((X - want).abs().max() / want.abs().max()) < 1e-9
        # backward error on the equilibrated system (what the Woodbury step needs)
        Y = X / sc[:, None]
        res = (Ss @ Y - sc[:, None] * B).abs().max() / (Ss.abs().max() * Y.abs().max())
        assert float(res) < 1e-13, float(res)


def test_chol_spd_jitter_retry_on_semidefinite(dev):
    """A rank-deficient PSD matrix fails the plain factorisation; the kernel retries with jitter on
    the device and reports how many retries it took."""
    E = ops.ext()
    r = 96
    A = torch.randn(r, 40, dtype=torch.float64)
    S = (A @ A.T).to(dev)                   # rank 40
    L = torch.empty(r, r, dtype=torch.float64, device=dev)
    sc = torch.empty(r, dtype=torch.float64, device=dev)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    E.chol_spd(S.data_ptr(), r, L.data_ptr(), sc.data_ptr(), info.data_ptr(), ops.stream_ptr(dev))
    assert int(info) >= 1
    Ss = S * sc[:, None] * sc[None, :]
    assert torch.allclose(L @ L.T, Ss, atol=1e-5)


@pytest.mark.parametrize("n,r", [(1, 1), (37, 17), (1000, 128), (20011, 509), (70000, 512), (5000, 700)])
def test_wsyrk_f64_matches_torch(dev, monkeypatch, n, r):
    """Native f64-MFMA weighted SYRK (upper tiles, deterministic split-K) vs Φᵀ diag(d) Φ."""
    from hfens.models import svc_lowrank
    from hfens.models.svc_lowrank import _weighted_gram
    monkeypatch.setattr(svc_lowrank, "NATIVE_SYRK", True)
    g = torch.Generator(device=dev).manual_seed(n + r)
    Phi = torch.randn(n, r, generator=g, device=dev, dtype=torch.float64)
    d = torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 10 ** torch.randint(-6, 6, (n,), generator=g, device=dev)
    S = _weighted_gram(Phi, d)
    want = Phi.T @ (d[:, None] * Phi)
    assert torch.equal(S, S.T)
    err = float((S - want).abs().max() / want.abs().max())
    assert err < 1e-12, err
    assert torch.equal(S, _weighted_gram(Phi, d))          # deterministic


@pytest.mark.parametrize("n,r,k", [(1, 1, 1), (999, 17, 2), (100003, 509, 1), (4096, 512, 4), (3, 64, 3)])
def test_phi_gemv_matches_torch(dev, n, r, k):
    from hfens.models.svc_lowrank import _phi_mv
    g = torch.Generator(device=dev).manual_seed(n * 7 + r)
    Phi = torch.randn(n, r, generator=g, device=dev, dtype=torch.float64)
    W = torch.randn(r, k, generator=g, device=dev, dtype=torch.float64)
    Y = _phi_mv(Phi, W)
    want = Phi @ W
    assert float((Y - want).abs().max() / want.abs().max()) < 1e-13


@pytest.mark.parametrize("n,r,k", [(1, 1, 1), (999, 17, 2), (100003, 428, 1), (70001, 512, 4), (65, 300, 3)])
def test_f32_phi_passes_match_torch_f64(dev, n, r, k):
    """The IPM's skinny passes over the f32 copy of Φ (phi_gemv_f32: Φ W; phit_f32: Φᵀ V, split-K
    with an ordered partial sum) equal the f64 products of the same (f32-representable) Φ."""
    from hfens.models.svc_lowrank import _phi_mv, _phit
    g = torch.Generator(device=dev).manual_seed(n * 5 + r)
    P32 = torch.randn(n, r, generator=g, device=dev, dtype=torch.float32)
    Phi = P32.double()
    W = torch.randn(r, k, generator=g, device=dev, dtype=torch.float64)
    V = torch.randn(n, k, generator=g, device=dev, dtype=torch.float64)
    Y = _phi_mv(Phi, W, P32)
    want = Phi @ W
    assert float((Y - want).abs().max() / want.abs().max()) < 1e-13
    O = _phit(Phi, V, P32)
    want = Phi.T @ V
    assert float((O - want).abs().max() / want.abs().max()) < 1e-12
    assert torch.equal(O, _phit(Phi, V, P32))              # deterministic


def test_lowrank_svc_threaded_platt_cv_identical(dev, monkeypatch):
    """The Platt-CV interior-point solves on host threads / streams (svc_lowrank.IPM_THREADS), the
    final solve beside them, and two fits at a time (FIT_THREADS) give the same fitted SVCs as one
    solve at a time: the same kernels on the same inputs."""
    from hfens.io.synth import make_hf_cohort
    from hfens.models import svc_lowrank
    from hfens.models.svc import SVC
    X, y, _ = make_hf_cohort(6000, 17, seed=12, nan_frac=0.0)
    Z = torch.as_tensor(X, device=dev)
    Z = (Z - Z.mean(0)) / Z.std(0).clamp(min=1e-12)
    yt = torch.as_tensor(y, device=dev)
    out = {}
    for nt, nf in ((1, 1), (2, 1), (3, 2)):
        monkeypatch.setattr(svc_lowrank, "IPM_THREADS", nt)
        monkeypatch.setattr(svc_lowrank, "FIT_THREADS", nf)
        ss = [SVC(kernel="rbf", probability=True, class_weight="balanced", random_state=r) for r in range(3)]
        svc_lowrank.fit_svc_lowrank_batch(ss, [Z, Z[:5000], Z[1000:]], [yt, yt[:5000], yt[1000:]], n_landmarks=128)
        out[(nt, nf)] = ss
    for key in ((2, 1), (3, 2)):
        for a, b in zip(out[(1, 1)], out[key]):
            assert a._hs == b._hs, key                      # (intercept, Platt A, Platt B)
            assert torch.equal(a.dual_coef_, b.dual_coef_), key


def test_ipm_fused_step_and_scaled_rows_match_torch(dev):
    """The interior point's fused kernels (lowrank.hip ipm_max_step, scale_rows_f32) give the torch
    expressions they replace bit for bit: the step-length bound over the four (v, dv) pairs and
    diag(d)·Φ from the exact f32 copy."""
    from hfens import ops
    from hfens.models import svc_lowrank as sl
    g = torch.Generator(device=dev).manual_seed(5)
    n = 300_001
    vs = [torch.rand(n, generator=g, device=dev, dtype=torch.float64) + 1e-3 for _ in range(4)]
    ds = [torch.randn(n, generator=g, device=dev, dtype=torch.float64) for _ in range(4)]
    ref = torch.minimum(torch.minimum(sl._max_step(vs[0], ds[0]), sl._max_step(vs[1], -ds[1])),
                        torch.minimum(sl._max_step(vs[2], ds[2]), sl._max_step(vs[3], ds[3])))
    out = torch.ones((), dtype=torch.float64, device=dev)
    ops.ext().ipm_max_step(vs[0].data_ptr(), ds[0].data_ptr(), vs[1].data_ptr(), ds[1].data_ptr(), vs[2].data_ptr(),
                           ds[2].data_ptr(), vs[3].data_ptr(), ds[3].data_ptr(), 1.0, -1.0, 1.0, 1.0, n,
                           out.data_ptr(), ops.stream_ptr(dev))
    assert float(out) == float(ref)
    P32 = torch.randn(n, 428, generator=g, device=dev, dtype=torch.float32)
    d = torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 1e6
    got = sl._scaled_rows(P32.double(), d, P32)
    assert torch.equal(got, P32.double() * d[:, None])


def test_ipm_fused_direction_kernels_bit_identical(dev, monkeypatch):
    """The interior point with its fused direction / Gondzio kernels (lowrank.hip ipm_dirs,
    ipm_gondzio_rhs, ipm_gondzio_apply, ipm_select3: the same IEEE operations in the same order,
    contraction off) reproduces the torch-expression iterates bit for bit."""
    from hfens.models import svc_lowrank as sl
    g = torch.Generator(device=dev).manual_seed(11)
    n, r = 60_000, 96
    Phi = torch.randn(n, r, generator=g, device=dev, dtype=torch.float64).to(torch.float32).to(torch.float64)
    y = torch.where(torch.rand(n, generator=g, device=dev) < 0.3, -1.0, 1.0).to(torch.float64)
    c = torch.where(y > 0, 0.7, 2.1).to(torch.float64)
    out = {}
    for fused in (False, True):
        monkeypatch.setattr(sl, "_FUSED_OFF", not fused)
        a, rho, it = sl.ipm_svc_dual(Phi, y, c)
        out[fused] = (a.cpu(), rho, it)
    assert out[False][2] == out[True][2]
    assert out[False][1] == out[True][1]
    assert torch.equal(out[False][0], out[True][0])


@pytest.mark.parametrize("n,r", [(37, 16), (20011, 428), (70000, 512), (5000, 132)])
def test_wsyrk_f32_matches_f64(dev, monkeypatch, n, r):
    """The f32-input-MFMA weighted SYRK (lowrank.hip wsyrk_f32: Φ exact in f32, d ⊙ Φ rounded to f32,
    f32 sums over ≤ 256 rows folded into f64) against the f64 product of the same Φ: every entry
    within 1e-6 of the magnitude of its terms, symmetric, deterministic."""
    from hfens.models import svc_lowrank
    from hfens.models.svc_lowrank import _weighted_gram
    monkeypatch.setattr(svc_lowrank, "GRAM", "f32")
    g = torch.Generator(device=dev).manual_seed(3 * n + r)
    P32 = torch.randn(n, r, generator=g, device=dev, dtype=torch.float32)
    Phi = P32.double()
    d = torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 10 ** torch.randint(-6, 6, (n,), generator=g, device=dev)
    S = _weighted_gram(Phi, d, P32)
    want = Phi.T @ (d[:, None] * Phi)
    mag = Phi.abs().T @ (d[:, None] * Phi.abs())
    assert torch.equal(S, S.T)
    err = float(((S - want).abs() / mag).max())
    assert err < 1e-6, err
    assert torch.equal(S, _weighted_gram(Phi, d, P32))      # deterministic


@pytest.mark.parametrize("n,r", [(37, 16), (20011, 428), (70000, 512), (5000, 132), (3000, 2048)])
def test_wsyrk_f64x_matches_f64(dev, monkeypatch, n, r):
    """The native f64 weighted SYRK from the exact f32 copy of Φ (lowrank.hip wsyrk_f64x: 64 × 64
    upper tiles, f64 MFMA, split-K summed in group order) against torch's f64 product: every entry
    within 1e-13 of the magnitude of its terms (f64 sums in another order), symmetric, deterministic."""
    from hfens.models import svc_lowrank
    from hfens.models.svc_lowrank import _weighted_gram
    monkeypatch.setattr(svc_lowrank, "GRAM", "f64x")
    g = torch.Generator(device=dev).manual_seed(7 * n + r)
    P32 = torch.randn(n, r, generator=g, device=dev, dtype=torch.float32)
    Phi = P32.double()
    d = torch.rand(n, generator=g, device=dev, dtype=torch.float64) * 10 ** torch.randint(-6, 6, (n,), generator=g, device=dev)
    S = _weighted_gram(Phi, d, P32)
    want = Phi.T @ (d[:, None] * Phi)
    mag = Phi.abs().T @ (d[:, None] * Phi.abs())
    assert torch.equal(S, S.T)
    err = float(((S - want).abs() / mag).max())
    assert err < 1e-13, err
    assert torch.equal(S, _weighted_gram(Phi, d, P32))      # deterministic


def test_ipm_f32_gram_matches_f64_path(dev, monkeypatch):
    """The interior point with the f32-MFMA Gram in its Newton systems (opt-in) converges to the
    f64 path's optimum: same stopping test (f64 residuals), dual coefficients and ρ within 1e-6; the
    default native f64 Gram (wsyrk_f64x) follows the library f64 path to rounding."""
    from hfens.io.synth import make_hf_cohort
    from hfens.models import svc_lowrank
    X, y, _ = make_hf_cohort(30000, 17, seed=5, nan_frac=0.0)
    Z = torch.as_tensor(X, device=dev)
    Z = (Z - Z.mean(0)) / Z.std(0).clamp(min=1e-12)
    g = torch.Generator().manual_seed(1)
    idx = torch.randperm(Z.shape[0], generator=g)[:256].to(dev)
    # (the map as this test was calibrated on: the library-form RBF.  With the native one-pass RBF
    # (nystrom.hip, rounding ≈ 1e-16 apart) the opt-in f32-Gram mode stalls at the iteration cap on
    # this problem (80 vs 19 iterations) while the f64 paths agree — the f32 Newton systems'
    # ≈ 1e-7 errors make that mode's convergence to the 1e-8 tolerances a matter of luck; it stays
    # opt-in, profiles/r6_config3.md §4)
    monkeypatch.setattr(svc_lowrank, "NATIVE_RBF", False)
    Phi, _ = svc_lowrank.nystrom_map(Z, idx, 1.0 / 17)
    Phi = Phi.to(torch.float32).to(torch.float64)          # exactly f32, as fit_svc_lowrank_batch
    yv = torch.as_tensor(np.where(y > 0.5, -1.0, 1.0), device=dev)
    c = torch.where(yv > 0, 0.62, 2.5).to(torch.float64)
    out = {}
    for mode in ("f64", "f32", "f64x"):
        monkeypatch.setattr(svc_lowrank, "GRAM", mode)
        a, rho, it = svc_lowrank.ipm_svc_dual(Phi, yv, c)
        out[mode] = (a, rho, it)
    a64, rho64, it64 = out["f64"]
    ax, rhox, itx = out["f64x"]
    assert abs(itx - it64) <= 1, (itx, it64)
    w64, wx = Phi.T @ (yv * a64), Phi.T @ (yv * ax)
    assert float((wx - w64).abs().max() / w64.abs().max()) <= 1e-6
    assert abs(rhox - rho64) <= 1e-7, (rhox, rho64)
    a32, rho32, it32 = out["f32"]
    assert it32 <= it64 + 5, (it32, it64)
    # Q = diag(y) Φ Φᵀ diag(y) has rank ≤ 256 < l: the dual optimum α is not unique, the model is —
    # the primal w = Φᵀ y α, ρ (hence every decision value) and the dual objective
    # (both stop on the same f64 tests — duality gap < 1e-8, dual residual < 1e-8, or < 1e-5 once the
    # gap has converged — so they agree to those tolerances: measured 2.4e-6 relative on w)
    w64, w32 = Phi.T @ (yv * a64), Phi.T @ (yv * a32)
    assert float((w32 - w64).abs().max() / w64.abs().max()) <= 1e-5
    assert abs(rho32 - rho64) <= 1e-6, (rho32, rho64)
    obj = lambda a, w: float(0.5 * (w @ w) - a.sum())   # noqa: E731
    assert abs(obj(a32, w32) - obj(a64, w64)) <= 1e-8 * abs(obj(a64, w64))


@pytest.mark.parametrize("r", [1, 31, 96, 300, 509, 512])
def test_chol_spd_mw_bit_identical(dev, r):
    """The multi-workgroup blocked Cholesky (diagonal block / panel rows / MFMA trailing update as
    separate launches) computes every element with the one-workgroup kernel's operations in its
    order: L, the equilibration and info are bit-identical."""
    E = ops.ext()
    S = _spd(r, 8, r + 1).to(dev)
    out = []
    for mw in (False, True):
        L = torch.full((r, r), float("nan"), dtype=torch.float64, device=dev)
        sc = torch.empty(r, dtype=torch.float64, device=dev)
        info = torch.full((1,), 99, dtype=torch.int32, device=dev)
        if mw:
            work = torch.zeros(4, dtype=torch.int32, device=dev)
            PT = torch.empty(32 * r, dtype=torch.float64, device=dev)
            E.chol_spd_mw(S.data_ptr(), r, L.data_ptr(), sc.data_ptr(), info.data_ptr(), work.data_ptr(),
                          PT.data_ptr(), ops.stream_ptr(dev))
        else:
            E.chol_spd(S.data_ptr(), r, L.data_ptr(), sc.data_ptr(), info.data_ptr(), ops.stream_ptr(dev))
        out.append((L.cpu(), sc.cpu(), int(info)))
    assert out[0][2] == out[1][2] == 0
    assert torch.equal(out[0][1], out[1][1])
    assert torch.equal(out[0][0], out[1][0])


def test_chol_spd_mw_falls_back_on_semidefinite(dev):
    """A failed plain attempt hands over to the one-workgroup kernel's jitter ladder: the same factor
    and retry count as chol_spd."""
    E = ops.ext()
    r = 200
    A = torch.randn(r, 60, dtype=torch.float64, generator=torch.Generator().manual_seed(5))
    S = (A @ A.T).to(dev)
    res = []
    for mw in (False, True):
        L = torch.empty(r, r, dtype=torch.float64, device=dev)
        sc = torch.empty(r, dtype=torch.float64, device=dev)
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        if mw:
            work = torch.zeros(4, dtype=torch.int32, device=dev)
            PT = torch.empty(32 * r, dtype=torch.float64, device=dev)
            E.chol_spd_mw(S.data_ptr(), r, L.data_ptr(), sc.data_ptr(), info.data_ptr(), work.data_ptr(),
                          PT.data_ptr(), ops.stream_ptr(dev))
        else:
            E.chol_spd(S.data_ptr(), r, L.data_ptr(), sc.data_ptr(), info.data_ptr(), ops.stream_ptr(dev))
        res.append((L.cpu(), int(info)))
    assert res[0][1] >= 1 and res[0][1] == res[1][1]
    assert torch.equal(res[0][0], res[1][0])
