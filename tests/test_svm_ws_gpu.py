"""Working-set decomposition SMO (svm_ws.hip) vs libsvm (through sklearn): the solution must meet
libsvm's KKT stopping rule, reach the same dual objective to O(eps), and give the same model."""
import numpy as np
import pytest
import torch

from hfens.models import smo
from hfens.models.svc import SVC

pytestmark = pytest.mark.gpu


def _data(n, F, seed):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, F, generator=g, dtype=torch.float64)
    w = torch.randn(F, generator=g, dtype=torch.float64)
    logit = X @ w / F ** 0.5 + 0.5 * torch.randn(n, generator=g, dtype=torch.float64) - 1.0
    y = (logit > 0).to(torch.float64)
    return X, y


def _dual(Z, y_pm, coef_sv, sv_idx, gamma):
    Zs = Z[sv_idx]
    d2 = ((Zs[:, None, :] - Zs[None, :, :]) ** 2).sum(-1)
    K = np.exp(-gamma * d2)
    a = np.abs(coef_sv)
    return 0.5 * coef_sv @ K @ coef_sv - a.sum()


@pytest.mark.parametrize("n,F,kc", [(1500, 17, "auto"), (6000, 17, "auto"), (4000, 40, "auto"), (6000, 17, "1"),
                                    (3000, 24, "1")])
def test_ws_solver_matches_libsvm(dev, monkeypatch, n, F, kc):
    """kc = "1": the K-cached q = 256 rounds (svm_ws.hip ws_kc_round_kernel) forced on a problem the
    q = 1024 solver would take."""
    from sklearn.svm import SVC as SK
    monkeypatch.setattr(smo, "SOLVER", "ws")
    monkeypatch.setattr(smo, "WS_KC", kc)
    X, y = _data(n, F, n + F)
    Z = ((X - X.mean(0)) / X.std(0, unbiased=False)).numpy()
    sk = SK(class_weight="balanced", probability=True, random_state=2020).fit(Z, y.numpy())
    m = SVC(class_weight="balanced", probability=True, random_state=2020)
    m.fit(torch.as_tensor(Z).to(dev), y.to(dev))
    st = smo.LAST_WS_STATS
    assert (st["gap"] < 1e-3).all(), st["gap"]          # libsvm's stopping rule, over all points
    gamma = 1.0 / (F * Z.var())
    ours = _dual(Z, None, m._dual_coef_[0].cpu().numpy(), m.support_.cpu().numpy(), gamma)
    theirs = _dual(Z, None, sk.dual_coef_[0], sk.support_, gamma)
    assert abs(ours - theirs) <= 1e-3 * abs(theirs)
    d = m.decision_function(torch.as_tensor(Z).to(dev)).cpu().numpy()
    assert np.abs(d - sk.decision_function(Z)).max() < 2e-2
    p = m.predict_proba(torch.as_tensor(Z).to(dev))[:, 1].cpu().numpy()
    assert np.abs(p - sk.predict_proba(Z)[:, 1]).max() < 1e-2
    assert abs(int(m._n_support.sum()) - int(sk.n_support_.sum())) <= 0.02 * n


def test_ws_and_exact_solvers_agree(dev, monkeypatch):
    X, y = _data(3000, 17, 5)
    Z = ((X - X.mean(0)) / X.std(0, unbiased=False)).to(dev)
    out = {}
    for solver in ("exact", "ws"):
        monkeypatch.setattr(smo, "SOLVER", solver)
        m = SVC(class_weight="balanced", probability=True, random_state=2020).fit(Z, y.to(dev))
        out[solver] = m.predict_proba(Z)[:, 1].cpu()
    assert (out["exact"] - out["ws"]).abs().max() < 1e-2


def test_ws_bench_scale_meets_libsvm_tolerance(dev, monkeypatch):
    """The headline's problem size (10k points, 17 features, balanced weights): the working-set
    solver (q = 256 K-cached, or q = 1024; half reuse) reaches libsvm's stopping rule, its dual
    objective matches libsvm's to O(eps) and its decision values match sklearn's to the solvers'
    tolerance (both stop at m(α) − M(α) < 1e-3, so they agree to O(1e-3), not bit for bit)."""
    from sklearn.svm import SVC as SK
    monkeypatch.setattr(smo, "SOLVER", "auto")
    X, y = _data(10000, 17, 77)
    Z = ((X - X.mean(0)) / X.std(0, unbiased=False)).numpy()
    m = SVC(class_weight="balanced", random_state=2020)
    m.fit(torch.as_tensor(Z).to(dev), y.to(dev))
    st = smo.LAST_WS_STATS
    assert smo.LAST_SMO_INFO["solver"] == "ws" and st["q"] == smo.ws_q(17, 10000)
    assert (st["gap"] < 1e-3).all(), st["gap"]
    assert int(st["outer"].max()) <= (400 if smo.ws_kc(17, 10000) else 120), st["outer"]
    sk = SK(class_weight="balanced", random_state=2020).fit(Z, y.numpy())
    gamma = 1.0 / (17 * Z.var())
    ours = _dual(Z, None, m._dual_coef_[0].cpu().numpy(), m.support_.cpu().numpy(), gamma)
    theirs = _dual(Z, None, sk.dual_coef_[0], sk.support_, gamma)
    assert abs(ours - theirs) <= 1e-3 * abs(theirs)
    d = m.decision_function(torch.as_tensor(Z).to(dev)).cpu().numpy()
    dd = np.abs(d - sk.decision_function(Z))
    assert np.median(dd) < 1e-3 and dd.max() < 1e-2, (np.median(dd), dd.max())
    assert (np.sign(d) == np.sign(sk.decision_function(Z))).mean() > 0.999


def test_ws_unconverged_batch_is_resolved_synchronously(dev, monkeypatch):
    """The working-set rounds are enqueued without host checks (WS_ROUNDS_AHEAD); a batch that has
    not converged after them is re-solved with host-checked rounds by finish_svc_batch — the same
    rounds in the same order, so the same model bit for bit."""
    import warnings
    X, y = _data(6000, 17, 31)
    Z = ((X - X.mean(0)) / X.std(0, unbiased=False)).to(dev)
    monkeypatch.setattr(smo, "SOLVER", "ws")
    ref = SVC(class_weight="balanced", probability=True, random_state=2020).fit(Z, y.to(dev))
    assert "ws_resolve" not in smo.LAST_SMO_INFO
    monkeypatch.setattr(smo, "WS_ROUNDS_AHEAD", 2)
    monkeypatch.setattr(smo, "WS_SEEDED_AHEAD", 2)
    monkeypatch.setattr(smo, "WS_KC_ROUNDS_AHEAD", 2)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        m = SVC(class_weight="balanced", probability=True, random_state=2020).fit(Z, y.to(dev))
    assert smo.LAST_SMO_INFO.get("ws_resolve") and any("host-checked" in str(x.message) for x in w)
    assert torch.equal(m.support_.cpu(), ref.support_.cpu())
    assert torch.equal(m._dual_coef_.cpu(), ref._dual_coef_.cpu())
    assert m._probA.item() == ref._probA.item() and m._probB.item() == ref._probB.item()


@pytest.mark.parametrize("coop", [False, True])
@pytest.mark.parametrize("ls", [[1500, 9000], [20000, 700]])
def test_platt_kernel_matches_host_sigmoid_train(dev, ls, coop):
    """platt_batch (svm.hip): each fit's decision values assembled in the kernel from f32 partials
    (d = −(Σ_s part[row][s] − ρ_k), per-fold constants, 0 for unmapped positions), then libsvm's
    sigmoid_train with one pass per Newton trial — against the host sigmoid_train on the same
    values summed in f64.  Fits ≤ 16k points keep the values in registers, larger ones in the
    global scratch (both paths covered); ``coop``: the ≤ 16k fits split over 8 workgroups per fit
    (platt_coop_kernel)."""
    from hfens import ops
    E = ops.ext()
    rng = np.random.default_rng(7)
    S = 3
    rows = sum(ls)
    part = rng.normal(0, 0.4, (rows, S)).astype(np.float32)
    nprob = 4
    rowk = rng.integers(0, nprob, rows).astype(np.int32)
    rho = rng.normal(0, 0.2, nprob)
    consts = np.array([0.0, 0.7, -1.3])
    maps, arr, off, r0 = [], np.zeros(len(ls), smo._PLATT_DT), 0, 0
    n0s = []
    for k, l in enumerate(ls):
        sm = rng.permutation(np.arange(r0, r0 + l, dtype=np.int32))
        sm[:5] = -2            # a degenerate fold's constant
        sm[5:7] = -3
        sm[7] = -1             # no fold: 0.0
        n0 = int(l * 0.3)
        arr[k] = (off, l, n0)
        maps.append(sm)
        n0s.append(n0)
        off += l
        r0 += l
    srcmap = np.concatenate(maps)
    d = lambda t: torch.as_tensor(t).to(dev)   # noqa: E731
    part_d, rowk_d, rho_d, c_d, map_d, pdev = (d(part), d(rowk), d(rho), d(consts), d(srcmap),
                                               d(arr.view(np.uint8)))
    dscr = torch.empty(off, dtype=torch.float64, device=dev)
    AB = torch.empty(2 * len(ls), dtype=torch.float64, device=dev)
    cbar = torch.zeros(len(ls), dtype=torch.int32, device=dev)
    cpart = torch.empty(len(ls) * 2 * 8 * 6, dtype=torch.float64, device=dev)
    E.platt_batch(pdev.data_ptr(), len(ls), part_d.data_ptr(), S, rowk_d.data_ptr(), rho_d.data_ptr(),
                  c_d.data_ptr(), map_d.data_ptr(), dscr.data_ptr(), AB.data_ptr(),
                  cbar.data_ptr() if coop else 0, cpart.data_ptr() if coop else 0, ops.stream_ptr(dev))
    got = AB.cpu().numpy()
    for k, sm in enumerate(maps):
        dec = np.where(sm >= 0, -(part.astype(np.float64)[np.maximum(sm, 0)].sum(1) - rho[rowk[np.maximum(sm, 0)]]),
                       consts[np.where(sm < 0, -1 - sm, 0)])
        lab = np.where(np.arange(sm.size) < n0s[k], 1.0, -1.0)
        A, B = smo._sigmoid_train_host(dec, lab)
        assert got[2 * k] == pytest.approx(A, rel=1e-9, abs=1e-12), (k, got[2 * k], A)
        assert got[2 * k + 1] == pytest.approx(B, rel=1e-9, abs=1e-12), (k, got[2 * k + 1], B)


def test_ws_seed_gradient_matches_f64(dev):
    """ws_seed (svm_ws.hip ws_seed_kernel): α ← a feasible seed, G = −1 + y ∘ K (y ∘ α) over the
    nonzero α — against the same expression in f64 on the host (f32 kernel values: ≤ 1e-4)."""
    from hfens import ops
    E = ops.ext()
    F = 17
    ls, nposs = [3000, 1700], [1300, 900]
    g = torch.Generator().manual_seed(5)
    Zs = [torch.randn(l, F, generator=g, dtype=torch.float32) for l in ls]
    gamma = 1.0 / F
    arr = np.zeros(2, smo._WS_DT)
    off = 0
    seeds = []
    for k, (l, npos) in enumerate(zip(ls, nposs)):
        arr[k] = (off, off, l, npos, 0.9, 1.3, -gamma * 1.4426950408889634, 0)
        a = torch.rand(l, generator=g, dtype=torch.float64) * 0.9
        a[torch.rand(l, generator=g) < 0.5] = 0.0       # about half the points are not support vectors
        a[npos:] = a[npos:].clamp(max=1.3)
        seeds.append(a)
        off += l
    n = off
    zcat = torch.cat(Zs).to(dev).contiguous()
    aseed = torch.cat(seeds).to(dev)
    pdev = smo._dev_struct(arr, dev)
    zn = torch.empty(n, dtype=torch.float32, device=dev)
    alpha = torch.empty(n, dtype=torch.float64, device=dev)
    G = torch.empty(n, dtype=torch.float64, device=dev)
    states = torch.zeros(2 * smo._WS_STATE_BYTES // 4, dtype=torch.int32, device=dev)
    keys = torch.zeros(2 * n, dtype=torch.int32, device=dev)
    hist = torch.zeros(1, dtype=torch.int32, device=dev)
    gkey = torch.zeros(4, dtype=torch.int64, device=dev)
    s = ops.stream_ptr(dev)
    E.ws_init(pdev.data_ptr(), 2, max(ls), zcat.data_ptr(), F, zn.data_ptr(), alpha.data_ptr(), G.data_ptr(),
              states.data_ptr(), keys.data_ptr(), n, hist.data_ptr(), gkey.data_ptr(), s)
    E.ws_seed(pdev.data_ptr(), 2, max(ls), zcat.data_ptr(), F, zn.data_ptr(), aseed.data_ptr(), alpha.data_ptr(),
              G.data_ptr(), keys.data_ptr(), n, gkey.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(alpha.cpu(), aseed.cpu())
    off = 0
    for k, (l, npos) in enumerate(zip(ls, nposs)):
        Z = Zs[k].double()
        y = torch.ones(l, dtype=torch.float64)
        y[npos:] = -1.0
        K = torch.exp(-gamma * torch.cdist(Z, Z) ** 2)
        ref = -1.0 + y * (K @ (y * seeds[k]))
        got = G[off:off + l].cpu()
        assert (got - ref).abs().max() <= 1e-4 * max(1.0, float(ref.abs().max())), (got - ref).abs().max()
        off += l


def test_ws_cascade_seed_matches_cold_solve(dev, monkeypatch):
    """The cascade warm start (smo._cascade_seed: disjoint class-stratified parts with the same C,
    solved loosely, then the full problem from their concatenated α) reaches the same stopping rule
    and the same model to the solver's tolerance as the cold solve, in fewer pairs."""
    X, y = _data(10000, 17, 77)
    Z = ((X - X.mean(0)) / X.std(0, unbiased=False)).to(dev)
    monkeypatch.setattr(smo, "SOLVER", "auto")
    out = {}
    for cascade in (False, True):
        monkeypatch.setattr(smo, "CASCADE", cascade)
        m = SVC(class_weight="balanced", random_state=2020).fit(Z, y.to(dev))
        st = smo.LAST_WS_STATS
        assert (st["gap"] < 1e-3).all(), st["gap"]
        gamma = 1.0 / (17 * float(Z.var(unbiased=False)))
        out[cascade] = dict(d=m.decision_function(Z).cpu().numpy(), pairs=int(st["inner"].max()),
                            obj=_dual(Z.cpu().numpy(), None, m._dual_coef_[0].cpu().numpy(),
                                      m.support_.cpu().numpy(), gamma))
    dd = np.abs(out[True]["d"] - out[False]["d"])
    assert np.median(dd) < 1e-3 and dd.max() < 1e-2, (np.median(dd), dd.max())
    assert abs(out[True]["obj"] - out[False]["obj"]) <= 1e-3 * abs(out[False]["obj"])
    assert out[True]["pairs"] < 0.8 * out[False]["pairs"], (out[True]["pairs"], out[False]["pairs"])


def test_cascade_where_matches_host_parts(dev):
    """stackdev.hip cascade_where (the parts' point lists, built on the device) equals the host
    mirror smo.cascade_parts for parents of assorted sizes and class balances."""
    from hfens import ops
    parents = [(10000, 2300), (8000, 1841), (6400, 1500), (4096, 7), (5000, 4990)]
    tab, ref, aoff, start = [], [], 0, 0
    for l, npos in parents:
        p = smo._Prob(0, -1, np.arange(l), npos, 1.0, 1.0, 0.1)
        P = smo.cascade_split(l, npos)
        for j, pos in enumerate(smo.cascade_parts(p)):
            cp = int((pos < npos).sum())
            tab.append((start, pos.shape[0], aoff, P, j, npos, cp))
            ref.append(aoff + pos)
            start += pos.shape[0]
        aoff += l
    tab = np.asarray(tab, dtype=np.int64)
    where = torch.empty(start, dtype=torch.int64, device=dev)
    ops.ext().cascade_where(torch.from_numpy(tab.reshape(-1)).to(dev).data_ptr(), tab.shape[0], int(tab[:, 1].max()),
                            where.data_ptr(), ops.stream_ptr(dev))
    assert np.array_equal(where.cpu().numpy(), np.concatenate(ref))
