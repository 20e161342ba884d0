"""Fused whole-stack inference (ops.stack_infer): the fp64 host
reference of the fused formula vs the per-model predict path (CPU), and the HIP kernel vs that
reference (GPU) — shipped checkpoint, odd row counts, f32/f64 inputs, SV chunking, deep trees."""
import numpy as np
import pytest
import torch

from hfens import ops
from hfens.cli.predict_hf import PATIENT_PARAMS
from hfens.io.checkpoint import load_checkpoint
from hfens.ops import reference as ref
from hfens.ops.packing import PackedStack, pack_forest, pack_stack, pack_svs, stump_table


def _patients(n, seed=1):
    rng = np.random.default_rng(seed)
    X = rng.integers(0, 2, size=(n, 17)).astype(np.float64)
    X[:, 6] += 1
    X[:, 13] = rng.normal(18.6, 4.4, n).round()
    X[:, 15] = rng.integers(0, 5, n)
    X[:, 16] = rng.normal(63, 5, n).round()
    X[0] = list(PATIENT_PARAMS.values())
    return torch.as_tensor(X)


def _random_pstack(F, m, T, depth, device, seed=0, stumps=True):
    g = torch.Generator().manual_seed(seed)
    sv = torch.randn(m, F, generator=g, dtype=torch.float64)
    coef = torch.randn(m, generator=g, dtype=torch.float64) / m ** 0.5
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
            left[t, i], right[t, i] = 2 * i + 1, 2 * i + 2
    tabs = [torch.as_tensor(a) for a in (feat, thr, left, right, val)]
    f = pack_forest(*tabs, device)
    return PackedStack(
        F=F, sv=pack_svs(sv, coef, device),
        mean=(0.1 * torch.randn(F, generator=g)).to(device), inv_scale=(0.5 + torch.rand(F, generator=g)).to(device),
        gamma=0.5 / F, svc_b=0.2, probA=-1.7, probB=0.1, forest=f,
        stumps=stump_table(*tabs, -0.4, 0.1, F, device) if stumps else None, gb_init=-0.4, gb_lr=0.1,
        lr_w=(0.3 * torch.randn(F, generator=g)).to(device), lr_b=-0.2,
        meta_w=(1.9, 0.5, 2.7), meta_b=-2.0)


def test_fused_reference_matches_per_model_path(ckpt_path):
    clf = load_checkpoint(ckpt_path)
    pk = pack_stack(clf, "cpu")
    assert pk is not None and pk.F == 17 and pk.forest.n_trees == 100
    assert pk.stumps is not None and pk.stumps.pairs.shape[0] == 17   # 100 stumps -> 17 pairs
    X = _patients(3000)
    want = clf.predict_proba(X)[:, 1]
    got = ref.stack_infer(X, pk)
    # only the f32 rounding of the packed scaler/SV/LR parameters separates the two
    assert torch.allclose(got, want, atol=1e-6)
    assert f"{100 * float(got[0]):.2f}" == "27.09"


def test_pack_stack_rejects_other_shapes(ckpt_path):
    clf = load_checkpoint(ckpt_path)
    clf.estimators_ = clf.estimators_[:2]
    assert pack_stack(clf, "cpu") is None


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 65, 4097, 100003])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_stack_infer_checkpoint(dev, ckpt_path, n, dtype):
    clf = load_checkpoint(ckpt_path)
    X = _patients(n, seed=n)
    want = clf.predict_proba(X)[:, 1]
    gpu = load_checkpoint(ckpt_path, device=dev)
    got = gpu.predict_p1(X.to(dev, dtype)).cpu().double()
    assert got.shape == (n,)
    assert torch.allclose(got, want, atol=2e-6)
    assert f"{100 * float(got[0]):.2f}" == "27.09"


@pytest.mark.gpu
def test_stack_infer_matches_unfused_gpu(dev, ckpt_path):
    gpu = load_checkpoint(ckpt_path, device=dev)
    X = _patients(20000, seed=3).to(dev)
    fused = gpu.predict_p1(X)
    gpu.fused_inference = False
    unfused = gpu.predict_p1(X)
    assert torch.allclose(fused.double(), unfused.double(), atol=2e-6)


def test_stump_table_reference_matches_tree_walk():
    pk = _random_pstack(17, 64, 300, 1, "cpu", seed=7)
    x = torch.randn(2000, 17, dtype=torch.float64)
    a = ref.stack_infer(x, pk)
    pk.stumps = None
    b = ref.stack_infer(x, pk)
    assert torch.allclose(a, b, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("F,m,T,depth,grid,stumps", [(17, 434, 100, 1, 0, True), (17, 434, 100, 1, 0, False),
                                                     (40, 3000, 30, 3, 0, False), (5, 64, 10, 2, 1, False),
                                                     (17, 6000, 200, 1, 3, True), (64, 500, 50, 1, 0, True)])
def test_stack_infer_random(dev, F, m, T, depth, grid, stumps):
    pk_h = _random_pstack(F, m, T, depth, "cpu", seed=F + m, stumps=stumps)
    pk_d = _random_pstack(F, m, T, depth, dev, seed=F + m, stumps=stumps)
    x = torch.randn(5000, F, dtype=torch.float64)
    want = ref.stack_infer(x.to(torch.float32), pk_h)
    got = ops.stack_infer(x.to(dev), pk_d, grid=grid).cpu().double()
    assert torch.allclose(got, want, atol=5e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("F,m,T,depth,stumps", [(17, 434, 100, 1, True), (5, 64, 10, 2, False), (11, 250, 30, 1, True)])
def test_stack_infer_x3_matches_f32_mfma(dev, monkeypatch, F, m, T, depth, stumps):
    """The RBF products as an exact three-way bf16 split on the bf16 matrix cores (stack.hip X3,
    the default when the SVs fit LDS) against the f32-MFMA kernel (HFENS_STACK_X3=0) and the fp64
    host reference: the decision values differ only by the dropped ≤ 3·2⁻²⁴ piece products."""
    pk_h = _random_pstack(F, m, T, depth, "cpu", seed=F * m, stumps=stumps)
    pk_d = _random_pstack(F, m, T, depth, dev, seed=F * m, stumps=stumps)
    x = torch.randn(20000, F, dtype=torch.float64)
    want = ref.stack_infer(x.to(torch.float32), pk_h)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("HFENS_STACK_X3", mode)
        out[mode] = ops.stack_infer(x.to(dev), pk_d).cpu().double()
    assert torch.allclose(out["1"], out["0"], atol=1e-6)
    assert torch.allclose(out["1"], want, atol=5e-6)


@pytest.mark.gpu
def test_stack_infer_out_buffer(dev, ckpt_path):
    gpu = load_checkpoint(ckpt_path, device=dev)
    pk = gpu._packed_stack(torch.device(dev))
    X = _patients(1000).to(dev, torch.float32)
    out = torch.full((1200,), -1.0, device=dev)
    ops.stack_infer(X, pk, out=out)
    assert float(out[1000:].min()) == -1.0 and float(out[:1000].min()) > 0


@pytest.mark.gpu
def test_batched_predictor_graph_and_stream(dev, ckpt_path):
    from hfens.infer import BatchedPredictor
    gpu = load_checkpoint(ckpt_path, device=dev)
    X = _patients(300001, seed=5).to(torch.float32)
    want = gpu.predict_p1(X.to(dev)).cpu()
    bp = BatchedPredictor(gpu, dev, chunk_rows=65536)
    Xd = X.to(dev)
    a = bp.predict_device(Xd).cpu()
    b = bp.predict_device(Xd).cpu()          # graph replay
    assert torch.equal(a, want) and torch.equal(b, want)
    h = bp.predict_host(X.pin_memory(), chunk_rows=50000)
    assert torch.equal(h, want)


def _force_generic(clf, fn):
    old = clf.HOST_NATIVE_MAX_ROWS
    clf.HOST_NATIVE_MAX_ROWS = -1
    try:
        return fn()
    finally:
        clf.HOST_NATIVE_MAX_ROWS = old


def test_native_host_predictor_matches_per_model_path(ckpt_path):
    """Small host batches go through ops/csrc/host.hip stack_predict_host (config 1 latency):
    f64 throughout, so it matches the per-model torch path to rounding."""
    if not ops.has_ext():
        pytest.skip("HIP extension not built")
    clf = load_checkpoint(ckpt_path)
    assert clf._host_pack() is not None
    X = _patients(200, seed=9)
    got = clf.predict_proba(X)[:, 1]
    want = _force_generic(clf, lambda: clf.predict_proba(X)[:, 1])
    assert float((got - want).abs().max()) < 1e-12
    one = clf.predict_proba(X[:1])
    assert abs(float(one[0, 1]) - 0.2709003008994077) < 1e-12
    assert f"{100 * float(one[0, 1]):.2f}" == "27.09"


def test_native_host_predictor_deep_trees():
    """A freshly trained stack with depth-3 GBC trees (general node walk, not stumps)."""
    if not ops.has_ext():
        pytest.skip("HIP extension not built")
    from hfens.config import EnsembleConfig, build_estimators
    from hfens.io.synth import make_hf_cohort
    X, y, _ = make_hf_cohort(400, 9, seed=4, nan_frac=0.0)
    X, y = torch.as_tensor(X), torch.as_tensor(y)
    clf = build_estimators(EnsembleConfig(gbc_estimators=20, gbc_depth=3)).fit(X, y)
    assert clf._host_pack() is not None
    Xt = torch.as_tensor(make_hf_cohort(150, 9, seed=5, nan_frac=0.0)[0])
    got = clf.predict_proba(Xt)[:, 1]
    want = _force_generic(clf, lambda: clf.predict_proba(Xt)[:, 1])
    assert float((got - want).abs().max()) < 1e-12


@pytest.mark.parametrize("flags", [(False, True), (True, False), (False, False)])
def test_native_host_predictor_honours_scaler_flags(flags):
    """A pipeline whose StandardScaler has with_mean / with_std off: the native host predictor
    uses an identity centre / scale like the per-model path (it used mean_/scale_)."""
    if not ops.has_ext():
        pytest.skip("HIP extension not built")
    from hfens.config import EnsembleConfig, build_estimators
    from hfens.io.synth import make_hf_cohort
    X, y, _ = make_hf_cohort(300, 9, seed=6, nan_frac=0.0)
    X, y = torch.as_tensor(X), torch.as_tensor(y)
    clf = build_estimators(EnsembleConfig(gbc_estimators=10))
    sc = clf.estimators[0][1].steps[0][1]
    sc.with_mean, sc.with_std = flags
    clf.fit(X, y)
    assert clf._host_pack() is not None
    Xt = torch.as_tensor(make_hf_cohort(50, 9, seed=7, nan_frac=0.0)[0])
    got = clf.predict_proba(Xt)[:, 1]
    want = _force_generic(clf, lambda: clf.predict_proba(Xt)[:, 1])
    assert float((got - want).abs().max()) < 1e-12
