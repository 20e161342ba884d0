"""Device layouts for the inference kernels (built once per model, cached)."""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass
class PackedSV:
    svt: torch.Tensor    # [2*KS, mp] f32, k-major, zero padded
    sn: torch.Tensor     # [mp] ‖sv‖²
    coef: torch.Tensor   # [mp] dual coefficients (0 in padding)
    mp: int
    F: int


def pack_svs(sv: torch.Tensor, coef: torch.Tensor, device) -> PackedSV:
    sv32 = sv.to(device=device, dtype=torch.float32)
    m, F = sv32.shape
    mp = (m + 31) // 32 * 32
    kp = (F + 1) // 2 * 2
    svt = torch.zeros(kp, mp, dtype=torch.float32, device=device)
    svt[:F, :m] = sv32.t()
    sn = torch.zeros(mp, dtype=torch.float32, device=device)
    sn[:m] = (sv32 * sv32).sum(1)
    c = torch.zeros(mp, dtype=torch.float32, device=device)
    c[:m] = coef.to(device=device, dtype=torch.float32)
    return PackedSV(svt.contiguous(), sn, c, mp, F)


def f32_round_down(thr: torch.Tensor) -> torch.Tensor:
    """Largest float32 t with t <= thr (elementwise), so that for float32 x:
    ``x <= t`` ⇔ ``float64(x) <= thr``."""
    t = thr.to(torch.float32)
    over = t.to(torch.float64) > thr
    return torch.where(over, torch.nextafter(t, torch.tensor(float("-inf"), dtype=torch.float32,
                                                             device=t.device)), t)


@dataclass
class PackedForest:
    nodes: torch.Tensor   # [T*K, 4] int32 {feature, left, right, bits(thr32)}
    values: torch.Tensor  # [T*K] f32
    n_trees: int
    max_nodes: int
    max_feature: int


def pack_forest(feature, threshold, left, right, value, device) -> PackedForest:
    T, K = feature.shape
    thr32 = f32_round_down(threshold.to(torch.float64).cpu())
    nodes = torch.stack([feature.to(torch.int32).cpu(), left.to(torch.int32).cpu(),
                         right.to(torch.int32).cpu(), thr32.view(torch.int32)], dim=-1)
    nodes = nodes.reshape(T * K, 4).contiguous().to(device)
    vals = value.to(torch.float32).reshape(T * K).contiguous().to(device)
    return PackedForest(nodes, vals, T, K, int(feature.max()))


@dataclass
class StumpTable:
    """Depth-1 ensemble folded per feature: ``init + lr·Σ_t v_t(x)`` =
    ``base + Σ_j [x[f_j] > thr_j]·delta_j`` with the pairs grouped by feature (``off[f]:off[f+1]``)
    and equal (feature, threshold) stumps merged — the shipped 100-stump GBC becomes 17 pairs."""
    off: torch.Tensor     # [F+1] int32
    pairs: torch.Tensor   # [P, 2] f32 (thr32 rounded down, lr·(v_right − v_left))
    base: float


def stump_table(feature, threshold, left, right, value, init: float, lr: float, F: int,
                device) -> "StumpTable | None":
    feature = feature.cpu()
    T, K = feature.shape
    if K < 3 or T == 0:
        return None
    left, right = left.cpu(), right.cpu()
    if bool((feature[:, 0] < 0).any()) or bool((feature[:, 1:3] >= 0).any()) or \
            bool((left[:, 0] != 1).any()) or bool((right[:, 0] != 2).any()):
        return None
    value = value.cpu().to(torch.float64)
    thr32 = f32_round_down(threshold[:, 0].to(torch.float64).cpu())
    base = float(init) + float(lr) * float(value[:, 1].sum())
    merged = {}
    for f, t, vl, vr in zip(feature[:, 0].tolist(), thr32.tolist(), value[:, 1].tolist(), value[:, 2].tolist()):
        merged[(f, t)] = merged.get((f, t), 0.0) + float(lr) * (vr - vl)
    keys = sorted(merged)
    off = torch.zeros(F + 1, dtype=torch.int32)
    for f, _ in keys:
        off[f + 1] += 1
    off = off.cumsum(0).to(torch.int32)
    pairs = torch.tensor([[t, merged[(f, t)]] for f, t in keys], dtype=torch.float32).reshape(-1, 2)
    return StumpTable(off.to(device), pairs.contiguous().to(device), base)


@dataclass
class PackedStack:
    """Everything the fused ``stack_infer`` kernel needs for one fitted HF stack
    (Pipeline(StandardScaler, SVC(rbf, probability)) + GBC + LogisticRegression → meta LR)."""
    F: int
    sv: PackedSV
    mean: torch.Tensor        # [F] f32
    inv_scale: torch.Tensor   # [F] f32
    gamma: float
    svc_b: float              # libsvm intercept (−rho)
    probA: float
    probB: float
    forest: PackedForest
    stumps: "StumpTable | None"
    gb_init: float
    gb_lr: float
    lr_w: torch.Tensor        # [F] f32
    lr_b: float
    meta_w: tuple             # weights of (p_svc, p_gbc, p_lg)
    meta_b: float


def pack_stack(clf, device) -> "PackedStack | None":
    """Pack a fitted binary :class:`StackingClassifier` for the fused kernel; ``None`` when
    its shape is not the HF stack (the caller then runs the per-model path)."""
    from ..models.gbdt import GradientBoostingClassifier
    from ..models.linear import LogisticRegression
    from ..models.scaler import StandardScaler
    from ..models.stacking import Pipeline
    from ..models.svc import SVC
    ests = getattr(clf, "estimators_", None)
    fin = getattr(clf, "final_estimator_", None)
    if ests is None or len(ests) != 3 or not isinstance(fin, LogisticRegression):
        return None
    if getattr(clf, "passthrough", False):
        return None
    slots = {}
    for i, e in enumerate(ests):
        if isinstance(e, Pipeline) and len(e.steps) == 2 and isinstance(e.steps[0][1], StandardScaler) \
                and isinstance(e.steps[1][1], SVC):
            slots["svc"] = (i, e)
        elif isinstance(e, GradientBoostingClassifier):
            slots["gbc"] = (i, e)
        elif isinstance(e, LogisticRegression):
            slots["lg"] = (i, e)
    if len(slots) != 3:
        return None
    _, pipe = slots["svc"]
    sc, svc = pipe.steps[0][1], pipe.steps[1][1]
    if svc.kernel != "rbf" or not svc.probability or svc._dual_coef_.shape[0] != 1:
        return None
    gbc, lg = slots["gbc"][1], slots["lg"][1]
    F = int(sc.mean_.numel())
    if int(lg.coef_.shape[1]) != F or int(gbc.tree_feature_.max()) >= F:
        return None
    mean = sc.mean_.to(torch.float64) if sc.with_mean else torch.zeros(F, dtype=torch.float64)
    scale = sc.scale_.to(torch.float64) if sc.with_std else torch.ones(F, dtype=torch.float64)
    mc = fin.coef_[0].to(torch.float64).cpu()
    w = (float(mc[slots["svc"][0]]), float(mc[slots["gbc"][0]]), float(mc[slots["lg"][0]]))
    return PackedStack(
        F=F,
        sv=pack_svs(svc.support_vectors_, svc._dual_coef_[0], device),
        mean=mean.to(device=device, dtype=torch.float32).contiguous(),
        inv_scale=(1.0 / scale).to(device=device, dtype=torch.float32).contiguous(),
        gamma=float(svc._gamma), svc_b=float(svc._intercept_[0]),
        probA=float(svc._probA[0]), probB=float(svc._probB[0]),
        forest=pack_forest(gbc.tree_feature_, gbc.tree_threshold_, gbc.tree_left_, gbc.tree_right_,
                           gbc.tree_value_, device),
        stumps=stump_table(gbc.tree_feature_, gbc.tree_threshold_, gbc.tree_left_, gbc.tree_right_,
                           gbc.tree_value_, float(gbc.init_raw_), float(gbc.learning_rate), F, device),
        gb_init=float(gbc.init_raw_), gb_lr=float(gbc.learning_rate),
        lr_w=lg.coef_[0].to(device=device, dtype=torch.float32).contiguous(),
        lr_b=float(lg.intercept_[0]),
        meta_w=w, meta_b=float(fin.intercept_[0]))
