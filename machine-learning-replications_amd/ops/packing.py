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
