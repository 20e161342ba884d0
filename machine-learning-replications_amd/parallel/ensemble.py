"""Seed (ensemble-member) parallelism for batched GBDT fits (SURVEY.md §2.4 "Task / ensemble
parallel": the 5 seeds of the deep ensemble are independent models; BASELINE.json config 5).

The N ranks are split into G = N / S groups of S ranks.  Seeds go to groups round-robin (seed k
→ group k mod G); inside a group the rows are sharded over its S ranks and the group's seeds
train together as ONE batched fit whose per-stage histogram sum runs over the group only
(peer-memory kernel or RCCL, ``models/hist_gbdt.py``).

* S = 1 ("seeds"): every rank trains its seeds on all rows; no collective at all while training.
* S = N ("rows"): every rank holds 1/N of the rows of every seed (plain data parallel).
* in between ("hybrid"): e.g. 8 ranks, 5 seeds, S = 4: two groups of 4 ranks, seeds {0, 2, 4} and
  {1, 3} on 250k-row shards.

Every model is trained on exactly the rows and with exactly the reductions of a one-process fit
(int64 histograms), so each seed's trees are bit-identical to the single-GPU fit whatever the
layout (tests/test_distributed.py::test_seed_parallel_bit_identical).

``auto`` picks S from a per-stage cost model of the stage loop measured on one MI355X
(profiles/r3_gbdt_dp.md, ``scripts/probes/gbdt_shard_probe.py``: 45.3 / 90.1 µs per stage for one
model at 125k / 1M rows, 72.9 / 297.8 µs for five): t(B, n) ≈ F0 + C·B·n with F0 ≈ 40 µs fixed and
C ≈ 51 µs per model per 1M rows, plus ≈ X = 10 µs for the peer reduction when S > 1 (measured at
world 1) — the layout with the smallest bottleneck group.
"""
from __future__ import annotations

import os
from typing import Dict, List, Tuple

STAGE_FIXED_US = float(os.environ.get("HFENS_SEED_COST_F0", "40"))
STAGE_ROW_US = float(os.environ.get("HFENS_SEED_COST_C", "51"))      # per model per 1M rows
STAGE_XGMI_US = float(os.environ.get("HFENS_SEED_COST_X", "10"))


def stage_cost_us(B: int, rows: int, S: int) -> float:
    if B == 0:
        return 0.0
    return STAGE_FIXED_US + STAGE_ROW_US * B * (rows / S) / 1e6 + (STAGE_XGMI_US if S > 1 else 0.0)


def seed_layout(world: int, n_models: int, rows: int, policy: str = "auto") -> int:
    """Ranks per group S (a divisor of ``world``) for ``policy`` ∈ auto | seeds | rows | <int>."""
    divisors = [s for s in range(1, world + 1) if world % s == 0]
    if policy == "seeds":
        return 1
    if policy == "rows":
        return world
    if policy not in ("auto", ""):
        s = int(policy)
        if s not in divisors:
            raise ValueError(f"seed layout: {s} ranks per group does not divide world {world}")
        return s

    def cost(S):
        G = world // S
        busiest = -(-n_models // G)     # seeds of the most loaded group
        return stage_cost_us(busiest, rows, S)
    return min(divisors, key=lambda S: (cost(S), S))


def my_seeds(rank: int, world: int, n_models: int, S: int) -> List[int]:
    G = world // S
    return [k for k in range(n_models) if k % G == rank // S]


_GROUPS: Dict[Tuple[int, int], object] = {}


def group_of(rank: int, world: int, S: int, parent=None):
    """The process group of this rank's S-rank group (every rank creates every group, in order)."""
    import torch.distributed as dist
    if S == 1:
        return None
    if S == world:
        return parent if parent is not None else dist.group.WORLD
    # members as GLOBAL ranks (new_group's numbering): position r of the parent is members[r]
    members = dist.get_process_group_ranks(parent) if parent is not None else list(range(world))
    if len(members) != world:
        raise ValueError(f"group_of: world {world} but the parent group has {len(members)} ranks")
    key = (world, S, tuple(members))
    if key not in _GROUPS:
        mine = None
        for g0 in range(0, world, S):
            # every rank of the DEFAULT group must call new_group for every subgroup, in order;
            # a parent that is not the whole world would need its non-members to call it too
            pg = dist.new_group(members[g0:g0 + S])
            if g0 <= rank < g0 + S:
                mine = pg
        _GROUPS[key] = mine
    return _GROUPS[key]


def fit_seed_ensemble(models, X, y, rank: int, world: int, S: int, parent=None):
    """Train this rank's share of ``models`` (identical lists on every rank; model k = seed k) on
    the full rows ``X, y`` (every rank holds all rows).  Returns the indices trained here; the
    other entries of ``models`` stay unfitted on this rank."""
    from ..models.hist_gbdt import fit_gbdt_batch
    from .dist import shard_bounds
    mine = my_seeds(rank, world, len(models), S)
    g = group_of(rank, world, S, parent)
    if not mine:
        return mine
    lo, hi = shard_bounds(X.shape[0], rank % S, S)
    fit_gbdt_batch([models[k] for k in mine], X[lo:hi], y[lo:hi], group=g)
    return mine
