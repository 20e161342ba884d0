"""Process-group plumbing and the collectives of the data-parallel ensemble
(call sites R1-R9).

One process per GPU; ``torch.distributed`` with backend ``nccl`` (= RCCL over
xGMI on ROCm) for device tensors, ``gloo`` for host tensors (CPU tests).  Rows
are sharded in contiguous rank-ordered blocks, so a row's global index is
``offset(rank) + local index`` and every fold assignment can be computed from
the global layout.

The collectives are few and small (the workload is latency-bound, not
bandwidth-bound): int64 histogram all-reduces (R1, ≤ 0.7 MB per tree level for
6 models × 40 features × 256 bins × 3; on one node through IPC peer memory,
parallel/xgmi.py), moment / Gram / gradient all-reduces (R3-R5, ≤ 40 KB), and
one-shot all-gathers of rows for the task-parallel SVM fits and the KNN donor set
(R6, R9).

What is exact across rank counts (tests/test_distributed.py, world 2/4/8):
* the integer reductions — GBDT fixed-point histograms (bit-identical trees), KNN
  donor arg-mins, sharded AUROC bucket counts — and every task-parallel result
  ('task' policy: all ranks fit on the full rows, bit-identical to one process);
* NOT the f64 sums of the 'dp' policy (LassoCV Grams, scaler moments, LR Newton
  moments/line-search losses): each rank sums its rows, then the ranks' partials are
  added, so the summation order depends on the rank count and a sum moves by a few
  ulp (≤ (N−1)·ε relative to Σ|terms|).  Pinned by test_develop_dp_matches_single:
  same selected features, held-out probabilities within 1e-12 (measured ≤ 4.4e-16).
  A discrete decision that sits on an exact tie of such a sum could still flip.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Sequence

import numpy as np
import torch
import torch.distributed as dist


def init_from_env(backend: str = None):
    """Initialise from torchrun's environment.  Returns ``(group, rank, world)``;
    ``group`` is None for a single process."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return None, 0, 1
    if not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("HFENS_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(rank_device())
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # fail fast instead of hanging on a dead peer
        timeout = datetime.timedelta(seconds=float(os.environ.get("HFENS_DIST_TIMEOUT", "600")))
        dist.init_process_group(backend=backend, timeout=timeout)
        if os.environ.get("HFENS_DIST_REQUIRE_DEVICE", "0") == "1" and torch.cuda.is_available():
            require_device_tensors()
    return dist.group.WORLD, dist.get_rank(), dist.get_world_size()


_TENSOR_COLLECTIVES = ("all_reduce", "all_gather", "broadcast", "reduce_scatter_tensor",
                       "all_gather_into_tensor", "all_to_all_single", "reduce", "gather", "scatter")


def require_device_tensors():
    """Make every tensor collective called through ``torch.distributed`` raise on a host tensor.
    RCCL (backend "nccl") only takes device tensors, while the gloo rehearsals on one card
    (scripts/dp_rehearsal.sh) accept both; with HFENS_DIST_REQUIRE_DEVICE=1 a rehearsal fails where
    an RCCL run would.  (Object collectives are not wrapped: torch stages them itself.)"""
    def wrap(name, fn):
        def checked(*args, **kw):
            for a in list(args) + list(kw.values()):
                ts = a if isinstance(a, (list, tuple)) else [a]
                for t in ts:
                    if isinstance(t, torch.Tensor) and not t.is_cuda:
                        raise RuntimeError(f"torch.distributed.{name} on a host tensor {tuple(t.shape)} "
                                           f"{t.dtype}: RCCL takes device tensors only")
            return fn(*args, **kw)
        checked.__wrapped__ = fn
        return checked
    for name in _TENSOR_COLLECTIVES:
        fn = getattr(dist, name, None)
        if fn is not None and not hasattr(fn, "__wrapped__"):
            setattr(dist, name, wrap(name, fn))


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def rank_device() -> torch.device:
    """This rank's GPU (one process per GPU).  With fewer visible GPUs than local ranks
    (rehearsing several ranks on one card over gloo) ranks share devices round-robin."""
    if not torch.cuda.is_available():
        return torch.device("cpu")
    n = torch.cuda.device_count()
    return torch.device("cuda", local_rank() % max(1, n))


def shutdown():
    if dist.is_initialized():
        from . import xgmi
        xgmi.release_all()
        # communicators cached per process group (keyed by the group object's id) die with it
        from ..models import svc_lowrank
        from . import ensemble
        svc_lowrank._GROUPS.clear()
        ensemble._GROUPS.clear()
        dist.destroy_process_group()


def _world(group):
    return dist.get_world_size(group), dist.get_rank(group)


def shard_bounds(n: int, rank: int, world: int):
    return rank * n // world, (rank + 1) * n // world


def shard_rows(a, rank: int, world: int):
    n = len(a)
    s, e = shard_bounds(n, rank, world)
    return a[s:e]


# ------------------------------------------------------------------------------ reductions
def all_reduce_sum_(t: torch.Tensor, group) -> torch.Tensor:
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def all_reduce_sum_f64(ts: Sequence[torch.Tensor], group) -> List[torch.Tensor]:
    """Sum a list of tensors in ONE collective (flatten → all-reduce → split)."""
    flat = torch.cat([t.reshape(-1).to(torch.float64) for t in ts])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    out, o = [], 0
    for t in ts:
        k = t.numel()
        out.append(flat[o:o + k].reshape(t.shape).to(t.dtype))
        o += k
    return out


def all_reduce_int(x: int, group, device=None) -> int:
    dev = device if device is not None else _default_device(group)
    t = torch.tensor([int(x)], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return int(t.item())


def _default_device(group):
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


# ------------------------------------------------------------------------------ gathers
def all_gather_rows(t: torch.Tensor, group) -> torch.Tensor:
    """Concatenate every rank's rows (variable counts) in rank order."""
    world, _ = _world(group)
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s) for s in sizes]
    m = max(sizes)
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)])


def row_offset(n_local: int, group, device) -> int:
    world, rank = _world(group)
    n = torch.tensor([n_local], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    return int(sum(int(s) for s in sizes[:rank])), int(sum(int(s) for s in sizes))


def merge_value_counts(u: torch.Tensor, c: torch.Tensor, group):
    """Union of per-rank (sorted distinct value, count) tables."""
    uu = all_gather_rows(u[:, None].to(torch.float64), group)[:, 0]
    cc = all_gather_rows(c[:, None].to(torch.int64), group)[:, 0]
    vals, inv = torch.unique(uu, sorted=True, return_inverse=True)
    counts = torch.zeros(vals.numel(), dtype=torch.int64, device=vals.device).index_add_(0, inv, cc)
    return vals.to(u.dtype), counts


def sharded_kfold_test_folds(n_local: int, k: int, group, device) -> torch.Tensor:
    from ..models.model_selection import kfold_test_folds
    off, n = row_offset(n_local, group, device)
    return torch.as_tensor(kfold_test_folds(n, k)[off:off + n_local], device=device)


def sharded_stratified_folds(y_local: torch.Tensor, k: int, group) -> torch.Tensor:
    from ..models.model_selection import stratified_kfold_test_folds
    y_all = all_gather_rows(y_local[:, None].to(torch.float64), group)[:, 0]
    off, _ = row_offset(y_local.shape[0], group, y_local.device)
    tf = stratified_kfold_test_folds(y_all.cpu().numpy(), k)
    return torch.as_tensor(tf[off:off + y_local.shape[0]], device=y_local.device)


def broadcast_tensors(ts: List[torch.Tensor], src: int, group) -> List[torch.Tensor]:
    """Broadcast a list of tensors of (receiver-unknown) shapes/dtypes from ``src``."""
    meta = [None]
    world, rank = _world(group)
    if rank == src:
        meta = [[(tuple(t.shape), str(t.dtype).split(".")[1]) for t in ts]]
    dist.broadcast_object_list(meta, src=src, group=group)
    dev = _default_device(group)
    out = []
    for i, (shape, dt) in enumerate(meta[0]):
        if rank == src:
            buf = ts[i].to(dev).contiguous()
        else:
            buf = torch.empty(shape, dtype=getattr(torch, dt), device=dev)
        dist.broadcast(buf, src=src, group=group)
        out.append(buf)
    return out
