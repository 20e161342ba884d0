"""Feature quantisation for histogram GBDT (SURVEY.md K7 ``quantize_bins``).

Trees compare the float32-cast input (sklearn's tree DTYPE), so bins are built on
``float32(x)``.  A feature with ≤ ``max_bins`` distinct values gets one bin per
distinct value — candidate splits are then exactly sklearn's exact-splitter
candidates and thresholds are midpoints of adjacent present values.  Otherwise
distinct values are grouped into ``max_bins`` quantile groups; a split between
groups uses the midpoint of the left group's max and the right group's min.

With a process group every rank bins identically, and exactly as one process on the concatenated
rows would: quantile-group ends are global order statistics found by bisection over
all-reduced counts (``_fit_bins_dp``), so no value table larger than [F, max_bins] is exchanged.  Single-process fits of up to
``HOST_BIN_MAX_ROWS`` rows take the distinct values from ONE device→host copy (numpy) instead of a
device ``unique`` + host read per feature; ``transform`` is one batched ``searchsorted`` against
the +inf-padded edge table of all features.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

# single-process GPU fits bin on the host below this many rows (numpy unique beats the device sorts
# and their syncs on small inputs); measured on the MI355X box: 125k rows took 13.8 ms on the host
# path against ~4 ms for the device path at 1M rows (profiles/r3_gbdt_dp.md)
HOST_BIN_MAX_ROWS = int(os.environ.get("HFENS_HOST_BIN_ROWS", str(1 << 15)))
# per-feature distinct-value all-gathers under DP (round-1 path, kept for A/B)
LEGACY_DP_BINS = os.environ.get("HFENS_DP_BINS", "") == "legacy"


@dataclass
class BinMapper:
    nbins: torch.Tensor     # [F] int32
    lo_val: torch.Tensor    # [F, 256] f64 (min value in bin)
    hi_val: torch.Tensor    # [F, 256] f64 (max value in bin)
    uppers: List[torch.Tensor]  # per feature f32 bin upper edges (= hi values)
    max_bins: int
    nb_host: Optional[np.ndarray] = None   # host copy of nbins
    edges: Optional[torch.Tensor] = None   # [F, max_nb] f32 upper edges, +inf padded

    def select(self, cols) -> "BinMapper":
        """The bin map of a column subset (every feature's bins depend on that column alone, so this
        equals a fit on the selected columns: the stacking trainer bins all candidate columns under
        the LassoCV path and keeps the selected ones)."""
        idx = np.asarray(cols, dtype=np.int64)
        it = torch.as_tensor(idx, device=self.nbins.device)
        nb = np.asarray(self.nb_host if self.nb_host is not None else self.nbins.cpu().numpy())[idx].astype(np.int32)
        edges = None
        if self.edges is not None:
            K = int(nb.max()) if nb.shape[0] else 1
            edges = self.edges.index_select(0, it)[:, :K].contiguous()
        return BinMapper(self.nbins.index_select(0, it).contiguous(), self.lo_val.index_select(0, it).contiguous(),
                         self.hi_val.index_select(0, it).contiguous(), [self.uppers[int(i)] for i in idx],
                         self.max_bins, nb_host=nb.copy(), edges=edges)

    @property
    def max_nb(self) -> int:
        return int(self.nb_host.max()) if self.nb_host is not None else int(self.nbins.max())

    def transform(self, X: torch.Tensor) -> torch.Tensor:
        """``X [n, F]`` → feature-major uint8 bins ``[F, n]`` (one batched searchsorted: a value
        above every real edge lands on the first +inf pad = the edge count, then clamps to the
        last bin exactly as a per-feature search would).  On the GPU: the ``quantize_bins`` kernel
        (edge table in LDS, row-major input read once, feature-major output)."""
        if X.is_cuda and X.dim() == 2 and X.shape[1] <= 128:
            from .. import ops
            Xc = X.contiguous() if X.dtype in (torch.float32, torch.float64) else X.to(torch.float32).contiguous()
            edges = (self.edges if self.edges is not None else _pad_edges(self.uppers, X.device)).to(X.device)
            edges = edges.contiguous()
            n, F = Xc.shape
            out = torch.empty(F, n, dtype=torch.uint8, device=X.device)
            ops.ext().quantize_bins(Xc.data_ptr(), int(Xc.dtype == torch.float64), n, F, edges.data_ptr(),
                                    int(edges.shape[1]), self.nbins.to(X.device).contiguous().data_ptr(),
                                    out.data_ptr(), n, ops.stream_ptr(X.device))
            return out
        X32 = X.to(torch.float32).t().contiguous()
        edges = self.edges if self.edges is not None else _pad_edges(self.uppers, X.device)
        idx = torch.searchsorted(edges.to(X32.device), X32)
        idx = torch.minimum(idx, (self.nbins.to(device=idx.device, dtype=idx.dtype) - 1)[:, None])
        return idx.to(torch.uint8)


def _fit_bins_device(X32: torch.Tensor, max_bins: int, guard=None) -> BinMapper:
    """All features at once on the device, then ONE device→host copy of the [F, max_bins] tables.

    * Features whose values are all integers in [0, 255] (binary flags, small ordinals — most of a
      Table-S1 cohort) need no sort: one batched ``bincount`` of the values gives their occupied
      values, i.e. the sorted distinct values.
    * The other features are sorted (one radix sort each), then run starts give the distinct counts
      and the ≤ max_bins distinct values, or the quantile group ends (hi = the value of rank
      ⌈i·n/max_bins⌉, lo of the next group = the next distinct value).
    Same bins as the per-feature path (run-rank ⇔ cumulative count)."""
    n, F = X32.shape
    dev = X32.device
    Xt = X32.t().contiguous()
    is_small_int = ((Xt == torch.round(Xt)) & (Xt >= 0) & (Xt <= 255)).all(1)
    occ = None
    if guard is not None:   # the caller's deferred input guards ride on this read (one sync, not three)
        flags, specs = guard
        h = torch.cat([is_small_int, torch.stack(list(flags))]).cpu()
        from ..utils.guards import raise_flags
        raise_flags(h[F:].tolist(), specs)
        si_h = h[:F]
    else:
        si_h = is_small_int.cpu()                                        # one sync: which features
    int_f = [f for f in range(F) if bool(si_h[f])]
    if int_f and max_bins < 256:
        # 256 distinct integers would exceed max_bins: those features go to the sorted path
        ii = torch.as_tensor(int_f, device=dev)
        codes = Xt.index_select(0, ii).to(torch.int64) + 256 * torch.arange(len(int_f), device=dev)[:, None]
        nocc = (torch.bincount(codes.reshape(-1), minlength=256 * len(int_f)).view(len(int_f), 256) > 0).sum(1).cpu()
        int_f = [f for j, f in enumerate(int_f) if int(nocc[j]) <= max_bins]
    sort_f = [f for f in range(F) if f not in set(int_f)]
    occ_d = None
    if int_f:
        ii = torch.as_tensor(int_f, device=dev)
        codes = Xt.index_select(0, ii).to(torch.int64) + 256 * torch.arange(len(int_f), device=dev)[:, None]
        occ_d = torch.bincount(codes.reshape(-1), minlength=256 * len(int_f)).view(len(int_f), 256) > 0
    srt = new = None
    if sort_f:
        srt = torch.empty(len(sort_f), n, dtype=X32.dtype, device=dev)   # [F_sort, n]
        for i_, f in enumerate(sort_f):   # one-dimensional radix sorts beat one segmented sort (measured)
            srt[i_] = torch.sort(Xt[f])[0]
        new = torch.ones_like(srt, dtype=torch.bool)
        new[:, 1:] = srt[:, 1:] != srt[:, :-1]
    # one read for both paths: occupied small integers, distinct counts of the sorted features
    parts = ([occ_d.reshape(-1).to(torch.int64)] if int_f else []) + ([new.sum(1)] if sort_f else [])
    hv = torch.cat(parts).cpu() if parts else torch.zeros(0, dtype=torch.int64)
    if int_f:
        occ = hv[:256 * len(int_f)].view(len(int_f), 256) > 0
    ks = hv[256 * len(int_f):] if int_f else hv
    k_h = torch.zeros(F, dtype=torch.int64)
    small_h = torch.full((F, max_bins), float("nan"), dtype=torch.float32)
    hi_h = torch.zeros(F, max_bins, dtype=torch.float32)
    lo_h = torch.zeros(F, max_bins, dtype=torch.float32)
    mn_h = torch.zeros(F, dtype=torch.float32)
    for j, f in enumerate(int_f):
        vals = torch.nonzero(occ[j])[:, 0].to(torch.float32)
        k_h[f] = vals.numel()
        small_h[f, :vals.numel()] = vals
        mn_h[f] = vals[0]
    if sort_f:
        k_h[sort_f] = ks
        small_s = [i_ for i_ in range(len(sort_f)) if int(ks[i_]) <= max_bins]
        big_s = [i_ for i_ in range(len(sort_f)) if int(ks[i_]) > max_bins]
        if small_s:
            packed = torch.full((len(small_s), max_bins), float("nan"), dtype=torch.float32, device=dev)
            for r_, i_ in enumerate(small_s):
                v = srt[i_][new[i_]]                                     # ≤ max_bins values
                packed[r_, :v.numel()] = v
            small_h[[sort_f[i_] for i_ in small_s]] = packed.cpu()
        mn_h[sort_f] = srt[:, 0].cpu()
        if big_s:
            bi = torch.as_tensor(big_s, device=dev)
            sb = srt.index_select(0, bi)
            tau = torch.arange(1, max_bins, dtype=torch.float64, device=dev) * (n / max_bins)
            idx = torch.cat([torch.ceil(tau).to(torch.int64) - 1, torch.tensor([n - 1], device=dev)]).clamp(0, n - 1)
            hq = sb[:, idx].contiguous()                                 # quantile group ends
            pos = torch.searchsorted(sb, hq, right=True).clamp(max=n - 1)
            big_f = [sort_f[i_] for i_ in big_s]
            hi_h[big_f] = hq.cpu()
            lo_h[big_f] = sb.gather(1, pos).cpu()                       # next distinct values
    return _assemble(k_h, small_h, hi_h, lo_h, mn_h, max_bins, dev)


def _keys(v32: torch.Tensor) -> torch.Tensor:
    """float32 → int64 keys in [0, 2³²) with the float order (negatives bit-flipped)."""
    b = v32.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    return torch.where(b >= 0x80000000, 0xFFFFFFFF - b, b + 0x80000000)


def _unkey(k: torch.Tensor) -> torch.Tensor:
    b = torch.where(k >= 0x80000000, k - 0x80000000, 0xFFFFFFFF - k)
    b = torch.where(b >= 0x80000000, b - (1 << 32), b)
    return b.to(torch.int32).view(torch.float32)


def _fit_bins_dp(X32: torch.Tensor, max_bins: int, group) -> BinMapper:
    """Row-sharded binning, the same bins as a single-process fit on the concatenated rows, with no
    row or value table crossing the ranks:

    * each rank sorts its shard per feature; one MAX all-reduce of the local distinct counts and one
      SUM of the row counts;
    * features whose every shard has ≤ max_bins distinct values all-gather those ≤ max_bins tables
      (the union decides: ≤ max_bins distinct → one bin per value, else quantile groups);
    * quantile-group ends are global order statistics (value of rank ⌈i·n/max_bins⌉ − 1), found for
      all features and groups at once by bisection on order-preserving 32-bit keys: 32 rounds of
      local ``searchsorted`` counts + one SUM all-reduce of an [F, max_bins] int64 table;
    * the next distinct value above each end and the minima: one MIN all-reduce each."""
    import torch.distributed as dist
    n_loc, F = X32.shape
    dev = X32.device
    inf = float("inf")
    Xt = (X32 + 0.0).t().contiguous()                                    # +0.0: −0 → +0 (one value)
    # small non-negative integer features (binary flags, ordinals: most of a Table-S1 cohort): their
    # distinct values over ALL ranks are the occupied cells of a [F, 256] bincount (one MAX
    # all-reduce) — no sort and no value-table gather for them
    si = ((Xt == torch.round(Xt)) & (Xt >= 0) & (Xt <= 255)).all(1).to(torch.int64)
    dist.all_reduce(si, op=dist.ReduceOp.MIN, group=group)
    occ = torch.zeros(F, 256, dtype=torch.int64, device=dev)
    si_d = si.bool()
    if n_loc > 0 and bool(si_d.any()):
        ii = torch.nonzero(si_d)[:, 0]
        codes = Xt.index_select(0, ii).to(torch.int64) + 256 * torch.arange(ii.numel(), device=dev)[:, None]
        occ[ii] = (torch.bincount(codes.reshape(-1), minlength=256 * ii.numel()).view(-1, 256) > 0).to(torch.int64)
    dist.all_reduce(occ, op=dist.ReduceOp.MAX, group=group)
    occ_h = occ.cpu().numpy() > 0
    si_h = si.cpu().numpy() > 0
    int_f = [f for f in range(F) if si_h[f] and int(occ_h[f].sum()) <= max_bins]
    rest = [f for f in range(F) if f not in set(int_f)]
    ri = torch.as_tensor(rest, dtype=torch.int64, device=dev)
    srt_r = torch.sort(Xt.index_select(0, ri), dim=1)[0] if rest else Xt[:0]
    srt = torch.zeros(F, n_loc, dtype=Xt.dtype, device=dev)
    if rest:
        srt[ri] = srt_r
    new = torch.ones_like(srt, dtype=torch.bool)
    new[:, 1:] = srt[:, 1:] != srt[:, :-1]
    k_loc = new.sum(1).to(torch.int64)
    kmax = k_loc.clone()
    dist.all_reduce(kmax, op=dist.ReduceOp.MAX, group=group)
    n_t = torch.tensor([n_loc], dtype=torch.int64, device=dev)
    dist.all_reduce(n_t, op=dist.ReduceOp.SUM, group=group)
    n = int(n_t.item())
    kmax_h = kmax.cpu()
    k_h = torch.full((F,), max_bins + 1, dtype=torch.int64)
    small_h = torch.full((F, max_bins), float("nan"), dtype=torch.float32)
    mn_int = {}
    for f in int_f:
        vals = np.nonzero(occ_h[f])[0].astype(np.float32)
        k_h[f] = int(vals.shape[0])
        small_h[f, :vals.shape[0]] = torch.from_numpy(vals)
        mn_int[f] = float(vals[0]) if vals.shape[0] else inf
    cand = [f for f in rest if int(kmax_h[f]) <= max_bins]
    if cand:
        tab = torch.full((len(cand), max_bins), float("nan"), dtype=torch.float32, device=dev)
        for i_, f in enumerate(cand):
            v = srt[f][new[f]]
            tab[i_, :v.numel()] = v
        world = dist.get_world_size(group)
        bufs = [torch.empty_like(tab) for _ in range(world)]
        dist.all_gather(bufs, tab, group=group)
        allv = torch.cat(bufs, 1).cpu()
        for i_, f in enumerate(cand):
            u = torch.unique(allv[i_][~torch.isnan(allv[i_])], sorted=True)
            if u.numel() <= max_bins:
                k_h[f] = u.numel()
                small_h[f, :u.numel()] = u
    big_f = [f for f in rest if int(k_h[f]) > max_bins]
    hi_h = torch.zeros(F, max_bins, dtype=torch.float32)
    lo_h = torch.zeros(F, max_bins, dtype=torch.float32)
    mn = srt[:, 0].clone() if n_loc > 0 else torch.full((F,), inf, dtype=torch.float32, device=dev)
    dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=group)
    mn_h = mn.cpu()
    for f, v in mn_int.items():
        mn_h[f] = v
    if big_f:
        bi = torch.as_tensor(big_f, device=dev)
        sb = srt.index_select(0, bi).contiguous()
        kb = _keys(sb)                                                    # sorted like sb
        tau = torch.arange(1, max_bins, dtype=torch.float64) * (n / max_bins)
        r = torch.cat([torch.ceil(tau).to(torch.int64) - 1, torch.tensor([n - 1])]).clamp(0, n - 1)
        need = (r + 1).to(dev).expand(len(big_f), max_bins).contiguous()
        lo_k = torch.zeros_like(need)
        hi_k = torch.full_like(need, 0xFFFFFFFF)
        # smallest key K with #(key ≤ K) ≥ rank + 1 over all ranks: a 16-way search, 4 key bits per
        # round — 9 rounds (the span shrinks ≥ 16× per round, ≤ 1 after 8; no host sync in the loop)
        # instead of 32 bisections;
        # the same K (each round keeps the sub-interval holding the first pivot that reaches it)
        m = torch.arange(1, 16, dtype=torch.int64, device=dev)
        for _ in range(9):
            span = hi_k - lo_k                                           # [Fb, G] (≥ 0)
            piv = lo_k[..., None] + (span[..., None] * m) // 16          # [Fb, G, 15] ascending
            if n_loc > 0:
                cnt = torch.searchsorted(kb, piv.reshape(len(big_f), -1), right=True).view_as(piv)
            else:
                cnt = torch.zeros_like(piv)
            dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=group)
            ge = cnt >= need[..., None]
            first = torch.where(ge.any(-1), ge.to(torch.int64).argmax(-1), torch.full_like(lo_k, 15))
            # answer in (piv[first-1], piv[first]] (piv[-1] = lo_k - 1, piv[15] = hi_k)
            prev = torch.where(first > 0, piv.gather(-1, (first - 1).clamp(min=0)[..., None])[..., 0] + 1, lo_k)
            nxt_hi = torch.where(first < 15, piv.gather(-1, first.clamp(max=14)[..., None])[..., 0], hi_k)
            lo_k, hi_k = prev, nxt_hi
        hq = _unkey(lo_k)                                                 # quantile group ends
        if n_loc > 0:
            pos = torch.searchsorted(sb, hq, right=True)
            nxt = torch.where(pos < n_loc, sb.gather(1, pos.clamp(max=n_loc - 1)), torch.full_like(hq, inf))
        else:
            nxt = torch.full_like(hq, inf)
        dist.all_reduce(nxt, op=dist.ReduceOp.MIN, group=group)        # next distinct values
        hi_h[big_f] = hq.cpu()
        lo_h[big_f] = nxt.cpu()
    return _assemble(k_h, small_h, hi_h, lo_h, mn_h, max_bins, dev)


def _assemble(k_h, small_h, hi_h, lo_h, mn_h, max_bins: int, dev) -> BinMapper:
    """BinMapper from per-feature host tables: ``k_h`` distinct counts; ``small_h`` the sorted
    distinct values of features with ≤ max_bins of them; ``hi_h`` the quantile group ends and
    ``lo_h`` the next distinct value above each end (features with more); ``mn_h`` the minima.
    Host numpy on [F, 256] tables (a fit's fixed cost: per-feature torch ops cost ~0.2 ms each)."""
    k_h = np.asarray(k_h, dtype=np.int64)
    small_h, hi_h, lo_h = np.asarray(small_h), np.asarray(hi_h), np.asarray(lo_h)
    mn_h = np.asarray(mn_h)
    F = int(k_h.shape[0])
    nb = np.empty(F, dtype=np.int32)
    lo = np.zeros((F, 256), dtype=np.float64)
    hi = np.zeros((F, 256), dtype=np.float64)
    for f in range(F):
        kf = int(k_h[f])
        if kf <= max_bins:
            u = small_h[f, :kf].astype(np.float64)
            nb[f] = kf
            lo[f, :kf] = u
            hi[f, :kf] = u
        else:
            h = hi_h[f]
            keep = np.ones(max_bins, dtype=bool)
            keep[1:] = h[1:] != h[:-1]
            ends = h[keep]
            nxt = lo_h[f][keep]
            g = int(ends.shape[0])
            nb[f] = g
            hi[f, :g] = ends.astype(np.float64)
            lo[f, 0] = float(mn_h[f])
            lo[f, 1:g] = nxt[:-1].astype(np.float64)
    return _finalize(nb, lo, hi, max_bins, dev)


def _finalize(nb: np.ndarray, lo: np.ndarray, hi: np.ndarray, max_bins: int, dev,
              non_blocking: bool = False) -> BinMapper:
    """Edges of every feature at once (:func:`_edges_all`) and the device tables.  ``non_blocking``:
    pinned copies that do not wait for the current stream's queued work."""
    E = _edges_all(lo, hi, nb)

    def up(a):
        t = torch.from_numpy(np.ascontiguousarray(a))
        if non_blocking and torch.device(dev).type == "cuda":
            return t.pin_memory().to(dev, non_blocking=True)
        return t.to(dev)
    edges = up(E)
    uppers = [edges[f, :int(nb[f])] for f in range(nb.shape[0])]
    return BinMapper(up(nb.astype(np.int32)), up(lo), up(hi), uppers, max_bins,
                     nb_host=nb.astype(np.int32).copy(), edges=edges)


def _edges_all(lo: np.ndarray, hi: np.ndarray, nb: np.ndarray) -> np.ndarray:
    """:func:`_threshold_edges` for all features at once: [F, 256] f64 bin bounds → [F, max nb] f32
    upper edges, +inf padded (the same IEEE operations element for element, so the same bits)."""
    a, c = hi[:, :-1], lo[:, 1:]
    with np.errstate(invalid="ignore", over="ignore"):
        t = a / 2.0 + c / 2.0
        t = np.where((t == c) | np.isinf(t), a, t)
        t32 = t.astype(np.float32)
        down = np.nextafter(t32, np.float32(-np.inf))
        t32 = np.where(t32.astype(np.float64) > t, down, t32)
        t32 = np.where(t32.astype(np.float64) >= c, a.astype(np.float32), t32)
    e = hi.astype(np.float32)
    inner = np.arange(255)[None, :] < (nb[:, None].astype(np.int64) - 1)
    e[:, :-1] = np.where(inner, t32, e[:, :-1])
    K = int(nb.max()) if nb.shape[0] else 1
    out = np.full((nb.shape[0], K), np.inf, dtype=np.float32)
    valid = np.arange(K)[None, :] < nb[:, None].astype(np.int64)
    out[valid] = e[:, :K][valid]
    return out


def _threshold_edges(lo: torch.Tensor, hi: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """Upper bin edges AT the split thresholds the trees use (gbdt.hip: t = hi[b]/2 + lo[b+1]/2,
    t == lo[b+1] → hi[b]; sklearn's midpoint rule), so ``bin(x) ≤ blo ⟺ x ≤ threshold`` for ANY x —
    binned inference (folded tables, the fp8 MFMA forest) then equals threshold inference on new
    data, not only on the training values.  Training values bin identically either way."""
    k = int(lo.numel())
    e = up.to(torch.float32).clone()
    if k >= 2:
        a, c = hi[:-1].double(), lo[1:].double()
        t = a / 2.0 + c / 2.0
        t = torch.where((t == c) | torch.isinf(t), a, t)
        t32 = t.to(torch.float32)
        # round toward a: a float32 x == t32 > t must bin right (the threshold walk: x <= t is
        # false), so an edge that rounded up steps back to the float below it (still ≥ a)
        down = torch.nextafter(t32, torch.full_like(t32, -float("inf")))
        t32 = torch.where(t32.double() > t, down, t32)
        t32 = torch.where(t32.double() >= c, a.to(torch.float32), t32)
        e[:-1] = t32
    return e


def _pad_edges(uppers: List[torch.Tensor], device) -> torch.Tensor:
    K = max(int(u.numel()) for u in uppers)
    E = torch.full((len(uppers), K), float("inf"), dtype=torch.float32)
    for f, u in enumerate(uppers):
        E[f, :u.numel()] = u.cpu()
    return E.to(device)


def _distinct(v32: torch.Tensor, group=None):
    u, c = torch.unique(v32, sorted=True, return_counts=True)
    if group is not None:
        from ..parallel import dist as pdist
        u, c = pdist.merge_value_counts(u, c, group)
    return u, c


def fit_bins(X: torch.Tensor, max_bins: int = 256, group=None, guard=None) -> BinMapper:
    """``guard``: optional (device bool flags, specs) of deferred input checks
    (``utils.guards.finite_flag``/``binary_flag``), read with the device bin fit's first transfer;
    on other paths they are read here."""
    if not 2 <= max_bins <= 256:
        raise ValueError("max_bins must be in [2, 256]")
    n, F = X.shape
    dev = X.device
    X32 = X.to(torch.float32)
    host = group is None and n <= HOST_BIN_MAX_ROWS
    if group is None and not host and X32.is_cuda:
        return _fit_bins_device(X32, max_bins, guard)
    if guard is not None:
        from ..utils.guards import raise_flags
        raise_flags(torch.stack(list(guard[0])).cpu().tolist(), guard[1])
    if group is not None and not LEGACY_DP_BINS:
        return _fit_bins_dp(X32, max_bins, group)
    if host:
        return fit_bins_host(X32.cpu().numpy(), max_bins, dev, non_blocking=X32.is_cuda)
    nb = np.empty(F, dtype=np.int32)
    lo = np.zeros((F, 256), dtype=np.float64)
    hi = np.zeros((F, 256), dtype=np.float64)
    for f in range(F):
        u, c = _distinct(X32[:, f].contiguous(), group)
        u = u.cpu()
        c = c.cpu()
        k = u.numel()
        if k <= max_bins:
            nb[f] = k
            lo[f, :k] = u.double().numpy()
            hi[f, :k] = u.double().numpy()
        else:
            cum = torch.cumsum(c, 0).double()
            tot = float(cum[-1])
            # group end = last distinct value whose cumulative count reaches the quantile
            targets = torch.arange(1, max_bins, dtype=torch.float64) * (tot / max_bins)
            ends = torch.searchsorted(cum, targets).clamp(max=k - 1)
            ends = torch.unique(torch.cat([ends, torch.tensor([k - 1])]))
            starts = torch.cat([torch.tensor([0]), ends[:-1] + 1])
            g = ends.numel()
            nb[f] = g
            lo[f, :g] = u[starts].double().numpy()
            hi[f, :g] = u[ends].double().numpy()
    return _finalize(nb, lo, hi, max_bins, dev)


def fit_bins_host(Xh32: np.ndarray, max_bins: int, dev, non_blocking: bool = False) -> BinMapper:
    """The host fit of :func:`fit_bins` from a float32 host array [n, F] (the caller already holds
    the rows on the host, e.g. a pinned copy read under earlier device work): numpy distinct values
    per column, the same bins as every other path."""
    if not 2 <= max_bins <= 256:
        raise ValueError("max_bins must be in [2, 256]")
    n, F = Xh32.shape
    nb = np.empty(F, dtype=np.int32)
    lo = np.zeros((F, 256), dtype=np.float64)
    hi = np.zeros((F, 256), dtype=np.float64)
    for f in range(F):
        u, c = np.unique(Xh32[:, f], return_counts=True)
        k = u.shape[0]
        if k <= max_bins:
            nb[f] = k
            lo[f, :k] = u.astype(np.float64)
            hi[f, :k] = u.astype(np.float64)
        else:
            cum = np.cumsum(c.astype(np.int64)).astype(np.float64)
            tot = float(cum[-1])
            # group end = last distinct value whose cumulative count reaches the quantile
            targets = np.arange(1, max_bins, dtype=np.float64) * (tot / max_bins)
            ends = np.minimum(np.searchsorted(cum, targets), k - 1)
            ends = np.unique(np.concatenate([ends, [k - 1]]))
            starts = np.concatenate([[0], ends[:-1] + 1])
            g = ends.shape[0]
            nb[f] = g
            lo[f, :g] = u[starts].astype(np.float64)
            hi[f, :g] = u[ends].astype(np.float64)
    return _finalize(nb, lo, hi, max_bins, dev, non_blocking)
