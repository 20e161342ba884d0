"""Batched histogram GBDT training (binomial deviance) on device.

B models — e.g. the 5 stacking OOF folds + the full refit, or several seeds —
share one binned matrix and train in lock-step: every boosting stage is one
``apply_prep`` launch, then per tree level one ``hist`` + one ``split`` (+ one
``route`` above the last level) launch, each covering all B models.  Kernels:
``ops/csrc/gbdt.hip``.  The same algorithm runs on host tensors through a
plain-PyTorch mirror (``_HostKernels``) so CPU runs and kernel tests share
semantics.

Exactness notes (vs sklearn ``GradientBoostingClassifier``):
* per-stage residual r = y − σ(raw), Newton leaf value Σr / Σp(1−p), raw += lr·value,
  init raw = log-odds of the (weighted) class prior; node values/impurities and
  ``train_score_`` (binomial deviance after each stage) as sklearn stores them.
* histogram sums are fixed-point int64 (scale 2^shift): exact, deterministic and
  identical for any data-parallel split of the rows.
* split candidates/thresholds = sklearn's exact splitter when a feature has ≤256
  distinct values; ties between features resolve to the lowest feature index
  (sklearn: first in a random feature permutation).
"""
from __future__ import annotations

import functools
import math
import os
import time
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from .binning import BinMapper, fit_bins

F32_EPS = float(np.finfo(np.float32).eps)


def _qshift(n_total: int) -> int:
    return 40 if n_total <= (1 << 22) else 32


# ============================================================================ bagging RNG
_M64 = (1 << 64) - 1


def _splitmix64_t(x: torch.Tensor) -> torch.Tensor:
    """splitmix64 on int64 tensors (two's-complement wraparound = mod 2^64)."""
    def srl(v, k):
        return (v >> k) & ((1 << (64 - k)) - 1)
    x = x + torch.tensor(0x9E3779B97F4A7C15 - (1 << 64), dtype=torch.int64, device=x.device)
    x = (x ^ srl(x, 30)) * torch.tensor(0xBF58476D1CE4E5B9 - (1 << 64), dtype=torch.int64, device=x.device)
    x = (x ^ srl(x, 27)) * torch.tensor(0x94D049BB133111EB - (1 << 64), dtype=torch.int64, device=x.device)
    return x ^ srl(x, 31)


def bag_mask(seeds: torch.Tensor, stage: int, gidx: torch.Tensor, subsample: float) -> torch.Tensor:
    """[B, n] in-bag mask of stage ``stage`` (mirror of gbdt.hip ``gb_in_bag``)."""
    thr = int(round(subsample * 16777216.0))
    k = _splitmix64_t((torch.as_tensor(stage, dtype=torch.int64) << 40) ^ gidx.to(torch.int64))
    h = _splitmix64_t(seeds.to(torch.int64)[:, None] ^ k[None, :])
    return ((h >> 40) & 0xFFFFFF) < thr


def _seed_u64(random_state) -> int:
    """Per-model bagging seed (the counter-based stream is ours, not sklearn's RandomState)."""
    v = 0 if random_state is None else int(random_state)
    return (v * 0x9E3779B97F4A7C15 + 0xD1B54A32D192ED03) & _M64


# ============================================================================ host mirror
class _HostKernels:
    """Plain-PyTorch mirror of gbdt.hip (same fixed-point semantics)."""

    @staticmethod
    def apply_prep(st, prev, t):
        raw, y = st.raw, st.y
        w = wp = st.w
        if st.subsample < 1.0:
            gidx = torch.arange(st.n, device=raw.device) + st.row_off
            w = st.w * bag_mask(st.seeds, t, gidx, st.subsample)
            wp = st.w * bag_mask(st.seeds, t - 1, gidx, st.subsample) if t > 0 else st.w
            st.wt = w
            if t < st.T:
                st.bagw[t] = w.double().sum(1)
        if prev is not None:
            feat, blo, value = prev
            nd = st.node
            f = feat.gather(1, nd)
            split = f >= 0
            fb = st.bins[f.clamp(min=0).long(), torch.arange(st.n, device=raw.device)[None, :].expand_as(f)]
            side = torch.where(fb.to(torch.int64) <= blo.gather(1, nd).to(torch.int64), 1, 2)
            nd = torch.where(split, 2 * nd + side, nd)
            p0 = torch.sigmoid(raw)
            r0 = y[None] - p0
            q = torch.round(wp * r0 * r0 * st.qscale).to(torch.int64) * (wp > 0)
            st.r2[t - 1].scatter_add_(1, nd, q)
            raw = raw + st.lr * value.gather(1, nd)
            st.raw = raw
            l1p = torch.where(raw > 0, raw + torch.log1p(torch.exp(-raw)), torch.log1p(torch.exp(raw)))
            dq = torch.round(wp * (-2.0) * (y[None] * raw - l1p) * st.dscale).to(torch.int64) * (wp > 0)
            st.dev[t - 1] += dq.sum(1)
        p = torch.sigmoid(st.raw)
        r = y[None] - p
        st.g = (w * r).to(torch.float32)
        st.h = (w * p * (1 - p)).to(torch.float32)
        st.node = torch.zeros_like(st.node)
        if t < st.T:
            q = torch.round(w * r * r * st.qscale).to(torch.int64) * (w > 0)
            st.r2[t][:, 0] += q.sum(1)

    @staticmethod
    def hist(st, node0, NL):
        B, n, F = st.B, st.n, st.F
        H = torch.zeros(B, NL, F, 256, 3, dtype=torch.int64, device=st.raw.device)
        qs = st.qscale
        qg = torch.round(st.g.double() * qs).to(torch.int64)
        qh = torch.round(st.h.double() * qs).to(torch.int64)
        qw = torch.round(st.wcur.double() * qs).to(torch.int64)
        for b in range(B):
            nd = st.node[b] - node0
            ok = (nd >= 0) & (nd < NL) & (st.wcur[b] > 0)
            rows = ok.nonzero().squeeze(1)
            if rows.numel() == 0:
                continue
            base = nd[rows][:, None] * (F * 256) + torch.arange(F, device=rows.device)[None, :] * 256
            idx = (base + st.bins[:, rows].t().to(torch.int64)).reshape(-1)
            flat = H[b].view(-1, 3)
            for s, q in enumerate((qg, qh, qw)):
                flat[:, s].index_add_(0, idx, q[b, rows][:, None].expand(-1, F).reshape(-1))
        return H

    @staticmethod
    def split(st, H, node0, NL, last, t):
        inv = 1.0 / st.qscale
        feat, blo, thr, value, stats = st.feat[t], st.blo[t], st.thr[t], st.value[t], st.stats[t]
        r2 = st.r2[t]
        nbins = st.bm.nbins.cpu()
        lo_val, hi_val = st.bm.lo_val.cpu(), st.bm.hi_val.cpu()
        Hc = H.cpu()
        for b in range(st.B):
            for j in range(NL):
                hn = node0 + j
                hb = Hc[b, j]
                nb0 = int(nbins[0])
                tg, th, tw = [int(hb[0, :nb0, s].sum()) for s in range(3)]
                if tw <= 0:
                    feat[b, hn] = -3
                    continue
                best = (-1.0, 1 << 30, 0)
                rk = st.frank[t, b].tolist() if st.frank is not None else list(range(st.F))
                if tw >= st.min_split_q:
                    for f in sorted(range(st.F), key=lambda f: rk[f]):   # sklearn visit order
                        nb = int(nbins[f])
                        cw = torch.cumsum(hb[f, :nb, 2], 0)[:-1]
                        cg = torch.cumsum(hb[f, :nb, 0], 0)[:-1]
                        rw, rg = tw - cw, tg - cg
                        ok = (cw.double() >= st.min_leaf_q) & (rw.double() >= st.min_leaf_q)
                        if not bool(ok.any()):
                            continue
                        dlw, drw = cw.double(), rw.double()
                        diff = drw * cg.double() - dlw * rg.double()
                        gain = torch.where(ok, diff / dlw * diff / drw, torch.full_like(dlw, -1.0))
                        k = int(torch.argmax(gain))
                        gv = float(gain[k])
                        if gv > best[0]:
                            best = (gv, f, k)
                stats[b, hn, 0], stats[b, hn, 1], stats[b, hn, 2] = tw, tg, th
                dw, dg = tw * inv, tg * inv
                imp = int(r2[b, hn]) * inv / dw - (dg / dw) ** 2
                bg, bf, bbin = best
                if not (bg >= 0 and bf < st.F and imp > 2.220446049250313e-16):
                    feat[b, hn] = -2
                    blo[b, hn] = 0
                    thr[b, hn] = -2.0
                    den = th * inv
                    value[b, hn] = 0.0 if abs(den) < 1e-150 else dg / den
                    continue
                hf = hb[bf]
                lg, lh, lw = [int(hf[:bbin + 1, s].sum()) for s in range(3)]
                hi = bbin + 1
                nbf = int(nbins[bf])
                while hi < nbf - 1 and int(hf[hi, 2]) == 0:
                    hi += 1
                a, c = float(hi_val[bf, bbin]), float(lo_val[bf, hi])
                tt = a / 2.0 + c / 2.0
                if tt == c or math.isinf(tt):
                    tt = a
                feat[b, hn], blo[b, hn], thr[b, hn], value[b, hn] = bf, bbin, tt, dg / dw
                L, R = 2 * hn + 1, 2 * hn + 2
                stats[b, L, 0], stats[b, L, 1], stats[b, L, 2] = lw, lg, lh
                stats[b, R, 0], stats[b, R, 1], stats[b, R, 2] = tw - lw, tg - lg, th - lh
                if last:
                    feat[b, L] = feat[b, R] = -2
                    blo[b, L] = blo[b, R] = 0
                    thr[b, L] = thr[b, R] = -2.0
                    dl, dr = lh * inv, (th - lh) * inv
                    value[b, L] = 0.0 if abs(dl) < 1e-150 else lg * inv / dl
                    value[b, R] = 0.0 if abs(dr) < 1e-150 else (tg - lg) * inv / dr

    @staticmethod
    def route(st, node0, NL, t):
        nd = st.node
        f = st.feat[t].gather(1, nd)
        inl = (nd >= node0) & (nd < node0 + NL) & (f >= 0)
        fb = st.bins[f.clamp(min=0).long(), torch.arange(st.n, device=nd.device)[None, :].expand_as(f)]
        child = 2 * nd + torch.where(fb.to(torch.int64) <= st.blo[t].gather(1, nd).to(torch.int64), 1, 2)
        new = torch.where(inl, child, nd)
        r = torch.where(st.wcur > 0, st.g.double() / st.wcur.clamp(min=1e-30), torch.zeros_like(st.raw))
        q = torch.round(st.wcur * r * r * st.qscale).to(torch.int64) * ((st.wcur > 0) & inl)
        st.r2[t].scatter_add_(1, new, q)
        st.node = new


# ============================================================================ state
@dataclass
class _State:
    B: int
    n: int
    F: int
    T: int
    D: int
    NN: int
    lr: float
    qscale: float
    dscale: float
    min_leaf_q: float
    min_split_q: float
    bm: BinMapper
    bins: torch.Tensor
    y: torch.Tensor
    w: torch.Tensor
    raw: torch.Tensor
    g: torch.Tensor
    h: torch.Tensor
    node: torch.Tensor
    feat: torch.Tensor
    blo: torch.Tensor
    thr: torch.Tensor
    value: torch.Tensor
    stats: torch.Tensor
    r2: torch.Tensor
    dev: torch.Tensor
    subsample: float = 1.0
    seeds: Optional[torch.Tensor] = None   # [B] int64 (u64 bit patterns) bagging seeds
    row_off: int = 0                       # global index of local row 0 (DP shards)
    wt: Optional[torch.Tensor] = None      # [B, n] this stage's in-bag weights (subsample < 1)
    bagw: Optional[torch.Tensor] = None    # [T, B] Σ in-bag weight per stage (train_score_ norm.)
    frank: Optional[torch.Tensor] = None   # [T, B, F] int32 tie-break rank (sklearn visit order)
    reduced: bool = False                  # r2 / dev / bagw already global (stage path)
    peer: Optional[object] = None          # parallel.xgmi.PeerComm used by the stage loop

    @property
    def wcur(self) -> torch.Tensor:
        return self.wt if self.wt is not None else self.w


def _check_same(models, attrs):
    for a in attrs:
        vals = {repr(getattr(m, a)) for m in models}
        if len(vals) != 1:
            raise ValueError(f"batched GBDT fit needs identical '{a}' across models: {vals}")


def fit_gbdt_batch(models, X: torch.Tensor, y: torch.Tensor, masks: Optional[torch.Tensor] = None,
                   group=None, binned: Optional[tuple] = None, deferred=None, finish=None,
                   state_out: Optional[dict] = None):
    """Fit ``len(models)`` GBDTs on row subsets ``masks[b]`` (bool [B, n]) of one matrix.

    ``group``: torch.distributed process group when rows are sharded across ranks
    (histograms / node sums / deviance are all-reduced; results are bit-identical
    to the single-device fit).  ``binned``: optional precomputed ``(BinMapper, bins)``.
    ``deferred`` (:class:`hfens.utils.guards.Deferred`, single process on the GPU): the input and
    leaf-value guards are queued on it instead of read here — the fit is then enqueued with no host
    synchronisation at all (the stacking trainer reads them once after the SVC).  ``finish``: the
    model indices whose fitted state is built (default all; the stacking trainer keeps only the
    refit).  ``state_out``: receives the device state (node tables, prior log-odds) for device
    out-of-fold predictions.
    """
    m0 = models[0]
    _check_same(models, ("n_estimators", "learning_rate", "max_depth", "min_samples_leaf",
                         "min_samples_split", "subsample", "max_bins", "loss", "criterion"))
    if m0.loss not in ("deviance", "log_loss") or m0.criterion != "friedman_mse":
        raise NotImplementedError("binomial deviance with friedman_mse only")
    if m0.max_features not in (None, "auto"):
        raise NotImplementedError("max_features is not supported by the batched fit")
    subsample = float(m0.subsample)
    if not 0.0 < subsample <= 1.0:
        raise ValueError("subsample must be in (0, 1]")
    from ..utils.guards import check_binary, check_finite
    from ..utils.timing import hmark
    hmark("gbc_start")
    guard = None
    dfr = deferred if (deferred is not None and X.is_cuda and group is None) else None
    if dfr is not None:
        from ..utils.guards import binary_flag, finite_flag
        dfr.flag(finite_flag(X), "finite", "GradientBoostingClassifier.fit X")
        dfr.flag(binary_flag(y), "binary", "GradientBoostingClassifier.fit y")
    elif binned is None and X.is_cuda:
        # deferred: read with the bin fit's first transfer (one host sync instead of three)
        from ..utils.guards import binary_flag, finite_flag
        guard = ([finite_flag(X), binary_flag(y)],
                 [("finite", "GradientBoostingClassifier.fit X"), ("binary", "GradientBoostingClassifier.fit y")])
    else:
        check_finite(X, "GradientBoostingClassifier.fit X")
        check_binary(y, "GradientBoostingClassifier.fit y")
    dev = X.device
    n, F = X.shape
    B = len(models)
    T, D = int(m0.n_estimators), int(m0.max_depth)
    if not 1 <= D <= 5:
        raise ValueError("max_depth must be in [1, 5]")
    NN = 2 ** (D + 1) - 1
    all_rows = masks is None and binned is None   # every model sees every row of the bin map's own matrix
    if masks is None:
        masks = torch.ones(B, n, dtype=torch.bool, device=dev)
    w = masks.to(device=dev, dtype=torch.float32).contiguous()
    yv = y.to(device=dev, dtype=torch.float32).contiguous()
    if binned is None:
        bm = fit_bins(X, int(m0.max_bins), group, guard=guard)
        bins = bm.transform(X).contiguous()
    else:
        bm, bins = binned
    hmark("gbc_binned")
    n_total = n
    if group is not None:
        from ..parallel import dist as pdist
        n_total = pdist.all_reduce_int(n, group)
    shift = _qshift(n_total)
    qscale = float(2 ** shift)
    dscale = float(2 ** 26)
    # init = log-odds of the weighted class prior (DummyClassifier 'prior')
    sw = w.double().sum(1)
    sy = (w.double() * yv.double()[None]).sum(1)
    if group is not None:
        sw, sy = pdist.all_reduce_sum_f64([sw, sy], group)
    p1 = (sy / sw).clamp(F32_EPS, 1 - F32_EPS)
    raw0 = torch.log(p1 / (1 - p1))
    st = _State(
        B=B, n=n, F=F, T=T, D=D, NN=NN, lr=float(m0.learning_rate), qscale=qscale, dscale=dscale,
        min_leaf_q=float(m0.min_samples_leaf) * qscale, min_split_q=float(m0.min_samples_split) * qscale,
        bm=bm, bins=bins, y=yv, w=w, raw=raw0[:, None].expand(B, n).contiguous(),
        g=torch.empty(B, n, dtype=torch.float32, device=dev), h=torch.empty(B, n, dtype=torch.float32, device=dev),
        node=torch.zeros(B, n, dtype=torch.int64 if not X.is_cuda else torch.int32, device=dev),
        feat=torch.full((T, B, NN), -3, dtype=torch.int32, device=dev),
        blo=torch.zeros(T, B, NN, dtype=torch.int32, device=dev),
        thr=torch.full((T, B, NN), -2.0, dtype=torch.float64, device=dev),
        value=torch.zeros(T, B, NN, dtype=torch.float64, device=dev),
        stats=torch.zeros(T, B, NN, 4, dtype=torch.int64, device=dev),
        r2=torch.zeros(T, B, NN, dtype=torch.int64, device=dev),
        dev=torch.zeros(T, B, dtype=torch.int64, device=dev))
    if subsample < 1.0:
        st.subsample = subsample
        st.seeds = torch.tensor([_seed_u64(m.random_state) - (1 << 64) if _seed_u64(m.random_state) >= 1 << 63
                                 else _seed_u64(m.random_state) for m in models], dtype=torch.int64, device=dev)
        st.wt = torch.empty_like(w)
        st.bagw = torch.zeros(T, B, dtype=torch.float64, device=dev)
        if group is not None:
            from ..parallel import dist as pdist
            st.row_off = pdist.row_offset(n, group, dev)[0]
    if D == 1 and SKLEARN_TIES and subsample == 1.0 and all(
            isinstance(m.random_state, (int, np.integer)) for m in models):
        if X.is_cuda and group is None and DEVICE_RANKS and F <= 128:
            st.frank = stump_ranks_device(models, bins, w, T)
        else:
            st.frank = sklearn_stump_ranks(models, bins, masks.to(dev), T, group,
                                           nb_host=bm.nb_host if (all_rows and group is None) else None)
    hmark("gbc_ranks")
    # (a persistent loop's barrier fallback needs a host read: under a deferred read only when the
    # caller handles it, PERSIST_STACK — the stacking trainer registers the loop's error word)
    st.no_persist = dfr is not None and not (PERSIST_STACK and state_out is not None)
    st.force_persist = dfr is not None and PERSIST_STACK and state_out is not None
    if X.is_cuda:
        _run_device(st, group)
    else:
        _run_host(st, group)
    hmark("gbc_enqueued")
    if dfr is not None:
        from ..utils.guards import finite_flag
        dfr.flag(finite_flag(st.value), "finite", "GBDT leaf values")
        # the fitted state (node tables → model attributes) is built by the caller after its
        # deferred read: building it here could queue blocking host→device copies behind the
        # stage loop on this stream, i.e. wait for it
        fin = lambda: _finish(models, st, sw, p1, group, only=finish)   # noqa: E731
        if state_out is None:
            fin()
        else:
            state_out.update(st=st, raw0=raw0, T=T, NN=NN, lr=float(m0.learning_rate), finish=fin)
        hmark("gbc_finished")
        return models
    check_finite(st.value, "GBDT leaf values")
    hmark("gbc_guarded")
    if getattr(st, "persist_err", None) is not None and int(st.persist_err.item()) != 0:
        # a grid-barrier wait of the persistent loop passed its deadline (sibling workgroups not
        # dispatched in time: CUs held by another stream's or process's kernels) — the trees are
        # partial.  Re-run the fit launch per stage (no co-residency needed): same trees, bit for bit.
        if _PERSIST_OFF[0]:
            raise RuntimeError("GBDT persistent stage loop: a grid-barrier wait passed its deadline")
        import warnings
        warnings.warn("GBDT persistent stage loop: a grid-barrier wait passed its deadline; "
                      "re-running with one launch per stage", RuntimeWarning, stacklevel=2)
        LAST_PATH["persist_fallback"] = LAST_PATH.get("persist_fallback", 0) + 1
        _PERSIST_OFF[0] = True
        try:
            return fit_gbdt_batch(models, X, y, None if all_rows else masks, group=group, binned=binned)
        finally:
            _PERSIST_OFF[0] = False
    if getattr(st, "peer", None) is not None:
        st.peer.check()     # (after the guard's host read: no extra synchronisation point)
    _finish(models, st, sw, p1, group, only=finish)
    if state_out is not None:
        state_out.update(st=st, raw0=raw0, T=T, NN=NN, lr=float(m0.learning_rate))
    hmark("gbc_finished")
    return models


# sklearn's tie-break between features with EXACTLY equal split gain: its
# BestSplitter visits features in a per-node Fisher-Yates order drawn from the tree's rand_r state
# and keeps the first strictly better one.  Depth-1 trees with an int random_state and no
# subsampling reproduce that order (ops/csrc/host.hip sklearn_stump_ranks); otherwise ties go to
# the lowest feature index.
SKLEARN_TIES = os.environ.get("HFENS_GBDT_SKLEARN_TIES", "1") != "0"
RAND_R_MAX = 2147483647


def sklearn_stump_ranks(models, bins: torch.Tensor, masks: torch.Tensor, T: int, group=None,
                        nb_host=None) -> torch.Tensor:
    """[T, B, F] int32: rank of each feature in sklearn's root visit order for every tree of every
    model.  Constant features (one occupied bin over the model's rows, across all ranks) are
    set aside exactly as sklearn does and never visited (rank F).  ``nb_host``: the bin counts,
    given when every model sees every row of a single-process fit — every bin of a fitted bin map
    is occupied, so the constant features are those with one bin and no device pass is needed."""
    F, n = bins.shape
    B = len(models)
    if nb_host is not None:
        const = np.repeat((np.asarray(nb_host) <= 1).astype(np.uint8)[None, :], B, axis=0)
    else:
        big = torch.iinfo(torch.int32).max
        bi = bins.to(torch.int32)
        # masked min / max per model without boolean indexing (no nonzero sync, no row gather);
        # a model with no rows keeps (big, −1): constant, as before
        bmin = torch.stack([torch.where(masks[b][None, :] > 0, bi, big).amin(1) for b in range(B)])
        bmax = torch.stack([torch.where(masks[b][None, :] > 0, bi, -1).amax(1) for b in range(B)])
        if group is not None:
            import torch.distributed as dist
            dist.all_reduce(bmin, op=dist.ReduceOp.MIN, group=group)
            dist.all_reduce(bmax, op=dist.ReduceOp.MAX, group=group)
        const = (bmax <= bmin).to(torch.uint8).cpu().numpy()
    out = np.empty((T, B, F), dtype=np.int32)
    for b, m in enumerate(models):
        # GradientBoostingClassifier._rng = RandomState(random_state); each tree's splitter draws
        # one randint(0, RAND_R_MAX) (checkpoint: MT position = n_estimators)
        seeds = _tree_seeds(int(m.random_state), T)
        rk = np.empty((T, F), dtype=np.int32)
        _stump_ranks(T, F, seeds, np.ascontiguousarray(const[b]), rk)
        out[:, b, :] = rk
    return torch.from_numpy(out).to(bins.device)


DEVICE_RANKS = os.environ.get("HFENS_GBDT_DEVICE_RANKS", "1") != "0"


@functools.lru_cache(maxsize=64)
def _tree_seeds(random_state: int, T: int) -> np.ndarray:
    """The trees' rand_r states: GradientBoostingClassifier._rng = RandomState(random_state), one
    randint(0, RAND_R_MAX) per tree (a pure function of its arguments, drawn once per process)."""
    s = np.random.RandomState(int(random_state)).randint(0, RAND_R_MAX, size=T).astype(np.int64)
    s.setflags(write=False)
    return s


def stump_ranks_device(models, bins: torch.Tensor, w: torch.Tensor, T: int) -> torch.Tensor:
    """:func:`sklearn_stump_ranks` on the device (ops/csrc/stackdev.hip gbdt_ranks_dev): each model's
    constant features from its rows' bins and every tree's visit order in one launch — no host read."""
    from .. import ops
    F, n = bins.shape
    B = len(models)
    seeds = np.stack([_tree_seeds(int(m.random_state), T) for m in models])
    from .smo import _to_dev
    sd = _to_dev(np.ascontiguousarray(seeds), bins.device)
    out = torch.empty(T, B, F, dtype=torch.int32, device=bins.device)
    bc = bins.contiguous()
    wc = w.to(torch.float32).contiguous()
    ops.ext().gbdt_ranks_dev(T, B, F, n, bc.data_ptr(), n, wc.data_ptr(), sd.data_ptr(), out.data_ptr(),
                             ops.stream_ptr(bins.device))
    return out


def _stump_ranks(T, F, seeds, const, out):
    from .. import ops
    if ops.has_ext():
        ops.ext().sklearn_stump_ranks(T, F, seeds.ctypes.data, const.ctypes.data, out.ctypes.data)
        return
    for t in range(T):
        s = int(seeds[t]) & 0xFFFFFFFF
        feats = list(range(F))
        out[t] = F
        f_i, n_found, n_total, visited, pos = F, 0, 0, 0, 0
        while f_i > n_total and (visited < F or visited <= n_found):
            visited += 1
            if s == 0:
                s = 1
            s ^= (s << 13) & 0xFFFFFFFF
            s ^= s >> 17
            s ^= (s << 5) & 0xFFFFFFFF
            f_j = (s % (RAND_R_MAX + 1)) % (f_i - n_found) + n_found
            cur = feats[f_j]
            if const[cur]:
                feats[f_j], feats[n_total] = feats[n_total], cur
                n_found += 1
                n_total += 1
                continue
            f_i -= 1
            feats[f_j], feats[f_i] = feats[f_i], cur
            out[t, cur] = pos
            pos += 1


def _run_host(st: _State, group):
    K = _HostKernels
    st.node = st.node.to(torch.int64)
    for t in range(st.T + 1):
        prev = None
        if t > 0:
            prev = (st.feat[t - 1].to(torch.int64), st.blo[t - 1].to(torch.int64), st.value[t - 1])
        snap = st.r2[t - 1].clone() if (group is not None and t > 0) else None
        K.apply_prep(st, prev, t)
        if snap is not None:
            # the previous tree's leaf Σw r² is a rank-local partial: reduce it with this stage's
            # root slot in ONE collective (the device launch path does the same)
            delta = st.r2[t - 1] - snap
            red = torch.cat([st.r2[t], delta]) if t < st.T else delta
            pdist_all_reduce(red, group)
            st.r2[t - 1] = snap + red[-st.B:]
            if t < st.T:
                st.r2[t] = red[:st.B]
        elif group is not None:
            _allreduce_r2(st, t, group)
        if t == st.T:
            break
        for level in range(st.D):
            node0, NL = 2 ** level - 1, 2 ** level
            H = K.hist(st, node0, NL)
            if group is not None:
                from ..parallel import dist as pdist
                pdist.all_reduce_sum_(H, group)
            K.split(st, H, node0, NL, level == st.D - 1, t)
            if level < st.D - 1:
                snap = st.r2[t].clone() if group is not None else None
                K.route(st, node0, NL, t)
                if group is not None:
                    _reduce_delta(st.r2[t], snap, group)


def pdist_all_reduce(t, group):
    from ..parallel import dist as pdist
    pdist.all_reduce_sum_(t, group)


def _reduce_delta(buf, snap, group):
    """``buf`` = global ``snap`` + this rank's new contributions → global: only the delta is
    reduced (re-reducing ``buf`` would multiply its already-global entries by the world size)."""
    delta = buf - snap
    pdist_all_reduce(delta, group)
    buf.copy_(snap + delta)


def _allreduce_r2(st, t, group):
    from ..parallel import dist as pdist
    pdist.all_reduce_sum_(st.r2[t], group)


# Depth-1 trees on up to FUSED_MAX_ROWS rows (one process) train in ONE launch
# (gbdt.hip ``gbdt_stumps_fused``: a workgroup per model runs every stage's apply/hist/split with
# the same fixed-point sums — bit-identical to the launch-per-step loop below, without its 4
# launches and host round trips per stage).
FUSED_STUMPS = os.environ.get("HFENS_GBDT_FUSED", "1") != "0"
FUSED_MAX_ROWS = int(os.environ.get("HFENS_GBDT_FUSED_ROWS", str(1 << 16)))
_FUSED_LDS = 120 * 1024
LAST_PATH = {"path": None}


def _fused_ok(st: _State, group) -> bool:
    nbh = st.bm.nb_host
    return (FUSED_STUMPS and STUMP_PATH != "launch" and group is None and st.D == 1 and st.F <= 128 and st.n <= FUSED_MAX_ROWS
            and nbh is not None and 24 * int(nbh.sum()) <= _FUSED_LDS)


def _run_fused(st: _State):
    from .. import ops
    bm = st.bm
    ops.ext().gbdt_stumps_fused(
        st.B, st.n, st.F, st.T, st.bins.data_ptr(), bm.nbins.data_ptr(), int(bm.nb_host.sum()),
        bm.lo_val.data_ptr(), bm.hi_val.data_ptr(), st.y.data_ptr(), st.w.data_ptr(), st.raw.data_ptr(),
        st.g.data_ptr(), st.h.data_ptr(), st.wt.data_ptr() if st.wt is not None else 0,
        st.seeds.data_ptr() if st.seeds is not None else 0, st.row_off, st.subsample,
        st.feat.data_ptr(), st.blo.data_ptr(), st.thr.data_ptr(), st.value.data_ptr(), st.stats.data_ptr(),
        st.r2.data_ptr(), st.dev.data_ptr(), st.bagw.data_ptr() if st.bagw is not None else 0,
        st.lr, st.qscale, st.dscale, st.min_leaf_q, st.min_split_q, ops.stream_ptr(st.raw.device))


# Depth-1 trees (any row count, single process or data parallel): one gbdt_stump_stage launch per
# boosting stage over (row tiles × models) workgroups + one int64 all-reduce per stage under DP.
STUMP_PATH = os.environ.get("HFENS_GBDT_STUMPS", "stage")     # stage | fused | launch
_STAGE_LDS = 150 * 1024
COLLECTIVES = {"per_stage": None}
# Stage-loop HIP graphs: "auto" = on for the device stage path when no stamps are
# collected and the process group (if any) is NCCL/RCCL (capturable collectives); "0" / "1".
STAGE_GRAPH = os.environ.get("HFENS_GBDT_GRAPH", "auto")
GRAPH_MIN_STAGES = 9
GRAPH_INFO: dict = {}
_GRAPH_KEEP: list = []


def _graph_units(st, group, prof, peer=None) -> int:
    if STAGE_GRAPH == "0" or prof is not None or st.T + 2 < GRAPH_MIN_STAGES:
        return 0
    if group is not None:
        import torch.distributed as dist
        if peer is None and dist.get_backend(group) != "nccl":
            return 0     # gloo collectives cannot be captured; peer kernels and RCCL can
        if not validate_stage_graph(group, st.raw.device, peer):
            return 0     # the group's replayed collectives disagreed with eager ones: eager loop
    elif STAGE_GRAPH != "1":
        return 0     # single process: the eager loop is GPU-bound already (measured), keep it
    # units of 3 stages t ≡ 0, 1, 2 (mod 3) while every stage of the unit still all-reduces (t ≤ T)
    return (st.T + 1) // 3


# First-use validation of the stage graph under a process group: a 3-stage unit of
# just the per-stage reduction (device stage counter tick + the peer kernel or the captured RCCL
# all-reduce, the slots rotating as in the fit) is captured once and replayed twice on
# rank-specific int64 payloads; the results must equal eager all-reduces of the same payloads bit
# for bit on every rank.  All ranks agree (MIN) and keep the graph or run the stage loop eagerly
# together; the outcome is logged and kept in GRAPH_PROBES.  HFENS_GBDT_GRAPH_PROBE_CORRUPT=<rank>
# perturbs that rank's replayed result (tests of the fallback).
GRAPH_PROBES: dict = {}


def validate_stage_graph(group, dev, peer) -> bool:
    import logging
    import torch.distributed as dist
    from .. import ops, runtime
    key = (id(group), id(peer) if peer is not None else 0)
    if key in GRAPH_PROBES:
        return GRAPH_PROBES[key]["ok"]
    W, me = dist.get_world_size(group), dist.get_rank(group)
    E = ops.ext()
    m, reps = 3 * 1024 + 5, 2
    if peer is not None:
        m = min(m, int(peer.cap))     # (one stage slot of the group's peer buffers)
    lib_dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else dev
    buf = torch.zeros(3 * m, dtype=torch.int64, device=dev)
    tdev = torch.zeros(1, dtype=torch.int32, device=dev)
    base = peer.epoch if peer is not None else 0

    def payload(rank, r):
        g = np.random.default_rng(0xB0057 + 104729 * rank + r)
        return torch.from_numpy(g.integers(-(1 << 40), 1 << 40, 3 * m, dtype=np.int64))
    ok, detail = True, ""
    fail_local = os.environ.get("HFENS_GBDT_GRAPH_PROBE_RAISE", "")
    g = None
    # Every rank issues the same collective sequence whatever fails locally: (1) the
    # capture is local; (2) one MIN agreement on it — only a group whose every rank captured
    # replays (a replayed RCCL all-reduce needs every rank's replay); (3) the eager references and
    # the final agreement run on every rank.
    try:
        if fail_local != "" and int(fail_local) == me:
            raise RuntimeError("HFENS_GBDT_GRAPH_PROBE_RAISE")
        cap = runtime.stream(dev, "gbdt_graph")
        cur = torch.cuda.current_stream(dev)
        cap.wait_stream(cur)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(cap):
            s = ops.stream_ptr(dev)
            g.capture_begin(capture_error_mode="thread_local")
            try:
                for k in range(3):
                    E.gbdt_stage_tick(tdev.data_ptr(), s)
                    if peer is not None:
                        peer.allreduce_(buf[k * m:(k + 1) * m], (base + k + 1) % 3, k, tdev, epoch_base=base, stream=s)
                    else:
                        dist.all_reduce(buf[k * m:(k + 1) * m], op=dist.ReduceOp.SUM, group=group)
            finally:
                g.capture_end()
    except RuntimeError as e:
        ok, detail, g = False, f"rank {me}: capture: {e}", None
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=lib_dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    captured = bool(int(flag.item()))
    if captured:
        got = []
        try:
            for r in range(reps):
                buf.copy_(payload(me, r).to(dev))
                g.replay()
                torch.cuda.synchronize(dev)
                got.append(buf.cpu())
            corrupt = os.environ.get("HFENS_GBDT_GRAPH_PROBE_CORRUPT", "")
            if corrupt != "" and int(corrupt) == me:
                got[-1][m + 7] += 1
        except RuntimeError as e:
            ok, detail = False, f"rank {me}: replay: {e}"
        if peer is not None:
            peer.advance(3 * reps)
            try:
                peer.check()      # (collective: every rank calls it; it raises after its all-reduce)
            except RuntimeError as e:
                ok, detail = False, f"rank {me}: {e}"
        for r in range(reps):
            ref = payload(me, r).to(lib_dev)
            dist.all_reduce(ref, op=dist.ReduceOp.SUM, group=group)
            if ok and not torch.equal(got[r], ref.cpu()):
                ok, detail = False, f"rank {me}: replay {r}: {int((got[r] != ref.cpu()).sum())} of {3 * m} differ"
    del g
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=lib_dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    notes = [None] * W
    dist.all_gather_object(notes, detail, group=group)
    joint = bool(int(flag.item()))
    GRAPH_PROBES[key] = dict(ok=joint, world=W, peer=peer is not None, mismatches=[d for d in notes if d])
    log = logging.getLogger("hfens.gbdt")
    if joint:
        log.info("GBDT stage graph validated against eager reductions (world %d, %s)", W,
                 "peer kernel" if peer is not None else "RCCL")
    else:
        log.warning("GBDT stage graph disagrees with eager reductions: %s — eager stage loop",
                    "; ".join(GRAPH_PROBES[key]["mismatches"]))
    return joint


def _prune_graphs():
    while _GRAPH_KEEP and _GRAPH_KEEP[0][1].query():
        _GRAPH_KEEP.pop(0)
PROFILE_STAGE_T = int(os.environ.get("HFENS_GBDT_STAGE_PROF", "-1"))   # stage whose s_memtime stamps to keep
# Persistent stage loop (the per-stage floor): ONE gbdt_stump_stage launch runs every
# boosting stage with a per-model device barrier between stages instead of a launch per stage.
# Measured (scripts/probes/gbdt_persist_probe.py, profiles/r4_gbdt_persist.md): 43.9 → 35.3 µs per
# stage at 125k rows × 1 model (123 workgroups), no gain at ≥ 205 workgroups (125k × 5, 1M × 1:
# the stage body, not the launch boundary, is the cost there).  "auto" = single process, no stamps,
# ≥ PERSIST_MIN_ROWS rows (small fits run beside the SVC's spinning SMO members in the stacking
# trainer and keep the launches) and ≤ PERSIST_MAX_WGS workgroups; "1" / "0" force it on / off.
PERSIST = os.environ.get("HFENS_GBDT_PERSIST", "auto")
PERSIST_MIN_ROWS = int(os.environ.get("HFENS_GBDT_PERSIST_MIN_ROWS", "65536"))
PERSIST_MAX_WGS = int(os.environ.get("HFENS_GBDT_PERSIST_MAX_WGS", "128"))
# the stacking trainer's deferred (no host read) GBC batch as ONE persistent launch too, whatever its
# size (the headline's 10k rows × 6 models: 60 workgroups, 100 stage launches otherwise); its barrier
# deadline word is read with the batch's deferred guards and a miss re-runs the fit per stage
# (measured on one box, profiles/r6_runs/r6m: 18.40 / 18.11 vs 19.20 / 19.21 ms / fit; gbc_done 15.0 vs
# 18.8 ms in the device timeline)
PERSIST_STACK = os.environ.get("HFENS_GBDT_PERSIST_STACK", "1") == "1"
_PERSIST_OFF = [False]     # set while a fit re-runs after a persistent-loop barrier timeout
LAST_STAGE_PROF: dict = {}


def stage_plan(n: int, B: int, hist_len: int, ncu: int) -> np.ndarray:
    """gbdt_stump_stage's launch geometry: [rows per workgroup, workgroups per model, partial
    slots used (0/1), partial buffer length in int64] (ops/csrc/gbdt.hip sg_plan)."""
    from .. import ops
    out = np.zeros(4, dtype=np.int64)
    ops.ext().gbdt_stage_plan(int(n), int(B), int(hist_len), int(ncu), out.ctypes.data)
    return out


def _stage_ok(st: _State) -> bool:
    nbh = st.bm.nb_host
    return (STUMP_PATH == "stage" and st.D == 1 and st.F <= 128 and nbh is not None
            and (3 * int(nbh.sum()) + 3 * 1088) * 8 <= _STAGE_LDS)


def _run_stage(st: _State, group):
    from .. import ops, runtime
    bm = st.bm
    dev = st.raw.device
    hist_len = int(bm.nb_host.sum())
    slot = st.B * (3 * hist_len + 8)
    comm = runtime.workspace(dev, "gbdt_stage_comm", 3 * slot, torch.int64)
    comm.zero_()
    E = ops.ext()
    s = ops.stream_ptr(dev)
    ptr = lambda x: x.data_ptr() if x is not None else 0   # noqa: E731
    # bins padded to a 1024-multiple row stride: every lane reads 16 rows of a feature with ONE
    # 16-byte load (pad bins are 0, their rows carry no weight)
    ldb = -(-st.n // 1024) * 1024
    if ldb == st.n and st.bins.data_ptr() % 16 == 0:
        binsp = st.bins
    else:
        binsp = runtime.workspace(dev, "gbdt_stage_bins", st.F * ldb, torch.uint8).view(st.F, ldb)
        binsp[:, st.n:].zero_()
        binsp[:, :st.n].copy_(st.bins)
    # per-workgroup partial slots (the kernel reduces them in a second small launch when a model
    # spans more than 16 workgroups), sized from the kernel's own launch plan (one source of truth)
    from .smo import _num_cus
    plan = stage_plan(st.n, st.B, hist_len, _num_cus(dev))
    groups, plen, uses_partials = int(plan[1]), max(1, int(plan[3])), bool(plan[2])
    partials = runtime.workspace(dev, "gbdt_stage_partials", plen, torch.int64)
    prof = torch.zeros(st.B * groups * 6, dtype=torch.int64, device=dev) if PROFILE_STAGE_T >= 0 else None
    n_coll, n_xg = [0], [0]
    # data parallel: the per-stage int64 sum goes through IPC-mapped peer buffers (one kernel, no
    # RCCL call, no host round trip: parallel/xgmi.py) when the ranks share a node, else RCCL
    peer = None
    if group is not None and dev.type == "cuda":
        from ..parallel import xgmi
        peer = xgmi.peer_comm(group, dev, slot)
    # (before the epoch base is read: a first-use graph validation takes epochs of its own)
    units = _graph_units(st, group, prof, peer)
    base = peer.epoch if peer is not None else 0

    def stage(t, host_t, t_dev=None):
        # a graph-replayed stage with a partial reduce advances the device counter inside that
        # reduce launch (one launch less per stage)
        tick_in_reduce = t_dev is not None and uses_partials and host_t <= st.T
        E.gbdt_stump_stage(host_t, st.B, st.n, st.F, st.T, binsp.data_ptr(), ldb, bm.nbins.data_ptr(), hist_len,
                           bm.lo_val.data_ptr(), bm.hi_val.data_ptr(), st.y.data_ptr(), st.w.data_ptr(),
                           st.raw.data_ptr(), ptr(st.wt), ptr(st.seeds), st.row_off, st.subsample,
                           comm.data_ptr(), st.feat.data_ptr(), st.blo.data_ptr(), st.thr.data_ptr(),
                           st.value.data_ptr(), st.stats.data_ptr(), st.r2.data_ptr(), st.dev.data_ptr(),
                           ptr(st.bagw), ptr(st.frank), partials.data_ptr(), plen, st.lr, st.qscale,
                           st.dscale, st.min_leaf_q,
                           st.min_split_q, ptr(prof) if (prof is not None and t == PROFILE_STAGE_T) else 0,
                           ptr(t_dev), int(tick_in_reduce), 0, 0, 0, s)
        if t_dev is not None and not tick_in_reduce:
            E.gbdt_stage_tick(t_dev.data_ptr(), s)
        if group is not None and (t_dev is not None or t <= st.T):
            # stage t's histogram + root Σw r² + previous tree's leaf Σw r² + deviance + bag count:
            # ONE exact int64 SUM per stage (SURVEY.md §5.8 R1/R2 merged)
            k = host_t % 3
            if peer is not None:
                # peer slot = epoch mod 3 (epoch = base + t + 1): the rotation every user of the
                # PeerComm follows, so consecutive epochs never share a slot across fits
                peer.allreduce_(comm[k * slot:(k + 1) * slot], (base + host_t + 1) % 3, t, t_dev,
                                epoch_base=base, stream=s)
                n_xg[0] += 1
            else:
                import torch.distributed as dist
                dist.all_reduce(comm[k * slot:(k + 1) * slot], op=dist.ReduceOp.SUM, group=group)
                n_coll[0] += 1

    t0 = time.perf_counter()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    persist = (group is None and prof is None and not uses_partials and st.B * groups <= _num_cus(dev)
               and not _PERSIST_OFF[0] and not getattr(st, "no_persist", False)
               and (PERSIST == "1" or (PERSIST == "auto" and getattr(st, "force_persist", False)
                                       and st.B * groups <= PERSIST_MAX_WGS)
                    or (PERSIST == "auto" and st.n >= PERSIST_MIN_ROWS and st.B * groups <= PERSIST_MAX_WGS)))
    GRAPH_INFO["persist"] = persist
    if persist:
        be = runtime.workspace(dev, "gbdt_persist_bar", st.B + 1, torch.int32)   # [B] counters, err
        be.zero_()
        E.gbdt_stump_stage(0, st.B, st.n, st.F, st.T, binsp.data_ptr(), ldb, bm.nbins.data_ptr(), hist_len,
                           bm.lo_val.data_ptr(), bm.hi_val.data_ptr(), st.y.data_ptr(), st.w.data_ptr(),
                           st.raw.data_ptr(), ptr(st.wt), ptr(st.seeds), st.row_off, st.subsample,
                           comm.data_ptr(), st.feat.data_ptr(), st.blo.data_ptr(), st.thr.data_ptr(),
                           st.value.data_ptr(), st.stats.data_ptr(), st.r2.data_ptr(), st.dev.data_ptr(),
                           ptr(st.bagw), ptr(st.frank), partials.data_ptr(), plen, st.lr, st.qscale,
                           st.dscale, st.min_leaf_q, st.min_split_q, 0, 0, 0, 1, be.data_ptr(),
                           be.data_ptr() + 4 * st.B, s)
        st.persist_err = be[st.B:st.B + 1]
        GRAPH_INFO.update(units=0, stages_eager=0, host_s=time.perf_counter() - t0)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        GRAPH_INFO["loop_events"] = (ev0, ev1)
        COLLECTIVES["per_stage"] = 0.0
        COLLECTIVES["xgmi_per_stage"] = 0.0
        st.reduced = True
        return
    if units:
        # HIP graph of one 3-stage unit (stage kernel [+ partial reduce] + counter tick [+ the
        # stage's all-reduce], × 3 — the comm slots rotate with period 3), captured once per fit
        # on a side stream and replayed for t = 0 … 3·units−1; the stage index comes from device
        # memory, so every replay advances the boosting.  The last stages run eagerly.
        tdev = runtime.workspace(dev, "gbdt_stage_t", 1, torch.int32)
        tdev.zero_()
        cap = runtime.stream(dev, "gbdt_graph")
        cur = torch.cuda.current_stream(dev)
        cap.wait_stream(cur)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(cap):
            s = ops.stream_ptr(dev)
            g.capture_begin(capture_error_mode="thread_local")
            try:
                for k in range(3):
                    stage(k, k, tdev)
            finally:
                g.capture_end()
        s = ops.stream_ptr(dev)
        for _ in range(units):
            g.replay()
        if group is not None:   # the capture issued one unit's worth
            (n_xg if peer is not None else n_coll)[0] = 3 * units
        GRAPH_INFO.update(units=units, nodes_per_unit=3, stages_eager=st.T + 2 - 3 * units)
        start = 3 * units
        keep_graph = g
    else:
        start = 0
        keep_graph = None
        GRAPH_INFO.update(units=0, stages_eager=st.T + 2)
    for t in range(start, st.T + 2):
        stage(t, t)
    GRAPH_INFO["host_s"] = time.perf_counter() - t0
    ev1 = torch.cuda.Event(enable_timing=True)
    ev1.record()
    GRAPH_INFO["loop_events"] = (ev0, ev1)   # device time of the stage loop (read after a sync)
    if keep_graph is not None:
        # the graph's launches must not outlive it: keep it referenced until the work is done
        _GRAPH_KEEP.append((keep_graph, torch.cuda.Event()))
        _GRAPH_KEEP[-1][1].record()
        _prune_graphs()
    n_coll = n_coll[0]
    COLLECTIVES["per_stage"] = n_coll / (st.T + 1) if group is not None else 0.0
    COLLECTIVES["xgmi_per_stage"] = n_xg[0] / (st.T + 1) if group is not None else 0.0
    if peer is not None:
        peer.advance(st.T + 2)
        st.peer = peer
    if prof is not None:
        LAST_STAGE_PROF["stamps"] = prof.view(-1, 6).cpu().numpy()
    st.reduced = True      # r2 / dev / bagw were booked from the all-reduced slots


def _run_device(st: _State, group):
    from .. import ops
    from ..ops import stream_ptr
    if _stage_ok(st):
        LAST_PATH["path"] = "stage"
        return _run_stage(st, group)
    st.frank = None   # the fused / launch kernels break ties by the lowest feature index
    if _fused_ok(st, group):
        LAST_PATH["path"] = "fused"
        return _run_fused(st)
    LAST_PATH["path"] = "launch"
    E = ops.ext()
    s = stream_ptr(st.raw.device)
    max_nb = st.bm.max_nb
    nb_ptr = st.bm.nbins.data_ptr()
    H = torch.empty(st.B * (2 ** (st.D - 1)) * st.F * 256 * 3, dtype=torch.int64, device=st.raw.device)
    scratch = torch.zeros(st.B, st.NN, dtype=torch.int64, device=st.raw.device)
    wt_ptr = st.wt.data_ptr() if st.wt is not None else 0
    seeds_ptr = st.seeds.data_ptr() if st.seeds is not None else 0
    wcur = st.wcur
    # under data parallelism the previous tree's leaf Σw r² (added by apply_prep) goes to a scratch
    # that is reduced in the SAME collective as this stage's root slot, then booked
    leafacc = torch.zeros(st.B, st.NN, dtype=torch.int64, device=st.raw.device) if group is not None else None
    for t in range(st.T + 1):
        if t > 0:
            pf, pb, pv = st.feat[t - 1], st.blo[t - 1], st.value[t - 1]
            if leafacc is not None:
                leafacc.zero_()
            prev = (pf.data_ptr(), pb.data_ptr(), pv.data_ptr(),
                    (leafacc if leafacc is not None else st.r2[t - 1]).data_ptr(), st.dev[t - 1].data_ptr())
        else:
            prev = (0, 0, 0, 0, 0)
        cur_r2 = st.r2[t] if t < st.T else scratch
        E.gbdt_apply_prep(st.B, st.n, st.F, st.NN, st.bins.data_ptr(), st.y.data_ptr(), st.w.data_ptr(),
                          st.raw.data_ptr(), st.g.data_ptr(), st.h.data_ptr(), st.node.data_ptr(),
                          prev[0], prev[1], prev[2], prev[3], prev[4], cur_r2.data_ptr(), st.lr,
                          st.qscale, st.dscale, wt_ptr, st.subsample, seeds_ptr, st.row_off, t, s)
        if group is not None and t > 0:
            if t < st.T:
                red = torch.cat([st.r2[t], leafacc])
                pdist_all_reduce(red, group)
                st.r2[t].copy_(red[:st.B])
                st.r2[t - 1] += red[st.B:]
            else:
                pdist_all_reduce(leafacc, group)
                st.r2[t - 1] += leafacc
        elif group is not None and t == 0:
            _allreduce_r2(st, t, group)
        if t == st.T:
            break
        if st.bagw is not None:
            st.bagw[t] = st.wt.double().sum(1)
        for level in range(st.D):
            node0, NL = 2 ** level - 1, 2 ** level
            Hl = H[: st.B * NL * st.F * 768]
            Hl.zero_()
            E.gbdt_hist(st.B, st.n, st.F, st.bins.data_ptr(), nb_ptr, max_nb, st.g.data_ptr(),
                        st.h.data_ptr(), wcur.data_ptr(), st.node.data_ptr(), node0, NL, Hl.data_ptr(),
                        st.qscale, s)
            if group is not None:
                from ..parallel import dist as pdist
                pdist.all_reduce_sum_(Hl, group)
            E.gbdt_split(st.B, st.F, st.NN, Hl.data_ptr(), nb_ptr, st.bm.lo_val.data_ptr(),
                         st.bm.hi_val.data_ptr(), node0, NL, int(level == st.D - 1), st.min_leaf_q,
                         st.min_split_q, st.qscale, st.feat[t].data_ptr(), st.blo[t].data_ptr(),
                         st.thr[t].data_ptr(), st.value[t].data_ptr(), st.stats[t].data_ptr(),
                         st.r2[t].data_ptr(), s)
            if level < st.D - 1:
                snap = st.r2[t].clone() if group is not None else None
                E.gbdt_route(st.B, st.n, st.NN, st.bins.data_ptr(), st.g.data_ptr(), wcur.data_ptr(),
                             st.node.data_ptr(), st.feat[t].data_ptr(), st.blo[t].data_ptr(),
                             st.r2[t].data_ptr(), node0, NL, st.qscale, s)
                if group is not None:
                    _reduce_delta(st.r2[t], snap, group)


def _finish(models, st: _State, sw, p1, group, only=None):
    if group is not None and not st.reduced:
        from ..parallel import dist as pdist
        pdist.all_reduce_sum_(st.dev, group)
    inv = 1.0 / st.qscale
    stats = st.stats.double() * inv            # [T,B,NN,4]
    r2 = st.r2.double() * inv
    wsum = stats[..., 0]
    mean = stats[..., 1] / wsum.clamp(min=1e-300)
    imp = (r2 / wsum.clamp(min=1e-300) - mean * mean).clamp(min=0.0)
    imp = torch.where(wsum > 0, imp, torch.zeros_like(imp))
    if st.bagw is not None:
        bagw = st.bagw
        if group is not None and not st.reduced:
            from ..parallel import dist as pdist
            bagw = pdist.all_reduce_sum_f64([bagw], group)[0]
        train_score = (st.dev.double() / st.dscale) / bagw.clamp(min=1e-300)
    else:
        train_score = (st.dev.double() / st.dscale) / sw[None, :]
    heap_l = torch.arange(st.NN, device=st.feat.device) * 2 + 1
    for b, m in enumerate(models):
        if only is not None and b not in only:
            continue
        feat = st.feat[:, b]
        leaf = feat < 0
        left = torch.where(leaf, torch.full_like(heap_l, -1), heap_l[None].expand(st.T, -1))
        right = torch.where(leaf, torch.full_like(heap_l, -1), heap_l[None].expand(st.T, -1) + 1)
        m.set_fitted(feature=torch.where(feat == -3, torch.full_like(feat, -2), feat),
                     threshold=st.thr[:, b], left=left, right=right, value=st.value[:, b],
                     impurity=imp[:, b], n_node_samples=torch.round(wsum[:, b]).to(torch.int64),
                     weighted_n_node_samples=wsum[:, b], node_count=torch.full((st.T,), st.NN, device=st.feat.device),
                     class_prior=torch.stack([1 - p1[b], p1[b]]).double(), train_score=train_score[:, b],
                     n_features=st.F, rng_state=None, device=st.feat.device)
        m.tree_layout_ = "heap"
        m._bin_mapper = st.bm
        m.tree_blo_ = st.blo[:, b]        # split bin per heap node (bins ≤ blo go left)
