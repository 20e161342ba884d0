"""KNN imputation (reference ``train_ensemble_public.py:37-40``:
``KNNImputer(missing_values=nan, n_neighbors=1)`` fit on the development set and
applied to both sets; semantics sklearn ``impute/_knn.py`` + ``nan_euclidean``).

For every missing cell (r, c) the donor is the fit row with column c present that
minimises the nan-euclidean distance ``F/|common|·Σ_common (x−y)²``; with no
defined distance the column mean of the fit rows is used.  Donor search runs in
the ``knn_donors`` HIP kernel (tie-break: lowest donor index; sklearn's
``argpartition`` tie order is unspecified).  ``n_neighbors > 1`` (uniform mean
over the k nearest) runs on the host path.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .base import Estimator, as_tensor

SLOTS = 8
# the donor search's filter on the bf16 matrix cores (knn.hip knn_donor_mfma_kernel; the exact
# direct-difference pass decides every slot as before, so the slots are the same bits): HFENS_KNN_MFMA
# "auto" (default) takes it from MFMA_MIN_PAIRS rows × donors — 0.35 / 0.40 / 0.70 / 6.3 / 43.6 ms
# against 0.41 / 0.42 / 1.22 / 18.0 / 142.6 ms for the packed-FMA filter at 8k / 10k / 20k / 100k /
# 300k rows (profiles/r5_knn_mfma.md); "1" always, "0" never
MFMA_FILTER = os.environ.get("HFENS_KNN_MFMA", "auto")
MFMA_MIN_PAIRS = 1 << 24
# f64-exact donors on the device (knn.hip knn_refine): the f32 search's near-ties re-decided in f64
EXACT = __import__("os").environ.get("HFENS_KNN_EXACT", "1") != "0"
KNN_DEBUG = __import__("os").environ.get("HFENS_KNN_DEBUG", "0") == "1"
# the receivers, their slots and operands planned by device kernels (knn.hip knn_plan_dev) instead
# of from a host read of the missing-value bitmasks: the donor search launches with no host round trip
DEVICE_PLAN = __import__("os").environ.get("HFENS_KNN_DEVICE_PLAN", "1") != "0"
LAST_REFINE: list = []


def _masks_u64(miss: torch.Tensor) -> torch.Tensor:
    F = miss.shape[1]
    w = (2 ** torch.arange(F, dtype=torch.int64, device=miss.device))
    bits = (miss.to(torch.int64) * w).sum(1)
    return bits


class KNNImputer(Estimator):
    _param_names = ("missing_values", "n_neighbors", "weights", "metric", "copy")

    def __init__(self, missing_values=np.nan, n_neighbors=5, weights="uniform", metric="nan_euclidean",
                 copy=True):
        self.missing_values = missing_values
        self.n_neighbors = n_neighbors
        self.weights = weights
        self.metric = metric
        self.copy = copy

    def fit(self, X):
        X = as_tensor(X)
        self._fit_X = X
        self._mask_fit = torch.isnan(X)
        self._valid = ~self._mask_fit.all(0)
        fx = torch.where(self._mask_fit, torch.zeros_like(X), X)
        cnt = (~self._mask_fit).sum(0).clamp(min=1)
        self._col_mean = fx.sum(0) / cnt
        self._keep_host = None
        return self

    def _keep(self):
        """Indices of the columns with a fit value (host array; one small read per fit, at the first
        transform — the output width must be known on the host)."""
        if self._keep_host is None:
            self._keep_host = np.nonzero(self._valid.cpu().numpy())[0].astype(np.int64)
        return self._keep_host

    def fit_transform(self, X):
        return self.fit(X).transform(X)

    def transform(self, X):
        return self.transform_many([X])[0]

    def transform_many(self, Xs, streams=None, defer=False):
        """Impute several matrices with ONE device→host read for all of them (the per-row
        missing-column bitmasks).  ``streams[i]`` (device path): the stream matrix i's donor
        search is queued on (it waits for the current stream first).  ``defer`` (device path):
        the side-stream matrices are NOT planned and launched here; the call returns
        ``(outs, run)`` and ``run()`` does it later — their host-side planning (≈ 1 ms at 10k
        rows) then runs where the caller's thread would otherwise wait on the device — and
        returns the finished list (those matrices only ever waited for this transform's inputs)."""
        Xs = [as_tensor(X, device=self._fit_X.device).clone() for X in Xs]
        if Xs and Xs[0].is_cuda and self.n_neighbors == 1:
            if DEVICE_PLAN and EXACT and Xs[0].shape[1] <= 64:
                return self._impute_planned_many(Xs, streams, defer)
            return self._impute_device_many(Xs, streams, defer)
        if defer:
            done = self.transform_many(Xs)
            return done, (lambda: done)
        for X in Xs:
            miss = torch.isnan(X)
            rows = torch.nonzero(miss.any(1)).squeeze(1)
            if rows.numel() > 0:
                self._impute_host(X, miss, rows)
        return [X[:, self._valid] for X in Xs]

    # ------------------------------------------------------------------ device
    def _fit_prep(self):
        """Donor-side operands of the kernel (centred f32 rows, missing-column bitmasks), built
        once per fit and shared by every transform."""
        pr = getattr(self, "_prep", None)
        if pr is None or pr[0] is not self._fit_X:
            D = torch.where(self._mask_fit, torch.zeros_like(self._fit_X), self._fit_X)
            center = self._col_mean  # centring improves f32 accuracy; distances are shift-invariant
            D32 = (D - center).where(~self._mask_fit, torch.zeros_like(D)).to(torch.float32).contiguous()
            dm = _masks_u64(self._mask_fit).contiguous()
            # the f64 refine's operands: raw values zero-filled (the host mirror's arithmetic) and the
            # largest centred magnitude (its error window), both left on the device
            D64 = D.to(torch.float64).contiguous()
            dmax = D32.abs().amax(0) if D32.numel() else torch.zeros(D32.shape[1], device=D.device)
            pr = self._prep = (self._fit_X, D32, dm, D64, dmax)
        return pr[1], pr[2]

    def _fit_prep64(self):
        self._fit_prep()
        return self._prep[3], self._prep[4]

    def _impute_planned_many(self, Xs, streams, defer=False):
        """:meth:`_impute_device_many` with the planning on the device (:meth:`_impute_planned`):
        nothing is read back but the fit's valid-column list (once per fit)."""
        from .smo import _to_dev
        from ..utils.timing import hmark
        dev = Xs[0].device
        F = Xs[0].shape[1]
        keep_h = self._keep()
        keep = None if keep_h.shape[0] == F else _to_dev(keep_h, dev)
        D32, dm = self._fit_prep()
        D64, dmax = self._fit_prep64()
        main = torch.cuda.current_stream(dev)
        ready = torch.cuda.Event()
        ready.record(main)
        out, jobs = [], []
        for i, X in enumerate(Xs):
            st = streams[i] if streams is not None and streams[i] is not None else None
            if st is None:
                self._impute_planned(X, D32, dm, D64, dmax)
                out.append(X if keep is None else X.index_select(1, keep))
                hmark("imp_main_enqueued")
            else:
                def job(i=i, X=X, st=st):
                    st.wait_event(ready)
                    for t in (X, D32, dm, D64, dmax, self._fit_X, self._col_mean) + ((keep,) if keep is not None else ()):
                        t.record_stream(st)
                    with torch.cuda.device(dev), torch.cuda.stream(st):
                        self._impute_planned(X, D32, dm, D64, dmax)
                        out[i] = X if keep is None else X.index_select(1, keep)
                out.append(None)
                jobs.append(job)
        if not defer:
            for job in jobs:
                job()
            return out
        state = {"done": False}

        def run():
            if not state["done"]:
                for job in jobs:
                    job()
                state["done"] = True
            return out
        return out, run

    def _impute_planned(self, X, D32, dm, D64, dmax):
        """One matrix, every step on the device: knn_plan_dev (receivers in row order, their slot
        columns in groups of 8, centred f32 / raw f64 operands, the refine's error scale, counts),
        the f32 donor search + f64 refine per slot group (kernels read the counts; groups past the
        widest row exit at once), then knn_apply writes the donors' values in place."""
        from .. import ops
        E = ops.ext()
        n, F = X.shape
        if n == 0:
            return
        dev = X.device
        s = ops.stream_ptr(dev)
        G = -(-F // SLOTS)
        Xc = X if X.is_contiguous() else X.contiguous()
        i64, i32 = torch.int64, torch.int32
        rows = torch.empty(n, dtype=i64, device=dev)
        rbits = torch.empty(n, dtype=i64, device=dev)
        slot = torch.empty(G, n, SLOTS, dtype=i32, device=dev)
        R32 = torch.empty(n, F, dtype=torch.float32, device=dev)
        R64 = torch.empty(n, F, dtype=torch.float64, device=dev)
        small = torch.empty(F + 1 + 4 + (n + 255) // 256, dtype=i32, device=dev)   # colmax | Mx | cnt | block counts
        colmax, Mx, cnt, bcnt = small[:F], small[F:F + 1], small[F + 1:F + 5], small[F + 5:]
        E.knn_plan_dev(Xc.data_ptr(), n, F, self._col_mean.data_ptr(), dmax.data_ptr(), rows.data_ptr(),
                       rbits.data_ptr(), slot.data_ptr(), G, R32.data_ptr(), R64.data_ptr(), colmax.data_ptr(),
                       Mx.data_ptr(), cnt.data_ptr(), bcnt.data_ptr(), s)
        best = torch.empty(G, n, SLOTS, dtype=i64, device=dev)
        alt = torch.empty(n, SLOTS, dtype=i32, device=dev)
        cap = max(1 << 18, 16 * n)
        work = torch.empty(4 * cap + n * SLOTS * 8 + 2 * n + 12, dtype=i32, device=dev)
        nd = D32.shape[0]
        mf = None
        use_mf = MFMA_FILTER == "1" or (MFMA_FILTER == "auto" and n * nd >= MFMA_MIN_PAIRS)
        if use_mf and F <= 48 and nd > 0:
            # the donors' bf16 operand items of the matrix-core filter, built once for every slot group
            wd = np.zeros(1, dtype=np.int64)
            E.knn_mfma_item_words(F, wd.ctypes.data)
            mf = (torch.empty(nd * int(wd[0]), dtype=torch.int32, device=dev), torch.empty(nd, dtype=torch.float32, device=dev))
            E.knn_mfma_prep(D32.data_ptr(), dm.data_ptr(), nd, F, mf[0].data_ptr(), mf[1].data_ptr(), s)
        for g in range(G):
            if mf is not None:
                E.knn_donors_mfma(R32.data_ptr(), rbits.data_ptr(), n, D32.data_ptr(), dm.data_ptr(), nd, F,
                                  slot[g].data_ptr(), best[g].data_ptr(), alt.data_ptr(), cnt.data_ptr(), g * SLOTS,
                                  mf[0].data_ptr(), mf[1].data_ptr(), s)
            else:
                E.knn_donors(R32.data_ptr(), rbits.data_ptr(), n, D32.data_ptr(), dm.data_ptr(), nd, F,
                             slot[g].data_ptr(), best[g].data_ptr(), alt.data_ptr(), cnt.data_ptr(), g * SLOTS, s)
            E.knn_refine(R32.data_ptr(), rbits.data_ptr(), n, D32.data_ptr(), dm.data_ptr(), nd, F,
                         slot[g].data_ptr(), best[g].data_ptr(), alt.data_ptr(), R64.data_ptr(), D64.data_ptr(),
                         Mx.data_ptr(), work.data_ptr(), cap, cnt.data_ptr(), g * SLOTS,
                         mf[0].data_ptr() if mf is not None else 0, mf[1].data_ptr() if mf is not None else 0, s)
        fx = self._fit_X if self._fit_X.is_contiguous() else self._fit_X.contiguous()
        E.knn_apply(Xc.data_ptr(), n, F, rows.data_ptr(), slot.data_ptr(), best.data_ptr(), fx.data_ptr(),
                    self._col_mean.data_ptr(), cnt.data_ptr(), s)
        if Xc is not X:
            X.copy_(Xc)

    def _impute_device_many(self, Xs, streams, defer=False):
        """The (row, column) work lists are built with numpy from the bitmasks and uploaded
        non-blocking, so the donor launches and the scatters queue without further host
        synchronisation."""
        F = Xs[0].shape[1]
        if F > 64:
            raise ValueError("KNNImputer device path supports at most 64 features")
        from ..utils.timing import hmark
        host = torch.cat([_masks_u64(torch.isnan(X)) for X in Xs] + [self._valid.to(torch.int64)]).cpu().numpy()
        hmark("imp_masks_read")
        bits_all = host[:-F].view(np.uint64)
        from .smo import _to_dev
        dev = Xs[0].device
        keep = _to_dev(np.nonzero(host[-F:])[0].astype(np.int64), dev)   # columns with a fit value
        D32, dm = self._fit_prep()
        main = torch.cuda.current_stream(dev)
        ready = torch.cuda.Event()
        ready.record(main)          # the inputs of every matrix: masks, fit operands, X itself
        off, out, jobs = 0, [], []
        for i, X in enumerate(Xs):
            bits = bits_all[off:off + X.shape[0]]
            off += X.shape[0]
            st = streams[i] if streams is not None and streams[i] is not None else None
            if st is None:
                self._impute_device(X, bits, D32, dm)
                out.append(X.index_select(1, keep))
                hmark("imp_main_enqueued")
            else:
                def job(i=i, X=X, bits=bits, st=st):
                    # everything that touches X — the imputation AND the column selection — is
                    # queued on st; the caller joins st before reading the result
                    st.wait_event(ready)
                    # X, keep and the fit operands were allocated on the current stream: without
                    # record_stream their blocks could be handed to new current-stream tensors while
                    # st still reads / writes them
                    for t in (X, keep, D32, dm, self._fit_X, self._col_mean):
                        t.record_stream(st)
                    with torch.cuda.device(dev), torch.cuda.stream(st):
                        self._impute_device(X, bits, D32, dm)
                        out[i] = X.index_select(1, keep)
                out.append(None)
                jobs.append(job)
        if not defer:
            for job in jobs:
                job()
            return out
        state = {"done": False}

        def run():
            if not state["done"]:
                for job in jobs:
                    job()
                state["done"] = True
            return out
        return out, run

    def _impute_device(self, X, bits, D32, dm):
        from .. import ops
        E = ops.ext()
        n, F = X.shape
        # the work lists from the rows' missing-column bitmasks, planned natively (host.hip
        # knn_plan_host) into ONE pinned buffer → one H2D copy, sliced on the device.  A counting
        # call sizes the buffer exactly (2·nr + nr·nslot + 3·nc: only the missing cells, not the
        # worst case of every cell missing)
        dev = X.device
        dims = np.zeros(4, dtype=np.int64)
        bits = np.ascontiguousarray(bits, dtype=np.uint64)
        E.knn_plan_host(bits.ctypes.data, n, F, SLOTS, 0, 0, dims.ctypes.data)
        nr, nc, nslot = (int(v) for v in dims[:3])
        if nr == 0:
            return
        cap = 2 * nr + nr * nslot + 3 * nc
        hb = torch.empty(cap, dtype=torch.int64, pin_memory=True)
        E.knn_plan_host(bits.ctypes.data, n, F, SLOTS, hb.data_ptr(), cap, dims.ctypes.data)
        if int(dims[3]) != 0 or int(dims[0]) != nr:
            raise RuntimeError(f"knn_plan_host: work-list buffer of {cap} words rejected (dims {dims.tolist()})")
        center = self._col_mean
        from ..utils.timing import hmark
        hmark("imp_plan")
        sizes = [nr, nr, nr * nslot, nc, nc, nc]
        buf = hb[:sum(sizes)].to(dev, non_blocking=True)
        o = np.concatenate([[0], np.cumsum(sizes)])
        rows, rm, slot_dev, flat, r_idx, c_idx = (buf[o[i]:o[i + 1]] for i in range(6))
        hmark("imp_h2d")
        Rm = ((rm[:, None] >> torch.arange(F, device=dev)) & 1) != 0
        slot_dev = slot_dev.view(nr, nslot).to(torch.int32)
        Xr = X.index_select(0, rows)
        R32 = torch.where(Rm, torch.zeros_like(Xr), Xr - center).to(torch.float32).contiguous()
        rm = rm.contiguous()
        best = torch.empty(nr, nslot, dtype=torch.int64, device=dev)
        alt = torch.empty(nr, SLOTS, dtype=torch.int32, device=dev)
        if EXACT:
            D64, dmax = self._fit_prep64()
            R64 = torch.where(Rm, torch.zeros_like(Xr), Xr).to(torch.float64).contiguous()
            # ‖m‖, m_f = the largest centred magnitude of column f over donors and receivers (the
            # f32 error bound of knn.hip knn_ambig)
            Mx = torch.linalg.vector_norm(torch.maximum(dmax, R32.abs().amax(0)).to(torch.float64)).reshape(1)
            Mx = Mx.to(torch.float32).contiguous()
            # knn.hip knn_refine scratch: pair keys u64 [cap] | dmin, dwin u64 | didx, didx2 i32 | thr, thr2
            # f32 per slot | pairs [2·cap] | two receiver lists | counts
            cap = max(1 << 18, 16 * nr)
            work = torch.empty(4 * cap + nr * SLOTS * 8 + 2 * nr + 12, dtype=torch.int32, device=dev)
        for s0 in range(0, nslot, SLOTS):
            slot = slot_dev[:, s0:s0 + SLOTS].contiguous()
            blk = best[:, s0:s0 + SLOTS] if nslot == SLOTS else torch.empty(slot.shape, dtype=torch.int64, device=dev)
            E.knn_donors(R32.data_ptr(), rm.data_ptr(), nr, D32.data_ptr(), dm.data_ptr(),
                         D32.shape[0], F, slot.data_ptr(), blk.data_ptr(), alt.data_ptr(), 0, 0, ops.stream_ptr(dev))
            if EXACT:
                # slots whose runner-up is within the f32 error of the best: re-decided in f64
                # (knn.hip knn_refine) — the donors then equal the host mirror's f64 choice
                E.knn_refine(R32.data_ptr(), rm.data_ptr(), nr, D32.data_ptr(), dm.data_ptr(), D32.shape[0], F,
                             slot.data_ptr(), blk.data_ptr(), alt.data_ptr(), R64.data_ptr(), D64.data_ptr(),
                             Mx.data_ptr(), work.data_ptr(), cap, 0, 0, 0, 0, ops.stream_ptr(dev))
                if KNN_DEBUG:   # re-scanned receivers, window pairs, overflow, pass-1 receivers (synchronising)
                    o = 4 * cap + 8 * nr * SLOTS + 2 * nr
                    LAST_REFINE.append((nr, int(work[o]), int(work[o + 8]), int(work[o + 9]), int(work[o + 4]),
                                        float(Mx[0])))
            if nslot != SLOTS:
                best[:, s0:s0 + SLOTS] = blk
        hmark("imp_knn_launched")
        # packed (d² float bits << 32 | donor); all-ones = no donor with a defined distance
        b = best.view(-1).index_select(0, flat)
        donor = torch.where(b == -1, torch.full_like(b, -1), b & 0xFFFFFFFF)
        vals = torch.where(donor >= 0, self._fit_X[donor.clamp(min=0), c_idx], self._col_mean[c_idx])
        X.index_put_((r_idx, c_idx), vals)

    # ------------------------------------------------------------------ host
    def _impute_host(self, X, miss, rows):
        fit = self._fit_X
        mf = self._mask_fit
        F = X.shape[1]
        D = torch.where(mf, torch.zeros_like(fit), fit)
        pres_f = (~mf).to(torch.float64)
        step = max(1, (1 << 24) // max(1, fit.shape[0] * F))
        for s in range(0, rows.numel(), step):
            rr = rows[s:s + step]
            R = X[rr]
            mr = torch.isnan(R)
            Rz = torch.where(mr, torch.zeros_like(R), R)
            pres_r = (~mr).to(torch.float64)
            # Σ_common (x−y)², direct differences in f64 summed in feature order (exact ties stay
            # ties; the device's f64 refine, knn.hip knn_dist64, does the same operations)
            both = pres_r[:, None, :] * pres_f[None, :, :]
            diff = Rz[:, None, :] - D[None, :, :]
            sq = both * (diff * diff)
            d2 = sq[..., 0].clone()
            for f in range(1, F):
                d2 = d2 + sq[..., f]
            common = both.sum(-1)
            dist = torch.where(common > 0, d2 * F / common.clamp(min=1),
                               torch.full_like(d2, float("inf")))
            for j, r in enumerate(rr.tolist()):
                for c in torch.nonzero(mr[j]).squeeze(1).tolist():
                    cand = ~mf[:, c]
                    dd = torch.where(cand, dist[j], torch.full_like(dist[j], float("inf")))
                    k = min(self.n_neighbors, int(cand.sum()))
                    if k == 0 or not torch.isfinite(dd).any():
                        X[r, c] = self._col_mean[c]
                        continue
                    if k == 1:
                        X[r, c] = fit[int(torch.argmin(dd)), c]   # first minimum = lowest index
                        continue
                    vals, idx = torch.topk(-dd, k)
                    ok = torch.isfinite(vals)
                    X[r, c] = fit[idx[ok], c].mean()
