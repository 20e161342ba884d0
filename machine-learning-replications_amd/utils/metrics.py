"""Evaluation/reporting (reference ``train_ensemble_public.py:62-90``).

* :func:`classification_report` — sklearn's text layout at the reference's strict
  ``> 0.5`` threshold (``train_ensemble_public.py:63-64``).
* :func:`roc_curve` / :func:`roc_auc` / :func:`precision_recall_curve` /
  :func:`average_precision` — tie-aware, device-resident (sort + cumulative sums);
  ``roc_curve`` drops collinear points like sklearn's ``drop_intermediate=True``.
* :func:`wald_band` — the reference's ``±1.96·sqrt(p(1−p)/n)`` band with ``n`` =
  total held-out rows (``train_ensemble_public.py:74-77,82-85``).
* :func:`save_plots` — headless PNGs of both figures (the reference calls
  ``plt.show()``; its PR axis labels are swapped, ``:86-87`` — kept here with a
  corrected label since the plot is re-drawn, not pixel-copied).
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import numpy as np
import torch


def _t(x) -> torch.Tensor:
    return x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))


def _binary_clf_curve(y_true, score):
    y = _t(y_true).to(torch.float64).reshape(-1)
    s = _t(score).to(torch.float64).reshape(-1).to(y.device)
    order = torch.argsort(s, descending=True, stable=True)
    s, y = s[order], y[order]
    distinct = torch.nonzero(s[1:] != s[:-1]).squeeze(1)
    thr_idx = torch.cat([distinct, torch.tensor([y.numel() - 1], device=y.device)])
    tps = torch.cumsum(y, 0)[thr_idx]
    fps = 1 + thr_idx.to(torch.float64) - tps
    return fps, tps, s[thr_idx]


def roc_curve(y_true, score, drop_intermediate: bool = True):
    fps, tps, thr = _binary_clf_curve(y_true, score)
    if drop_intermediate and fps.numel() > 2:
        d2f = fps[2:] - 2 * fps[1:-1] + fps[:-2]
        d2t = tps[2:] - 2 * tps[1:-1] + tps[:-2]
        keep = torch.cat([torch.tensor([True], device=fps.device),
                          (d2f != 0) | (d2t != 0), torch.tensor([True], device=fps.device)])
        fps, tps, thr = fps[keep], tps[keep], thr[keep]
    z = torch.zeros(1, dtype=torch.float64, device=fps.device)
    fps = torch.cat([z, fps])
    tps = torch.cat([z, tps])
    thr = torch.cat([torch.full((1,), float("inf"), dtype=torch.float64, device=fps.device), thr])
    fpr = fps / fps[-1] if fps[-1] > 0 else torch.full_like(fps, float("nan"))
    tpr = tps / tps[-1] if tps[-1] > 0 else torch.full_like(tps, float("nan"))
    return fpr, tpr, thr


def auc(x, y) -> float:
    x, y = _t(x).to(torch.float64), _t(y).to(torch.float64)
    return float(torch.trapezoid(y, x))


def roc_auc(y_true, score) -> float:
    fpr, tpr, _ = roc_curve(y_true, score, drop_intermediate=False)
    return auc(fpr, tpr)


def roc_auc_sharded(y_local, score_local, group, bins: int = 1 << 16) -> float:
    """Exact AUROC of rows sharded over a process group without gathering them (SURVEY.md §5.8
    R8): scores are bucketed on a global [min, max] grid and every rank's per-bucket positive /
    negative counts are summed in ONE int64 all-reduce; pairs in different buckets are then
    ordered by their buckets.  Only the rows of buckets holding both classes are all-gathered; the
    pairs inside them are ordered by one sort + binary searches (ties count ½, as sklearn): O(m log m)
    in the gathered rows m, also when every score is tied into one bucket."""
    from ..parallel import dist as pdist
    import torch.distributed as dist
    y = _t(y_local).to(torch.float64).reshape(-1)
    s = _t(score_local).to(torch.float64).reshape(-1).to(y.device)
    dev = s.device
    big = torch.tensor([float("inf")], dtype=torch.float64, device=dev)
    mm = torch.cat([s.min().reshape(1) if s.numel() else big, (-s.max()).reshape(1) if s.numel() else big])
    dist.all_reduce(mm, op=dist.ReduceOp.MIN, group=group)
    lo, hi = float(mm[0]), -float(mm[1])
    width = (hi - lo) / bins if hi > lo else 1.0
    b = torch.clamp(((s - lo) / width).floor().to(torch.int64), 0, bins - 1)
    pos = y > 0.5
    cnt = torch.zeros(2, bins, dtype=torch.int64, device=dev)
    cnt[1].index_add_(0, b[pos], torch.ones_like(b[pos]))
    cnt[0].index_add_(0, b[~pos], torch.ones_like(b[~pos]))
    dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=group)
    neg_c, pos_c = cnt[0].to(torch.float64), cnt[1].to(torch.float64)
    n_pos, n_neg = float(pos_c.sum()), float(neg_c.sum())
    if n_pos == 0 or n_neg == 0:
        return float("nan")
    neg_below = torch.cumsum(neg_c, 0) - neg_c
    cross = float((pos_c * neg_below).sum())
    mixed = (pos_c > 0) & (neg_c > 0)
    mine = mixed[b]
    rows = pdist.all_gather_rows(torch.stack([s[mine], y[mine]], 1), group)
    within = 0.0
    if rows.shape[0]:
        # pairs inside a mixed bucket, by one sort: a positive beats the negatives of its bucket
        # with a lower score (ties ½); negatives of lower buckets are already in ``cross``.
        # Equal scores share a bucket, so the counts below never straddle one.
        sc, pos_r = rows[:, 0], rows[:, 1] > 0.5
        bb = torch.clamp(((sc - lo) / width).floor().to(torch.int64), 0, bins - 1)
        neg_s, _ = torch.sort(sc[~pos_r])
        neg_b, _ = torch.sort(bb[~pos_r])
        sp, bp = sc[pos_r], bb[pos_r]
        less = torch.searchsorted(neg_s, sp, right=False)
        leq = torch.searchsorted(neg_s, sp, right=True)
        lower_buckets = torch.searchsorted(neg_b, bp, right=False)
        within = float((less - lower_buckets).sum()) + 0.5 * float((leq - less).sum())
    return (cross + within) / (n_pos * n_neg)


def precision_recall_curve(y_true, score):
    fps, tps, thr = _binary_clf_curve(y_true, score)
    ps = tps + fps
    precision = torch.where(ps > 0, tps / ps.clamp(min=1), torch.ones_like(tps))
    recall = tps / tps[-1] if tps[-1] > 0 else torch.ones_like(tps)
    # reverse so recall is decreasing, then append (precision=1, recall=0)
    precision = torch.cat([precision.flip(0), torch.ones(1, dtype=torch.float64, device=tps.device)])
    recall = torch.cat([recall.flip(0), torch.zeros(1, dtype=torch.float64, device=tps.device)])
    return precision, recall, thr.flip(0)


def average_precision(y_true, score) -> float:
    precision, recall, _ = precision_recall_curve(y_true, score)
    return float(-torch.sum(torch.diff(recall) * precision[:-1]))


def wald_band(p, n: int):
    p = _t(p).to(torch.float64)
    ci = 1.96 * torch.sqrt(p * (1 - p) / n)
    return p - ci, p + ci


def confusion(y_true, y_pred) -> Tuple[int, int, int, int]:
    yt = _t(y_true).to(torch.float64).reshape(-1) > 0.5
    yp = _t(y_pred).to(torch.float64).reshape(-1).to(yt.device) > 0.5
    tp = int((yt & yp).sum())
    tn = int((~yt & ~yp).sum())
    fp = int((~yt & yp).sum())
    fn = int((yt & ~yp).sum())
    return tn, fp, fn, tp


def classification_report(y_true, y_pred, digits: int = 2) -> str:
    """sklearn ``classification_report`` text for a binary problem."""
    tn, fp, fn, tp = confusion(y_true, y_pred)
    rows = []
    for lab, (t, f_p, f_n) in ((0.0, (tn, fn, fp)), (1.0, (tp, fp, fn))):
        prec = t / (t + f_p) if t + f_p > 0 else 0.0
        rec = t / (t + f_n) if t + f_n > 0 else 0.0
        f1 = 2 * prec * rec / (prec + rec) if prec + rec > 0 else 0.0
        rows.append((str(lab), prec, rec, f1, t + f_n))
    total = sum(r[4] for r in rows)
    acc = (tp + tn) / total if total else 0.0
    macro = [np.mean([r[k] for r in rows]) for k in (1, 2, 3)]
    weighted = [sum(r[k] * r[4] for r in rows) / total for k in (1, 2, 3)]
    headers = ["precision", "recall", "f1-score", "support"]
    width = max(len("weighted avg"), max(len(r[0]) for r in rows), digits)
    head_fmt = "{:>{width}s} " + " {:>9}" * len(headers)
    out = head_fmt.format("", *headers, width=width) + "\n\n"
    row_fmt = "{:>{width}s} " + " {:>9.{digits}f}" * 3 + " {:>9}\n"
    for r in rows:
        out += row_fmt.format(r[0], r[1], r[2], r[3], r[4], width=width, digits=digits)
    out += "\n"
    out += ("{:>{width}s} " + " {:>9}" * 2 + " {:>9.{digits}f} {:>9}\n").format(
        "accuracy", "", "", acc, total, width=width, digits=digits)
    out += row_fmt.format("macro avg", *macro, total, width=width, digits=digits)
    out += row_fmt.format("weighted avg", *weighted, total, width=width, digits=digits)
    return out


def evaluate(y_true, proba1) -> Dict[str, float]:
    yy = (_t(proba1) > 0.5).to(torch.float64)
    tn, fp, fn, tp = confusion(y_true, yy)
    return {"auroc": roc_auc(y_true, proba1), "average_precision": average_precision(y_true, proba1),
            "accuracy": (tp + tn) / max(1, tp + tn + fp + fn), "tp": tp, "fp": fp, "tn": tn, "fn": fn}


def _svg_curve(path: str, x, y, lo, hi, xlabel: str, ylabel: str, label: str, diagonal: bool) -> str:
    """Minimal dependency-free SVG line plot with a shaded ±band (headless nodes without
    matplotlib): same content as the reference figures (T:66-90)."""
    W, H, m = 480, 400, 50
    def px(v):
        return m + float(v) * (W - 2 * m)
    def py(v):
        return H - m - float(v) * (H - 2 * m)
    xs = [float(v) for v in x]
    pts = " ".join(f"{px(a):.2f},{py(b):.2f}" for a, b in zip(xs, y))
    band = " ".join(f"{px(a):.2f},{py(min(1.0, max(0.0, float(b)))):.2f}" for a, b in zip(xs, hi))
    band += " " + " ".join(f"{px(a):.2f},{py(min(1.0, max(0.0, float(b)))):.2f}"
                           for a, b in zip(reversed(xs), reversed([float(v) for v in lo])))
    parts = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{W}" height="{H}" font-family="sans-serif" font-size="12">',
             f'<rect x="{m}" y="{m}" width="{W - 2 * m}" height="{H - 2 * m}" fill="none" stroke="black"/>',
             f'<polygon points="{band}" fill="grey" fill-opacity="0.2"/>',
             f'<polyline points="{pts}" fill="none" stroke="#1f77b4" stroke-width="2"/>']
    if diagonal:
        parts.append(f'<line x1="{px(0)}" y1="{py(0)}" x2="{px(1)}" y2="{py(1)}" stroke="black" stroke-dasharray="5,4"/>')
    for t in (0.0, 0.25, 0.5, 0.75, 1.0):
        parts.append(f'<text x="{px(t) - 8:.1f}" y="{H - m + 16}">{t:g}</text>')
        parts.append(f'<text x="{m - 34}" y="{py(t) + 4:.1f}">{t:g}</text>')
    parts += [f'<text x="{W / 2 - 50}" y="{H - 12}">{xlabel}</text>',
              f'<text x="12" y="{H / 2}" transform="rotate(-90 12 {H / 2})">{ylabel}</text>',
              f'<text x="{m + 10}" y="{m + 18}">{label}</text>', "</svg>"]
    with open(path, "w") as f:
        f.write("\n".join(parts) + "\n")
    return path


def save_plots(y_true, proba1, prefix: str) -> Optional[Tuple[str, str]]:
    """ROC and PR figures with the Wald ±band (reference T:66-90; saved instead of shown).
    PNG through matplotlib when it is installed, otherwise self-contained SVG."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:
        y = _t(y_true).cpu()
        p = _t(proba1).cpu()
        n = y.numel()
        fpr, tpr, _ = roc_curve(y, p)
        lo, hi = wald_band(tpr, n)
        roc = _svg_curve(prefix + "_roc.svg", fpr, tpr, lo, hi, "False Positive Rate", "True Positive Rate",
                         f"ensemble (AUC = {auc(fpr, tpr):.2f})", True)
        prec, rec, _ = precision_recall_curve(y, p)
        lo, hi = wald_band(prec, n)
        pr = _svg_curve(prefix + "_pr.svg", rec, prec, lo, hi, "Recall", "Precision",
                        f"ensemble (AP = {average_precision(y, p):.2f})", False)
        return roc, pr
    y = _t(y_true).cpu()
    p = _t(proba1).cpu()
    n = y.numel()
    fpr, tpr, _ = roc_curve(y, p)
    lo, hi = wald_band(tpr, n)
    fig = plt.figure()
    plt.plot(fpr.numpy(), tpr.numpy(), label=f"ensemble (AUC = {auc(fpr, tpr):.2f})")
    plt.plot([0, 1], [0, 1], "k--")
    plt.fill_between(fpr.numpy(), lo.numpy(), hi.numpy(), color="grey", alpha=.2, label=r"$\pm$ 1 std. dev.")
    plt.xlim([0.0, 1.0]); plt.ylim([0.0, 1.0])
    plt.xlabel("False Positive Rate"); plt.ylabel("True Positive Rate"); plt.grid(True); plt.legend()
    roc_path = prefix + "_roc.png"
    fig.savefig(roc_path, dpi=120)
    plt.close(fig)
    prec, rec, _ = precision_recall_curve(y, p)
    lo, hi = wald_band(prec, n)
    fig = plt.figure()
    plt.plot(rec.numpy(), prec.numpy(), label=f"ensemble (AP = {average_precision(y, p):.2f})")
    plt.fill_between(rec.numpy(), lo.numpy(), hi.numpy(), color="grey", alpha=.2, label=r"$\pm$ 1 std. dev.")
    plt.xlim([0.0, 1.0]); plt.ylim([0.0, 1.0])
    plt.xlabel("Recall"); plt.ylabel("Precision"); plt.grid(True); plt.legend()
    pr_path = prefix + "_pr.png"
    fig.savefig(pr_path, dpi=120)
    plt.close(fig)
    return roc_path, pr_path
