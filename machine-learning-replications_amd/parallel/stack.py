"""Task-parallel SVC fits for the sharded stack (SURVEY.md §2.4 "ensemble parallel",
call site R9).

An SVM dual QP is not row-separable, so the six SVC fits of a stacking fit (5 OOF
folds + refit, each = 6 SMO problems) are distributed over ranks instead (the large fits of the
Nyström + interior-point path ARE row-separable and stay row-sharded, see
``fit_svc_batch_distributed``):
every fit's (scaled) training rows are all-gathered once, fit ``f`` is solved by
rank ``f mod world`` with the batched SMO, and the fitted parameters are
broadcast back so every rank holds the full model.
"""
from __future__ import annotations

import torch

from ..models.smo import finish_svc_batch, launch_svc_batch, use_lowrank
from . import dist as pdist


def fit_svc_batch_distributed(svcs, Zs, ys, group):
    """``Zs[f]`` / ``ys[f]``: this rank's rows of fit ``f``."""
    return finish_svc_batch_distributed(launch_svc_batch_distributed(svcs, Zs, ys, group), group)


def launch_svc_batch_distributed(svcs, Zs, ys, group) -> dict:
    """Exact-solver fits: all-gather every fit's rows (collective), then enqueue this rank's fits on
    the current stream (no host sync after the SMO launch).  Large fits (:func:`use_lowrank` on the
    GLOBAL sizes) stay row-sharded instead: every rank works on every interior-point solve
    (svc_lowrank, data parallel), synchronously.  Collectives stay on the calling thread, so all
    ranks issue them in one order on one communicator."""
    sizes = pdist.all_reduce_sum_f64([torch.tensor([float(y.numel()) for y in ys], dtype=torch.float64,
                                                   device=pdist._default_device(group))], group)[0]
    if use_lowrank([int(v) for v in sizes.tolist()], int(Zs[0].shape[1]), Zs[0].device.type):
        from ..models import smo
        from ..models.svc_lowrank import fit_svc_lowrank_batch
        smo.LAST_SMO_INFO.clear()
        smo.LAST_SMO_INFO.update(solver="nystrom-ipm", problems=6 * len(svcs), max_l=int(sizes.max()),
                                 row_sharded=True)
        fit_svc_lowrank_batch(svcs, Zs, ys, group=group)
        return dict(svcs=svcs, Zs=Zs, st=None, done=True)
    world, rank = pdist.dist.get_world_size(group), pdist.dist.get_rank(group)
    full_Z = [pdist.all_gather_rows(Z, group) for Z in Zs]
    full_y = [pdist.all_gather_rows(y[:, None].to(torch.float64), group)[:, 0] for y in ys]
    mine = [f for f in range(len(svcs)) if f % world == rank]
    st = None
    if mine:
        st = launch_svc_batch([svcs[f] for f in mine], [full_Z[f] for f in mine], [full_y[f] for f in mine])
    return dict(svcs=svcs, Zs=Zs, st=st, world=world, rank=rank)


def finish_svc_batch_distributed(pre: dict, group):
    """Complete this rank's fits, then broadcast every fit from its owner (collectives)."""
    svcs, Zs = pre["svcs"], pre["Zs"]
    if pre.get("done"):
        return svcs
    if pre["st"] is not None:
        finish_svc_batch(pre["st"])
    return broadcast_svc_fits(svcs, Zs, group)


COLLECTIVES = {"broadcast_svc_fits": 0}


def broadcast_svc_fits(svcs, Zs, group):
    """Every rank receives fit ``f`` from its owner, rank ``f mod world``, in TWO collectives for
    all fits (the per-fit object broadcast + 9 tensor broadcasts were ≈ 60 RCCL
    calls per stacking fit): a SUM of an int64 shape table, then a SUM of ONE packed f64 buffer in
    which each fit's slice is written by its owner alone.  The buffer is summed as its int64 bit
    patterns (in f64, an owner's −0.0 plus the others' +0.0 would arrive as +0.0); an
    integer x + 0 = x for every pattern, so every rank ends with the owner's bits (integers below
    2^53 travel exactly in f64)."""
    world, rank = pdist.dist.get_world_size(group), pdist.dist.get_rank(group)
    dev = pdist._default_device(group)
    K = len(svcs)
    mine = [f for f in range(K) if f % world == rank]
    shp = torch.zeros(K, 4, dtype=torch.int64)
    for f in mine:
        svc = svcs[f]
        shp[f] = torch.tensor([int(svc.support_vectors_.shape[0]), int(svc.support_vectors_.shape[1]),
                               int(svc._n_support.numel()), int(svc.class_weight_.numel())])
    shp = shp.to(dev)
    pdist.dist.all_reduce(shp, op=pdist.dist.ReduceOp.SUM, group=group)
    shp = shp.cpu().tolist()
    # per fit: support | SV rows | n_support | dual coef | −ρ | A | B | class weights | γ, shape_fit
    lens = [nsv + nsv * F + ns + nsv + 3 + cw + 3 for nsv, F, ns, cw in shp]
    offs = [0]
    for v in lens:
        offs.append(offs[-1] + v)
    f64 = torch.float64
    buf = torch.zeros(offs[-1], dtype=f64, device=dev)
    for f in mine:
        svc = svcs[f]
        parts = [svc.support_.reshape(-1), svc.support_vectors_.reshape(-1), svc._n_support.reshape(-1),
                 svc._dual_coef_[0].reshape(-1), svc._intercept_.reshape(-1), svc._probA.reshape(-1),
                 svc._probB.reshape(-1), svc.class_weight_.reshape(-1),
                 torch.tensor([svc._gamma, float(svc.shape_fit_[0]), float(svc.shape_fit_[1])], dtype=f64)]
        buf[offs[f]:offs[f + 1]] = torch.cat([t.to(device=dev, dtype=f64) for t in parts])
    pdist.dist.all_reduce(buf.view(torch.int64), op=pdist.dist.ReduceOp.SUM, group=group)
    COLLECTIVES["broadcast_svc_fits"] = 2
    for f, svc in enumerate(svcs):
        if f in mine:
            continue
        nsv, F, ns, cw = shp[f]
        o = offs[f]
        take = []
        for n_ in (nsv, nsv * F, ns, nsv, 1, 1, 1, cw, 3):
            take.append(buf[o:o + n_])
            o += n_
        sup, sv, nsup, coef, ic, pa, pb, cwt, misc = take
        d = Zs[f].device
        misc = misc.cpu().tolist()
        svc.set_fitted(support=sup.to(d).to(torch.int32), support_vectors=sv.reshape(nsv, F).to(d),
                       n_support=nsup.to(d).to(torch.int32), dual_coef_libsvm=coef.to(d), rho=-float(ic[0]),
                       probA=float(pa[0]), probB=float(pb[0]), gamma=float(misc[0]), class_weight=cwt.to(d),
                       shape_fit=(int(misc[1]), int(misc[2])), n_features=F, device=d)
    return svcs
