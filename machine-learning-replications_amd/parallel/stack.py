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


def broadcast_svc_fits(svcs, Zs, group):
    """Every rank receives fit ``f`` from its owner, rank ``f mod world`` (collectives)."""
    world, rank = pdist.dist.get_world_size(group), pdist.dist.get_rank(group)
    for f, svc in enumerate(svcs):
        src = f % world
        if rank == src:
            ts = [svc.support_, svc.support_vectors_, svc._n_support, svc._dual_coef_[0],
                  svc._intercept_, svc._probA, svc._probB, svc.class_weight_,
                  torch.tensor([svc._gamma, float(svc.shape_fit_[0]), float(svc.shape_fit_[1])],
                               dtype=torch.float64, device=svc.support_vectors_.device)]
        else:
            ts = None
        got = pdist.broadcast_tensors(ts, src, group)
        if rank != src:
            sup, sv, ns, coef, ic, pa, pb, cw, misc = got
            dev = Zs[f].device
            svc.set_fitted(support=sup.to(dev), support_vectors=sv.to(dev), n_support=ns.to(dev),
                           dual_coef_libsvm=coef.to(dev), rho=-float(ic[0]), probA=float(pa[0]),
                           probB=float(pb[0]), gamma=float(misc[0]), class_weight=cw.to(dev),
                           shape_fit=(int(misc[1]), int(misc[2])), n_features=sv.shape[1], device=dev)
    return svcs
