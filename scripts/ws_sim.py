import sys, numpy as np, time
exec(open('ws.py').read().split("def ws(")[0])
def ws_gpu(q, frac, max_inner):
    a = np.zeros(l); G = -np.ones(l); outer = inner = 0; prev = np.array([], dtype=int)
    while True:
        up = np.where(pos, a < C, a > 0); low = np.where(pos, a > 0, a < C)
        f = -yv * G
        gap = (f[up].max() if up.any() else -np.inf) - (f[low].min() if low.any() else np.inf)
        if gap < eps: break
        iu = np.flatnonzero(up); il = np.flatnonzero(low)
        ku = min(q // 4, len(iu))
        su = iu[np.argsort(-f[iu], kind='stable')[:ku]]
        il2 = il[~np.isin(il, su)]
        kl = min(q // 4, len(il2))
        sl = il2[np.argsort(f[il2], kind='stable')[:kl]]
        new = np.concatenate([np.sort(su), np.sort(sl)])
        keep = prev[~np.isin(prev, new)]
        B = np.concatenate([new, keep])[:q]
        prev = new
        Q = (yv[B][:, None] * yv[B][None, :] * K[np.ix_(B, B)]).astype(np.float64)
        aB = a[B].copy(); GB = G[B].copy()
        upB = np.where(yv[B] > 0, aB < C[B], aB > 0); lowB = np.where(yv[B] > 0, aB > 0, aB < C[B])
        fb = -yv[B] * GB
        gap0 = fb[upB].max() - fb[lowB].min()
        n_in = smo_sub(Q, GB, aB, C[B], yv[B], max(eps, frac * gap0), max_inner)
        inner += n_in
        da = aB - a[B]; ch = np.flatnonzero(da != 0)
        G += yv * (K[:, B[ch]].astype(np.float64) @ (yv[B[ch]] * da[ch]))
        a[B] = aB; outer += 1
        if n_in == 0: break
    return outer, inner, gap
for q in (512, 1024, 2048):
    for frac in (0.1, 0.2):
        print(q, frac, ws_gpu(q, frac, 8 * q), flush=True)
