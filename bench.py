"""Headline benchmark: training rows/s (+ held-out AUROC) of the HF-progression
stacking ensemble (BASELINE.json metric; BASELINE.md config 2 shape: synthetic
Table-S1 cohort, 40 candidate features, 10,000 development rows).

One *step* = the complete development fit of the reference pipeline
(``train_ensemble_public.py:37-61``): KNN imputation of the development rows,
LassoCV(10-fold, 100 alphas) + top-17 SelectFromModel, and the stacking fit —
SVC (Platt, 36 SMO problems), GBC (100 stumps) and L1-LR, each as 5 OOF folds +
refit, then the L2 meta-learner.  Nothing is skipped or cached inside the timed
region.  The held-out AUROC (independent synthetic draw, imputed with the fitted
imputer) is computed after timing.

Multi-GPU (``torchrun --nproc-per-node N``): strong scaling — the SAME
``--rows``-row development set is sharded over the N ranks (contiguous row
blocks) and the job trains ONE ensemble on it: KNN donors all-gathered, LassoCV
moments / GBDT fixed-point histograms / LR gradients all-reduced over RCCL, the 6
SVC fits (36 SMO problems) task-parallel over ranks.  An exact SVM is
super-linear in rows, so weak scaling (rows ∝ N) would grow per-GPU work; the
fixed-size problem is the honest multi-GPU setting for this ensemble.
``value`` = development rows × steps ÷ slowest rank's time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rows R] [--features F]

``--config gbdt`` (BASELINE config 3 analog, GBC-only row of BASELINE.md): histogram GBDT,
100 depth-1 trees, 1M synthetic rows × 40 features; DP = rows sharded over ranks with int64
fixed-point histogram all-reduces (results bit-identical for any N).  ``--config deep``
(BASELINE config 5): 1000 stumps × 5 seeds (``--subsample`` < 1 makes the seeds differ; the
CPU baseline's seeds were identical fits), metric rows·seeds/s.  Both time binning + fitting;
held-out AUROC from the folded stump-table inference kernel.

``--config infer`` (BASELINE config 4): batched inference of the shipped checkpoint
(``assets/hf_predict_model.pkl``) over 100M synthetic patient rows with the fused
whole-stack HIP kernel; one step = one pass over all rows (device-resident, HIP-graph
replay); the host-streaming (pinned H2D ∥ kernel ∥ D2H) rate is reported alongside.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CPU_BASELINE_ROWS_PER_S = 305.0   # sklearn pipeline, 10k x 40, 8-vCPU Xeon


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows", type=int, default=10000, help="development rows (whole job)")
    ap.add_argument("--features", type=int, default=40)
    ap.add_argument("--seed", type=int, default=2020)
    ap.add_argument("--timings", action="store_true", help="print a per-stage table to stderr")
    ap.add_argument("--config", default="train", choices=["train", "infer", "gbdt", "deep"])
    ap.add_argument("--trees", type=int, default=None, help="gbdt/deep: boosting stages")
    ap.add_argument("--seeds", type=int, default=None, help="gbdt/deep: models (seeds) trained together")
    ap.add_argument("--depth", type=int, default=1)
    ap.add_argument("--subsample", type=float, default=1.0)
    ap.add_argument("--dp-policy", default="auto",
                    help="gbdt/deep multi-GPU layout: auto | seeds | rows | <ranks per seed group>")
    a = ap.parse_args()
    if a.config == "infer":
        return bench_infer(a)
    if a.config in ("gbdt", "deep"):
        return bench_gbdt(a)

    import numpy as np
    import torch
    from hfens.parallel import dist as pdist
    from hfens.io.synth import make_hf_cohort
    from hfens.pipeline import develop
    from hfens.utils.timing import StageTimer
    from hfens.utils import metrics
    from hfens import ops

    # long device-bound fits (config 3: ≥ 2^18 rows) let host waits sleep instead of spin
    # (runtime.blocking_sync; HFENS_BLOCKING_SYNC=0/1 overrides)
    bs = os.environ.get("HFENS_BLOCKING_SYNC", "1" if a.rows >= (1 << 18) else "0") == "1"
    blocking = False
    if bs and torch.cuda.device_count() > 0:
        from hfens import runtime
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
        blocking = runtime.blocking_sync()
    group, rank, world = pdist.init_from_env()
    if world != a.gpus:
        if rank == 0:
            print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dev = pdist.rank_device()
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
        ops.ext()  # the HIP extension must be there; no silent fallback
        # the host side of a GPU step is bookkeeping on small arrays: intra-op thread pools only
        # wake OpenMP workers that then spin (measured: 15 workers at ~12 % CPU each, host CPU
        # fraction 2.9 — they compete with the submitting thread on a loaded box)
        torch.set_num_threads(int(os.environ.get("HFENS_HOST_THREADS", "1")))
    # strong scaling: every rank draws the same cohort and keeps its contiguous row block
    Xd, yd, names = make_hf_cohort(a.rows, a.features, seed=a.seed, nan_frac=0.02)
    Xs, ys, _ = make_hf_cohort(a.rows, a.features, seed=a.seed + 1, nan_frac=0.02)
    if group is not None:
        Xd, yd = pdist.shard_rows(Xd, rank, world), pdist.shard_rows(yd, rank, world)
        Xs, ys = pdist.shard_rows(Xs, rank, world), pdist.shard_rows(ys, rank, world)
    Xd_t = torch.as_tensor(Xd, device=dev)
    yd_t = torch.as_tensor(yd, device=dev)
    Xs_t = torch.as_tensor(Xs, device=dev)
    ys_t = torch.as_tensor(ys, device=dev)

    def step(evaluate=False, timer=None):
        return develop(Xd_t, yd_t, Xs_t, ys_t, names, device=dev, group=group, evaluate=evaluate,
                       timer=timer or StageTimer(enabled=False))

    def barrier():
        if group is not None:
            torch.distributed.barrier(group)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for w in range(a.warmup):
        if w == a.warmup - 1 and os.environ.get("HFENS_GC_FREEZE", "1") != "0":
            # long-lived objects (the cohort, extension handles, cached workspaces) to the permanent
            # generation: a timed step then never pays a full-heap generation-2 scan of them.  Done
            # before the LAST warmup step, which also runs with an event stage timer like the timed
            # steps: the first timed step was ≈ 1.5 ms slower than the rest when the collection
            # (tens of ms of device idle) and the first event timer came right before it
            barrier()
            import gc
            gc.collect()
            gc.freeze()
            step(timer=StageTimer(enabled=True, events=True))
        else:
            step()
    barrier()
    # every timed step carries an event-based stage timer (no host synchronisation: it costs
    # the timed region nothing); the per-stage table below is the median over the timed steps
    # (HFENS_BENCH_STAGE_EVENTS=0: no timing events in the timed steps — the per-stage table is then
    # empty; an A/B of the events' own cost, profiles/r6_runs/r6bt)
    stage_events = os.environ.get("HFENS_BENCH_STAGE_EVENTS", "1") != "0"
    timers = [StageTimer(enabled=stage_events, events=True) for _ in range(a.steps)]
    threads0 = _thread_cpu()
    sampler = _SyscallSampler() if os.environ.get("HFENS_THREAD_SAMPLE") == "1" else None
    cpu0 = time.process_time()
    t0 = time.perf_counter()
    step_ends = []
    for k in range(a.steps):
        res = step(timer=timers[k])
        step_ends.append(time.perf_counter())
    barrier()
    elapsed = time.perf_counter() - t0
    cpu = time.process_time() - cpu0
    threads1 = _thread_cpu()
    if sampler is not None:
        print("[thread-sample] " + sampler.stop(), file=sys.stderr)
    if group is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=group)
        elapsed = float(t)
    n_total = res.n_train
    for tm in timers:
        tm.collect()
    stage_med = {k: round(float(np.median([tm.times.get(k, 0.0) for tm in timers])), 4)
                 for k in timers[0].times}
    host_med = {k: round(float(np.median([tm.host_times.get(k, 0.0) for tm in timers])), 4)
                for k in timers[0].host_times}
    # untimed: held-out AUROC of a final fit (+ the device-synchronised stage table for --timings)
    prof = StageTimer(enabled=True, device=dev if dev.type == "cuda" else None)
    final = step(evaluate=True, timer=prof)
    value = n_total * a.steps / elapsed
    if rank == 0:
        if a.timings:
            print(prof.table(), file=sys.stderr)
        out = {
            "metric": "train_rows_per_sec",
            "value": round(value, 2),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * elapsed / a.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / CPU_BASELINE_ROWS_PER_S, 2),
            "dtype": "fp32",
            "data": "synthetic (Table S1-shaped HCM cohort, 2% NaN, random-init models)",
            "auroc": round(final.scores["auroc"], 4),
            "average_precision": round(final.scores["average_precision"], 4),
            "config": {"model": "HF-progression stack: KNN-impute + LassoCV top-17 + "
                                "Stacking{Scaler+SVC(rbf,Platt), GBC(100 stumps), LR-L1} -> LR-L2",
                       "global_batch": n_total, "seq_len": a.features, "rows_per_gpu": a.rows // max(1, world),
                       "features": a.features, "parallelism": f"dp{world}",
                       "stage_seconds": stage_med},
            "diag": dict(run_facts(dev, a.steps, elapsed, cpu, host_med, step_ends, t0), blocking_sync=blocking,
                         busiest_threads_cpu_s=_thread_delta(threads0, threads1)),
        }
        print(json.dumps(out), flush=True)
    pdist.shutdown()


def _ws_critical(st):
    """The working-set solve of the problem with the most pairs (the fit's critical path): rounds,
    pairs and its in-kernel s_memtime phase totals (shader-clock kilocycles; the per-pair figure is
    the inner loop's)."""
    k = int(st["inner"].argmax())
    pairs = max(int(st["inner"][k]), 1)
    return {"rounds": int(st["outer"][k]), "pairs": pairs,
            "kcyc_select": round(float(st["cyc_select"][k]) / 1e3, 1),
            "kcyc_select_keys": round(float(st["cyc_p0"][k]) / 1e3, 1),      # key loads, counts, gap test
            "kcyc_select_pick": round(float(st["cyc_p1"][k]) / 1e3, 1),      # radix histograms + compaction
            "kcyc_build": round(float(st["cyc_build"][k]) / 1e3, 1),
            "kcyc_inner": round(float(st["cyc_inner"][k]) / 1e3, 1),
            "cyc_per_pair": round(float(st["cyc_inner"][k]) / pairs),
            # shader clock of the inner phase: s_memtime cycles per 100 MHz s_memrealtime tick
            "inner_clock_ghz": (round(float(st["cyc_inner"][k]) / float(st["cyc_p2"][k]) * 0.1, 3)
                                if float(st["cyc_p2"][k]) > 0 else None)}


def run_facts(dev, steps, elapsed, cpu, host_med, step_ends, t0):
    """Facts that explain a training-bench run (VERDICT r1 'next round' #1): device, which
    solver / kernel paths ran, and how host-bound the timed steps were."""
    import numpy as np
    import torch
    from hfens.models import hist_gbdt, logreg_solver, smo, stack_trainer, svc_lowrank
    facts = {"host_cpu_s_per_step": round(cpu / steps, 4),
             "host_cpu_fraction": round(cpu / max(elapsed, 1e-12), 3),
             "stage_host_seconds": host_med,
             "step_ms_min_med_max": [round(1e3 * x, 2) for x in _step_stats(step_ends, t0)],
             "step_ms": [round(1e3 * (b - a), 2) for a, b in zip([t0] + list(step_ends[:-1]), step_ends)],
             "svm": dict(smo.LAST_SMO_INFO, **({"lowrank": {k: v for k, v in svc_lowrank.LAST_INFO.items()}}
                                              if smo.LAST_SMO_INFO.get("solver") == "nystrom-ipm" else {}),
                         **({"ws_rounds_max": int(smo.LAST_WS_STATS["outer"].max()),
                             "ws_pairs_max": int(smo.LAST_WS_STATS["inner"].max()),
                             "ws_critical": _ws_critical(smo.LAST_WS_STATS)}
                            if smo.LAST_SMO_INFO.get("solver") == "ws" else {})),
             "gbdt_path": hist_gbdt.LAST_PATH.get("path"),
             "logreg_path": logreg_solver.LAST_PATH.get("path"),
             "concurrent_bases": bool(stack_trainer.CONCURRENT_BASES and dev.type == "cuda"),
             "cpu_count": os.cpu_count(),
             "cpu_affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
             "loadavg": [round(x, 2) for x in os.getloadavg()]}
    if dev.type == "cuda":
        p = torch.cuda.get_device_properties(dev)
        facts.update(gpu=p.name, arch=getattr(p, "gcnArchName", None), cus=p.multi_processor_count,
                     hw_queues=os.environ.get("GPU_MAX_HW_QUEUES"))
    return facts


class _SyscallSampler:
    """HFENS_THREAD_SAMPLE=1: samples /proc/self/task/*/syscall every ≈ 0.5 ms over the timed steps
    and reports, per thread, how often it was in user space ("running") or in which system call
    (x86-64 numbers: 16 ioctl, 7 poll, 202 futex, 23 select, 35 nanosleep) — what the busy
    runtime thread of the headline's host profile is doing."""

    def __init__(self):
        import threading
        self._stop = threading.Event()
        self.counts = {}
        self._me = None
        self._th = threading.Thread(target=self._run, name="hfens-sampler", daemon=True)
        self._th.start()

    def _run(self):
        self._me = str(threading_native_id())
        while not self._stop.is_set():
            for tid in os.listdir("/proc/self/task"):
                if tid == self._me:
                    continue
                try:
                    with open(f"/proc/self/task/{tid}/syscall") as f:
                        w = f.read().split()
                except OSError:
                    continue
                key = w[0] if w else "?"
                d = self.counts.setdefault(tid, {})
                d[key] = d.get(key, 0) + 1
            time.sleep(0.0005)

    def stop(self) -> str:
        self._stop.set()
        self._th.join()
        tot = {t: sum(d.values()) for t, d in self.counts.items()}
        busy = sorted(self.counts, key=lambda t: -(tot[t] - self.counts[t].get("202", 0)))[:4]
        return " | ".join(f"tid {t}: " + ", ".join(f"{k}={v}" for k, v in sorted(self.counts[t].items(), key=lambda x: -x[1])[:4])
                          for t in busy)


def threading_native_id():
    import threading
    return threading.get_native_id()


def _thread_cpu():
    """{(tid, name): CPU seconds} of this process's threads (Linux /proc), {} elsewhere."""
    out = {}
    try:
        tick = os.sysconf("SC_CLK_TCK")
        for tid in os.listdir("/proc/self/task"):
            try:
                with open(f"/proc/self/task/{tid}/stat") as f:
                    st = f.read()
                fields = st[st.rindex(")") + 2:].split()
                with open(f"/proc/self/task/{tid}/comm") as f:
                    name = f.read().strip()
                out[(tid, name)] = (int(fields[11]) + int(fields[12])) / tick
                out[(tid, name + ":sys")] = int(fields[12]) / tick
            except OSError:
                continue
    except OSError:
        pass
    return out


def _thread_delta(a, b, top=5):
    """CPU seconds per thread name over the timed steps, the busiest few (explains host load)."""
    import threading
    main = str(os.getpid())
    py = {str(t.native_id): t.name for t in threading.enumerate() if t.native_id is not None}
    agg = {}
    for k, v in b.items():
        d = v - a.get(k, 0.0)
        if d > 0:
            tag = "(main)" if k[0] == main else (f"({py[k[0]]})" if k[0] in py else "(native)")
            agg[f"{k[1]}{tag}#{k[0]}"] = d
    return {k: round(v, 3) for k, v in sorted(agg.items(), key=lambda x: -x[1])[:top]}


def _step_stats(ends, t0):
    import numpy as np
    d = np.diff(np.array([t0] + list(ends)))
    return (float(d.min()), float(np.median(d)), float(d.max())) if d.size else (0.0, 0.0, 0.0)


CPU_BASELINE_INFER_ROWS_PER_S = 158e3   # numpy full-stack batched inference
CPU_BASELINE_GBDT_ROWS_PER_S = 286e3    # sklearn HistGB, 100 stumps, 1M × 40
CPU_BASELINE_DEEP_ROWS_SEEDS_PER_S = 53e3   # HistGB 1000 stumps × 5 seeds, 1M × 40


def bench_gbdt(a):
    import torch
    from hfens.parallel import dist as pdist
    from hfens.io.synth import make_hf_cohort_device
    from hfens.models.gbdt import GradientBoostingClassifier
    from hfens.models.hist_gbdt import fit_gbdt_batch
    from hfens.models.forest_infer import ensemble_raw_binned, stump_bin_tables
    from hfens.utils import metrics
    from hfens import ops

    deep = a.config == "deep"
    trees = a.trees or (1000 if deep else 100)
    seeds = a.seeds or (5 if deep else 1)
    rows = a.rows if a.rows != 10000 else 1_000_000
    group, rank, world = pdist.init_from_env()
    dev = pdist.rank_device()
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
        ops.ext()
    # multi-GPU layout (parallel/ensemble.py): S ranks per seed group — S = 1 trains whole seeds
    # per rank with no collective, S = N shards the rows of every seed (per-stage peer-memory
    # sum), in between a hybrid; every seed's trees are bit-identical to the one-GPU fit
    from hfens.parallel import ensemble
    S = ensemble.seed_layout(world, seeds, rows, a.dp_policy) if group is not None else 1
    G = world // S
    mine = ensemble.my_seeds(rank, world, seeds, S)
    glo, ghi = pdist.shard_bounds(rows, rank % S, S)     # this rank's rows within its group
    X, y = make_hf_cohort_device(rows, a.features, seed=a.seed, rows=(glo, ghi), device=dev)
    sub = ensemble.group_of(rank, world, S, group) if group is not None else None
    n_hold = max(1, rows // 5)
    Xh, yh = make_hf_cohort_device(n_hold, a.features, seed=a.seed + 1, rows=(0, n_hold), device=dev)

    def fit():
        ms = [GradientBoostingClassifier(n_estimators=trees, max_depth=a.depth, subsample=a.subsample,
                                         random_state=a.seed + k) for k in range(seeds)]
        if mine:
            fit_gbdt_batch([ms[k] for k in mine], X, y, group=sub)
        return [ms[k] for k in mine]

    def barrier():
        if group is not None:
            torch.distributed.barrier(group)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for _ in range(a.warmup):
        fit()
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ms = fit()
    barrier()
    elapsed = time.perf_counter() - t0
    if group is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=group)
        elapsed = float(t)
    # untimed: held-out AUROC of the seed-averaged ensemble (folded stump tables) and its speed;
    # every rank scores its own seeds on all held-out rows, one SUM over the seed groups' leaders
    lead = rank % S == 0
    t_inf = float("nan")
    ssum = torch.zeros(n_hold, dtype=torch.float64, device=dev)
    if ms and lead:
        bins_h = ms[0]._bin_mapper.transform(Xh)
        if a.depth == 1:
            T, init = stump_bin_tables(ms)
            raw = ensemble_raw_binned(T, init, bins_h)
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            for _ in range(5):
                raw = ensemble_raw_binned(T, init, bins_h)
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            t_inf = (time.perf_counter() - t1) / 5
        else:
            raw = torch.stack([m.decision_function(Xh) for m in ms])
        ssum = torch.sigmoid(raw.double()).sum(0)
    if group is not None:
        pdist.all_reduce_sum_(ssum, group)
    score = ssum / seeds
    # fp8 leaf values on the matrix cores (BASELINE config 5): the same ensemble as a leaf one-hot ×
    # two-term e4m3 leaf-value GEMV (ops/csrc/forest_fp8.hip), timed, with its AUROC delta
    # (one-process runs: it needs every seed's trees on one device)
    fp8 = None
    if dev.type == "cuda" and seeds <= 8 and group is None:
        from hfens.models.forest_infer import Fp8Forest
        f8 = Fp8Forest(ms)
        raw8 = f8.raw(bins_h)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        for _ in range(5):
            raw8 = f8.raw(bins_h)
        torch.cuda.synchronize(dev)
        t_f8 = (time.perf_counter() - t2) / 5
        score8 = torch.sigmoid(raw8.double()).mean(0)
        fp8 = dict(score=score8, t=t_f8, max_raw_err=float((raw8.double() - raw.double()).abs().max()))
    auc = metrics.roc_auc(yh.double(), score)
    if fp8 is not None:
        fp8["auroc"] = metrics.roc_auc(yh.double(), fp8["score"])
    value = rows * seeds * a.steps / elapsed
    if rank == 0:
        base = CPU_BASELINE_DEEP_ROWS_SEEDS_PER_S if deep else CPU_BASELINE_GBDT_ROWS_PER_S
        print(json.dumps({
            "metric": "train_rows_x_seeds_per_sec" if deep else "train_rows_per_sec",
            "value": round(value, 1), "unit": "rows*seeds/s" if deep else "rows/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(1000 * elapsed / a.steps, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": round(value / base, 2),
            # dtype = the precision of the TIMED work (training); the fp8 leaf-value inference runs
            # after the clock and reports its own dtype in fp8_leaf_inference
            "dtype": "fp32",
            "train_dtype": "fp32 gradients, int64 fixed-point histograms, f64 leaf values",
            "infer_dtype": "fp32 folded stump tables" + (" (+ fp8 e4m3 leaf GEMV, see fp8_leaf_inference)"
                                                         if fp8 is not None else ""),
            "data": "synthetic Table S1-shaped cohort (device generator), no NaN",
            "auroc": round(float(auc), 4),
            "infer_rows_x_models_per_sec": round(n_hold * seeds / max(t_inf, 1e-12), 1) if t_inf == t_inf else None,
            "fp8_leaf_inference": None if fp8 is None else {
                "leaf_dtype": "fp8 e4m3 two-term (hi + lo), per-model power-of-two scale",
                "kernel": "forest_fp8: leaf one-hot x fp8 leaf values, v_mfma_scale_f32_16x16x128_f8f6f4",
                "auroc": round(float(fp8["auroc"]), 5), "auroc_fp32_tables": round(float(auc), 5),
                "auroc_delta": round(float(fp8["auroc"] - auc), 6), "max_abs_raw_err": fp8["max_raw_err"],
                "rows_x_models_per_sec": round(n_hold * seeds / max(fp8["t"], 1e-12), 1)},
            "config": {"model": f"hist GBDT {trees} trees depth {a.depth} x {seeds} seeds, subsample {a.subsample}",
                       "global_batch": rows, "seq_len": a.features,
                       "parallelism": f"dp{world}" if S == world else
                       (f"seeds{G}" if S == 1 else f"seeds{G}xdp{S}"),
                       "seed_groups": G, "ranks_per_group": S},
        }), flush=True)
    pdist.shutdown()


def synth_patients(n: int, device, seed: int = 0, chunk: int = 1 << 24):
    """[n, 17] f32 patient rows in predict_hf.py's feature order (binary flags, NYHA 1-2,
    FEV-like, count 0-4, age), generated on the device chunk by chunk."""
    import torch
    g = torch.Generator(device=device).manual_seed(seed)
    X = torch.empty(n, 17, dtype=torch.float32, device=device)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        m = e - s
        blk = torch.randint(0, 2, (m, 17), generator=g, device=device).to(torch.float32)
        blk[:, 6] += 1
        blk[:, 13] = (18.6 + 4.4 * torch.randn(m, generator=g, device=device)).round()
        blk[:, 15] = torch.randint(0, 5, (m,), generator=g, device=device).to(torch.float32)
        blk[:, 16] = (63 + 5 * torch.randn(m, generator=g, device=device)).round()
        X[s:e] = blk
    return X


def bench_infer(a):
    import torch
    from hfens.parallel import dist as pdist
    from hfens.io.checkpoint import load_checkpoint
    from hfens.infer import BatchedPredictor

    group, rank, world = pdist.init_from_env()
    dev = pdist.rank_device()
    if dev.type != "cuda":
        raise SystemExit("bench --config infer needs a GPU")
    torch.cuda.set_device(dev)
    rows = a.rows if a.rows != 10000 else 100_000_000
    lo, hi = pdist.shard_bounds(rows, rank, world)
    n = hi - lo
    model = load_checkpoint(device=dev)
    pred = BatchedPredictor(model, dev)
    X = synth_patients(n, dev, seed=a.seed + rank)
    out = torch.empty(n, dtype=torch.float32, device=dev)

    def barrier():
        if group is not None:
            torch.distributed.barrier(group)
        torch.cuda.synchronize(dev)

    for _ in range(max(1, a.warmup)):
        pred.predict_device(X, out)
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        pred.predict_device(X, out)
    barrier()
    elapsed = time.perf_counter() - t0
    # spot-check against the per-model path on a slice (untimed)
    model.fused_inference = False
    ref = model.predict_p1(X[:4096])
    model.fused_inference = True
    max_err = float((out[:4096].double() - ref.double()).abs().max())
    # host streaming (untimed by the step clock, reported alongside)
    Xh = X.cpu().pin_memory()
    oh = torch.empty(n, dtype=torch.float32).pin_memory()
    pred.predict_host(Xh, oh)
    barrier()
    t1 = time.perf_counter()
    pred.predict_host(Xh, oh)
    barrier()
    t_stream = time.perf_counter() - t1
    stream_ok = bool(torch.equal(oh[:65536], out[:65536].cpu()))
    if group is not None:
        t = torch.tensor([elapsed, t_stream], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=group)
        elapsed, t_stream = float(t[0]), float(t[1])
    value = rows * a.steps / elapsed
    if rank == 0:
        out_line = {
            "metric": "infer_rows_per_sec",
            "value": round(value, 1),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * elapsed / a.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / CPU_BASELINE_INFER_ROWS_PER_S, 1),
            "dtype": "fp32",
            "data": "synthetic patient rows; shipped hf_predict_model.pkl weights",
            "host_stream_rows_per_sec": round(rows / t_stream, 1),
            "host_stream_matches": stream_ok,
            "max_abs_err_vs_per_model_path": max_err,
            "config": {"model": "hf_predict_model.pkl stack (SVC 434 SV + GBC 100 stumps + LR-L1 -> LR)",
                       "global_batch": rows, "seq_len": 17, "parallelism": f"dp{world}",
                       "kernel": "fused stack_infer, HIP-graph replay"},
        }
        print(json.dumps(out_line), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
