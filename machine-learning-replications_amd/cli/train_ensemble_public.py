"""Model development entry point (reference ``train_ensemble_public.py``).

No-argument behaviour follows the reference: load ``develop_data.mat`` and
``model_select_data.mat`` from the directory of the script that was run
(``T:33-39``: ``os.path.dirname(__file__)``), print the selected feature names and
count (``T:56-59``), fit the stack, print the held-out ``classification_report`` at
``> 0.5`` (``T:62-64``) and ALWAYS draw the ROC/PR curves with Wald bands
(``T:66-90``; written as ``hf_roc.png`` / ``hf_pr.png`` in the working directory
instead of ``plt.show()`` on a headless node, ``--no-plots`` to skip).  Those
``.mat`` files are private, so when they are absent a Table-S1-shaped synthetic
cohort is generated (``--rows``, ``--features``).  Extras: ``--device cuda``, ``--save-model``
(writes the sklearn-0.23.2 ``.pkl`` layout that ``predict_hf.py`` reads),
``--timings``; under ``torchrun`` the development rows are sharded over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np


def main(argv=None, script_dir=None) -> int:
    ap = argparse.ArgumentParser(description="train the HF-progression stacking ensemble")
    ap.add_argument("--data-dir", default=None,
                    help="directory with develop_data.mat / model_select_data.mat (default: the script's)")
    ap.add_argument("--rows", type=int, default=713, help="synthetic rows per set (when no .mat files)")
    ap.add_argument("--features", type=int, default=64, help="synthetic candidate features")
    ap.add_argument("--seed", type=int, default=2020)
    ap.add_argument("--device", default=None, help="cpu | cuda (default: cuda if available)")
    ap.add_argument("--save-model", default=None, help="write a 0.23.2-layout hf_predict_model.pkl")
    ap.add_argument("--plots", default="hf", help="PNG prefix for the ROC/PR plots (default 'hf')")
    ap.add_argument("--no-plots", action="store_true", help="skip the ROC/PR figures")
    ap.add_argument("--timings", action="store_true")
    ap.add_argument("--json", default=None, help="append a JSON result line to this file")
    ap.add_argument("--lr-optimum", action="store_true",
                    help="solve 'lg' to its exact optimum on the device instead of reproducing liblinear's "
                         "default-tolerance iterate and seed draw (the reference's T:31/T:46 behaviour)")
    a = ap.parse_args(argv)
    if a.no_plots:
        a.plots = None

    import torch
    from ..io.mat import load_data, names_list
    from ..io.synth import make_dev_select
    from ..pipeline import develop
    from ..utils import metrics
    from ..parallel import dist as pdist

    group, rank, world = pdist.init_from_env()
    device = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    if device == "cuda":
        device = str(pdist.rank_device())
        torch.cuda.set_device(torch.device(device))
    # T:33-34: the .mat files sit next to the script that was run (not the working directory)
    data_dir = a.data_dir or script_dir or os.path.dirname(os.path.abspath(sys.argv[0] or "."))
    dev_path = os.path.join(data_dir, "develop_data.mat")
    sel_path = os.path.join(data_dir, "model_select_data.mat")
    if os.path.exists(dev_path) and os.path.exists(sel_path):
        X_dev, y_dev, names = load_data(dev_path)
        X_sel, y_sel, _ = load_data(sel_path)
        names = names_list(names)
        source = "mat"
    else:
        X_dev, y_dev, X_sel, y_sel, names = make_dev_select(a.rows, a.features, seed=a.seed)
        source = "synthetic"
        if rank == 0:
            print(f"[hfens] {dev_path} not found: using a synthetic Table-S1 cohort "
                  f"({a.rows} rows x {a.features} features per set)")
    if group is not None:
        X_dev, y_dev = pdist.shard_rows(X_dev, rank, world), pdist.shard_rows(y_dev, rank, world)
        X_sel, y_sel = pdist.shard_rows(X_sel, rank, world), pdist.shard_rows(y_sel, rank, world)
    from ..config import EnsembleConfig
    cfg = EnsembleConfig(liblinear_exact=not a.lr_optimum)
    # T:31: numpy's GLOBAL generator seeded with init_rs — liblinear's seeds ('lg', random_state=None)
    # are drawn from it, six times, in the stacking fit's order
    np.random.seed(cfg.seed)
    res = develop(X_dev, y_dev, X_sel, y_sel, names, device=device, group=group, cfg=cfg)
    if a.plots:
        # collectives on EVERY rank (before the rank-0 block); only rank 0 draws
        p_all = res.proba_sel
        y_all = torch.as_tensor(y_sel, device=p_all.device)
        if group is not None:
            p_all = pdist.all_gather_rows(p_all[:, None], group)[:, 0]
            y_all = pdist.all_gather_rows(y_all.to(p_all.dtype)[:, None], group)[:, 0]
    if rank == 0:
        print("Important Features")
        print(np.array(res.selected_names, dtype=object))
        print("number of features = ", len(res.selected_names))
        print(res.report)
        print(f"AUROC = {res.scores['auroc']:.4f}   AP = {res.scores['average_precision']:.4f}")
        if a.timings:
            print(res.timer.table())
        if a.plots:
            print("plots:", metrics.save_plots(y_all, p_all, a.plots))
        if a.save_model:
            from ..io.checkpoint import save_checkpoint
            model = res.model
            model.to("cpu")
            save_checkpoint(model, a.save_model)
            print(f"saved {a.save_model}")
        if a.json:
            with open(a.json, "a") as f:
                f.write(json.dumps({"source": source, "n_train": res.n_train, "scores": res.scores,
                                    "timings": dict(res.timer.times), "world_size": world}) + "\n")
    pdist.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
