"""Deterministic CV splitters with sklearn's fold assignment (so OOF meta-features
and LassoCV paths follow the same rows as the reference run).

* :func:`stratified_kfold_test_folds` — ``StratifiedKFold(n_splits, shuffle=False)``
  (``StackingClassifier``'s ``cv=None`` on a classifier; reference
  ``train_ensemble_public.py:48``): classes encoded by first appearance, the sorted
  label vector dealt round-robin over folds, then each class's members assigned to
  folds in row order.
* :func:`kfold_test_folds` — ``KFold(n_splits)`` unshuffled (``LassoCV(cv=10)``,
  reference ``train_ensemble_public.py:51``): contiguous blocks, the first
  ``n % k`` folds one row larger.
"""
from __future__ import annotations

import numpy as np
import torch


def stratified_kfold_test_folds(y, n_splits: int = 5) -> np.ndarray:
    y = np.asarray(y.cpu() if isinstance(y, torch.Tensor) else y).ravel()
    if y.size:
        tf = _stratified_binary(y, n_splits)
        if tf is not None:
            return tf
    return _stratified_generic(y, n_splits)


def _stratified_binary(y: np.ndarray, n_splits: int):
    """Two-class labels (the stacking fit's): the same assignment as :func:`_stratified_generic`
    in a few vector ops — class 0 is the first label seen, the sorted encoded labels are class 0's
    count then class 1's, so fold i's share of class 0 is the count of positions ≡ i (mod k)
    below that count.  None when the labels are not two-valued."""
    enc = y != y[0]
    j = int(enc.argmax())
    if not enc[j] or not ((y == y[0]) | (y == y[j])).all():
        return None
    n = y.size
    c0 = n - int(np.count_nonzero(enc))
    counts = np.array([c0, n - c0])
    if np.all(n_splits > counts):
        raise ValueError(f"n_splits={n_splits} cannot be greater than the number of members in each class")
    i = np.arange(n_splits)
    tot = (n - i + n_splits - 1) // n_splits                   # positions ≡ i (mod k) in [0, n)
    a0 = np.where(c0 > i, (c0 - i + n_splits - 1) // n_splits, 0)
    test_folds = np.empty(n, dtype=np.int64)
    test_folds[~enc] = np.repeat(i, a0)
    test_folds[enc] = np.repeat(i, tot - a0)
    return test_folds


def _stratified_generic(y: np.ndarray, n_splits: int) -> np.ndarray:
    _, y_idx, y_inv = np.unique(y, return_index=True, return_inverse=True)
    _, class_perm = np.unique(y_idx, return_inverse=True)
    y_enc = class_perm[y_inv]
    n_classes = len(y_idx)
    counts = np.bincount(y_enc)
    if np.all(n_splits > counts):
        raise ValueError(f"n_splits={n_splits} cannot be greater than the number of members in each class")
    y_order = np.sort(y_enc)
    alloc = np.asarray([np.bincount(y_order[i::n_splits], minlength=n_classes) for i in range(n_splits)])
    test_folds = np.empty(len(y), dtype=np.int64)
    for k in range(n_classes):
        test_folds[y_enc == k] = np.arange(n_splits).repeat(alloc[:, k])
    return test_folds


def kfold_test_folds(n: int, n_splits: int) -> np.ndarray:
    sizes = np.full(n_splits, n // n_splits, dtype=np.int64)
    sizes[: n % n_splits] += 1
    return np.repeat(np.arange(n_splits), sizes)


def fold_masks(test_folds, n_splits: int, device=None, with_full: bool = True) -> torch.Tensor:
    """Training masks ``[n_splits (+1), n]``: fold k trains on rows not in test fold k;
    the optional last row is the full refit."""
    tf = torch.from_numpy(np.ascontiguousarray(test_folds))
    if device is not None and torch.device(device).type == "cuda":
        # pinned, non-blocking: a pageable upload would hold the host until the stream's queued work
        # (e.g. the LassoCV path under which the stacking trainer is prelaunched) has finished
        tf = tf.pin_memory().to(device, non_blocking=True)
    elif device is not None:
        tf = tf.to(device)
    # one comparison against [0, …, K−1] (and K, which no fold id equals: the all-true refit row).
    # (no element assignment on the device tensor: a host scalar written into it was a blocking
    # copy that waited for the stream's queued work — ≈ 0.6 ms of the prelaunch's host time)
    ks = torch.arange(n_splits + int(with_full), device=tf.device, dtype=tf.dtype)
    return tf[None, :] != ks[:, None]
