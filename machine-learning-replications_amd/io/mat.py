"""MATLAB table loader (reference ``load_data_public.py:4-14``).

``load_data(path) -> (X float64 [n, p], Y float64 [n], var_names)``: the
``data_tb`` matrix's last column is the outcome, ``clin_var_names`` the
cellstr of column names.  MAT v5 parsing is scipy's; :func:`save_data` writes
the same layout (used to build fixtures, since the reference's ``.mat`` files
are private and not shipped).
"""
from __future__ import annotations

import numpy as np


def load_data(dataset_path: str):
    import scipy.io as sio
    dataset = sio.loadmat(dataset_path)
    data = dataset["data_tb"]
    var_names = dataset["clin_var_names"]
    X = data[:, 0:-1].astype(float)
    Y = data[:, -1].astype(float)
    return X, Y, var_names


def save_data(path: str, X, Y, names) -> None:
    import scipy.io as sio
    data = np.column_stack([np.asarray(X, dtype=float), np.asarray(Y, dtype=float)])
    cell = np.empty((1, len(names)), dtype=object)
    for i, nm in enumerate(names):
        cell[0, i] = np.array([nm])
    sio.savemat(path, {"data_tb": data, "clin_var_names": cell})


def names_list(var_names) -> list:
    """MATLAB cellstr (1×p object array) → list of str."""
    arr = np.asarray(var_names)
    out = []
    for v in arr.reshape(-1):
        while isinstance(v, np.ndarray):
            v = v.reshape(-1)[0] if v.size else ""
        out.append(str(v))
    return out
