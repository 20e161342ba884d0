"""``hf_predict_model.pkl`` ⇄ native models.

Reader: :func:`load_checkpoint` decodes the sklearn-0.23.2 pickle inertly
(:mod:`hfens.io.skpickle`) and converts the fitted ``StackingClassifier`` graph
(schema: SURVEY.md Appendix A) into the framework's native estimators.

Writer: :func:`save_checkpoint` emits a freshly trained native stack in the same
0.23.2 layout — same class paths, attribute sets and orders, dtypes (7-field
tree node records, intc vs int32 dtype objects), MT19937 ``RandomState``
record, memo sharing (``estimators_`` ≡ ``named_estimators_``; one RandomState
shared by the GBC and all its trees).  For the shipped checkpoint,
``save_checkpoint(load_checkpoint(f))`` reproduces every byte of ``f``
(tests/test_checkpoint.py).
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from . import skpickle as sp
from .skpickle import Builder, NpRandomState, SkObject
from ..models.gbdt import GradientBoostingClassifier
from ..models.linear import LogisticRegression
from ..models.scaler import StandardScaler
from ..models.stacking import Pipeline, StackingClassifier
from ..models.svc import SVC

SK_VERSION = "0.23.2"
NODE_DTYPE = np.dtype([("left_child", "<i8"), ("right_child", "<i8"), ("feature", "<i8"),
                       ("threshold", "<f8"), ("impurity", "<f8"), ("n_node_samples", "<i8"),
                       ("weighted_n_node_samples", "<f8")])

_CLS = {
    "stack": ("sklearn.ensemble._stacking", "StackingClassifier"),
    "pipe": ("sklearn.pipeline", "Pipeline"),
    "scaler": ("sklearn.preprocessing._data", "StandardScaler"),
    "svc": ("sklearn.svm._classes", "SVC"),
    "gbc": ("sklearn.ensemble._gb", "GradientBoostingClassifier"),
    "lr": ("sklearn.linear_model._logistic", "LogisticRegression"),
    "le": ("sklearn.preprocessing._label", "LabelEncoder"),
    "loss": ("sklearn.ensemble._gb_losses", "BinomialDeviance"),
    "dummy": ("sklearn.dummy", "DummyClassifier"),
    "dtr": ("sklearn.tree._classes", "DecisionTreeRegressor"),
    "tree": ("sklearn.tree._tree", "Tree"),
    "bunch": ("sklearn.utils", "Bunch"),
}


def default_checkpoint_path() -> str:
    here = os.path.dirname(os.path.abspath(__file__))
    return os.path.normpath(os.path.join(here, "..", "..", "assets", "hf_predict_model.pkl"))


# ============================================================================ reader
def _params(obj: SkObject, names):
    return {k: obj.state[k] for k in names if k in obj.state}


def _scaler_from(o: SkObject) -> StandardScaler:
    s = StandardScaler(**_params(o, StandardScaler._param_names))
    if "mean_" in o.state:
        s._set(torch.as_tensor(o["mean_"]), torch.as_tensor(o["var_"]), int(o["n_samples_seen_"]))
        s.scale_ = torch.as_tensor(o["scale_"])
    return s


def _svc_from(o: SkObject) -> SVC:
    m = SVC(**_params(o, SVC._param_names))
    if "support_" in o.state:
        m.set_fitted(support=o["support_"], support_vectors=o["support_vectors_"],
                     n_support=o["_n_support"], dual_coef_libsvm=o["_dual_coef_"],
                     rho=-float(o["_intercept_"][0]), probA=float(o["_probA"][0]),
                     probB=float(o["_probB"][0]), gamma=float(o["_gamma"]),
                     class_weight=o["class_weight_"], shape_fit=o["shape_fit_"],
                     n_features=o["n_features_in_"])
        m.dual_coef_ = torch.as_tensor(o["dual_coef_"])
        m.intercept_ = torch.as_tensor(o["intercept_"])
    return m


def _lr_from(o: SkObject) -> LogisticRegression:
    m = LogisticRegression(**_params(o, LogisticRegression._param_names))
    if "coef_" in o.state:
        m.set_fitted(o["coef_"], o["intercept_"], o["n_iter_"], o["n_features_in_"])
    return m


def _gbc_from(o: SkObject) -> GradientBoostingClassifier:
    m = GradientBoostingClassifier(**_params(o, GradientBoostingClassifier._param_names))
    if "estimators_" not in o.state:
        return m
    trees = o["estimators_"][:, 0]
    T = len(trees)
    K = max(int(t["tree_"]["node_count"]) for t in trees)
    feat = np.full((T, K), -2, np.int64)
    thr = np.full((T, K), -2.0)
    left = np.full((T, K), -1, np.int64)
    right = np.full((T, K), -1, np.int64)
    val = np.zeros((T, K))
    imp = np.zeros((T, K))
    nns = np.zeros((T, K), np.int64)
    wnns = np.zeros((T, K))
    cnt = np.zeros(T, np.int64)
    for t, dtr in enumerate(trees):
        tr = dtr["tree_"]
        nodes = tr["nodes"]
        c = int(tr["node_count"])
        cnt[t] = c
        feat[t, :c] = nodes["feature"]
        thr[t, :c] = nodes["threshold"]
        left[t, :c] = nodes["left_child"]
        right[t, :c] = nodes["right_child"]
        imp[t, :c] = nodes["impurity"]
        nns[t, :c] = nodes["n_node_samples"]
        wnns[t, :c] = nodes["weighted_n_node_samples"]
        val[t, :c] = tr["values"][:, 0, 0]
    rng = o["_rng"]
    m.set_fitted(feature=feat, threshold=thr, left=left, right=right, value=val, impurity=imp,
                 n_node_samples=nns, weighted_n_node_samples=wnns, node_count=cnt,
                 class_prior=o["init_"]["class_prior_"], train_score=o["train_score_"],
                 n_features=o["n_features_"], rng_state=rng)
    m.tree_max_depth_ = [int(t["tree_"]["max_depth"]) for t in trees]
    return m


def _est_from(o: SkObject):
    cls = o.cls.rsplit(".", 1)[1]
    if cls == "Pipeline":
        steps = [(n, _est_from(s)) for n, s in o["steps"]]
        return Pipeline(steps, o.state.get("memory"), o.state.get("verbose", False))
    if cls == "StandardScaler":
        return _scaler_from(o)
    if cls == "SVC":
        return _svc_from(o)
    if cls == "GradientBoostingClassifier":
        return _gbc_from(o)
    if cls == "LogisticRegression":
        return _lr_from(o)
    raise ValueError(f"unsupported estimator class {o.cls}")


def load_checkpoint(path: Optional[str] = None, device=None) -> StackingClassifier:
    """Decode ``hf_predict_model.pkl`` (inert, nothing imported) into a native stack."""
    path = path or default_checkpoint_path()
    with open(path, "rb") as f:
        root = sp.parse(f.read())
    v = sp.to_py(root)
    if not (isinstance(v, SkObject) and v.cls.endswith("StackingClassifier")):
        raise ValueError(f"{path}: not a StackingClassifier checkpoint ({getattr(v, 'cls', type(v))})")
    st = v.state
    templates = [(n, _est_from(e)) for n, e in st["estimators"]]
    clf = StackingClassifier(templates, _est_from(st["final_estimator"]), st["cv"], st["stack_method"],
                             st["n_jobs"], st["passthrough"], st["verbose"])
    clf.estimators_ = [_est_from(e) for e in st["estimators_"]]
    clf.final_estimator_ = _est_from(st["final_estimator_"])
    clf.stack_method_ = list(st["stack_method_"])
    clf.classes_ = torch.as_tensor(st["classes_"])
    if device is not None:
        clf.to(device)
    return clf


# ============================================================================ writer
def _np(t, dtype=None):
    if isinstance(t, torch.Tensor):
        t = t.detach().cpu().numpy()
    a = np.asarray(t)
    return a.astype(dtype) if dtype is not None else a


class _W:
    """Node-graph builder replicating sklearn 0.23.2's object sharing."""

    def __init__(self):
        self.b = Builder()
        self.ver = None
        # numpy-1.x dtype instances: liblinear's n_iter_ came back as a *separate*
        # int32 (intc) dtype object from the one libsvm/lbfgs arrays used.
        self.dt_i4_intc = None
        self.step_names = {}

    def s(self, x):
        return self.b.s(x)

    def v(self, x):
        return self.b.value(x)

    def arr(self, a, dtype=None):
        return self.b.array(_np(a, dtype))

    def i4_intc(self, a):
        if self.dt_i4_intc is None:
            b = self.b
            st = sp.TupleN([sp.Prim(3), b.s("<"), sp.Prim(None), sp.Prim(None), sp.Prim(None),
                            sp.Prim(-1), sp.Prim(-1), sp.Prim(0)])
            self.dt_i4_intc = sp.Call(b.g("numpy", "dtype"), sp.TupleN([sp.Str("i4"), sp.Prim(False),
                                                                       sp.Prim(True)]),
                                      newobj=False, state=st)
        node = self.b.array(_np(a, np.int32))
        node.state.items[2] = self.dt_i4_intc
        return node

    def version(self):
        return [("_sklearn_version", self.s(SK_VERSION))]

    def obj(self, key, pairs):
        return self.b.obj(*_CLS[key], pairs)

    # -- estimators -----------------------------------------------------------
    def scaler(self, m: StandardScaler, fitted: bool):
        p = [("with_mean", self.v(m.with_mean)), ("with_std", self.v(m.with_std)), ("copy", self.v(m.copy))]
        if fitted:
            p += [("n_features_in_", self.v(int(m.n_features_in_))),
                  ("n_samples_seen_", self.b.scalar(np.int64(m.n_samples_seen_))),
                  ("mean_", self.arr(m.mean_, np.float64)), ("var_", self.arr(m.var_, np.float64)),
                  ("scale_", self.arr(m.scale_, np.float64))]
        return self.obj("scaler", p + self.version())

    def svc(self, m: SVC, fitted: bool):
        p = [(k, self.v(getattr(m, k))) for k in
             ("decision_function_shape", "break_ties", "kernel", "degree", "gamma", "coef0", "tol", "C")]
        p += [("nu", self.v(0.0)), ("epsilon", self.v(0.0))]
        p += [(k, self.v(getattr(m, k))) for k in
              ("shrinking", "probability", "cache_size", "class_weight", "verbose", "max_iter", "random_state")]
        if fitted:
            p += [("_sparse", self.v(False)), ("n_features_in_", self.v(int(m.n_features_in_))),
                  ("class_weight_", self.arr(m.class_weight_, np.float64)),
                  ("classes_", self.arr(m.classes_, np.int64)),
                  ("_gamma", self.b.scalar(np.float64(m._gamma))),
                  ("support_", self.arr(m.support_, np.int32)),
                  ("support_vectors_", self.arr(m.support_vectors_, np.float64)),
                  ("_n_support", self.arr(m._n_support, np.int32)),
                  ("dual_coef_", self.arr(m.dual_coef_, np.float64)),
                  ("intercept_", self.arr(m.intercept_, np.float64)),
                  ("_probA", self.arr(m._probA, np.float64)), ("_probB", self.arr(m._probB, np.float64)),
                  ("fit_status_", self.v(0)),
                  ("shape_fit_", self.v(tuple(int(s) for s in m.shape_fit_))),
                  ("_intercept_", self.arr(m._intercept_, np.float64)),
                  ("_dual_coef_", self.arr(m._dual_coef_, np.float64))]
        return self.obj("svc", p + self.version())

    def lr(self, m: LogisticRegression, fitted: bool, liblinear_iter_dtype: bool):
        p = [(k, self.v(getattr(m, k))) for k in LogisticRegression._param_names]
        if fitted:
            n_iter = (self.i4_intc(m.n_iter_) if liblinear_iter_dtype else self.arr(m.n_iter_, np.int32))
            p += [("n_features_in_", self.v(int(m.n_features_in_))),
                  ("classes_", self.arr(m.classes_, np.int64)),
                  ("coef_", self.arr(m.coef_, np.float64)),
                  ("intercept_", self.arr(m.intercept_, np.float64)), ("n_iter_", n_iter)]
        return self.obj("lr", p + self.version())

    def gbc(self, m: GradientBoostingClassifier, fitted: bool):
        names = ("n_estimators", "learning_rate", "loss", "criterion", "min_samples_split",
                 "min_samples_leaf", "min_weight_fraction_leaf", "subsample", "max_features", "max_depth",
                 "min_impurity_decrease", "min_impurity_split", "ccp_alpha", "init", "random_state",
                 "alpha", "verbose", "max_leaf_nodes", "warm_start", "presort", "validation_fraction",
                 "n_iter_no_change", "tol")
        p = [(k, self.v(getattr(m, k))) for k in names]
        if not fitted:
            return self.obj("gbc", p + self.version())
        b = self.b
        nf = int(m.n_features_)
        classes = lambda: self.arr(m.classes_, np.int64)  # noqa: E731
        p += [("n_features_in_", self.v(nf)), ("n_features_", self.v(nf)), ("classes_", classes()),
              ("n_classes_", self.v(2)),
              ("loss_", b.obj(*_CLS["loss"], [("K", sp.Prim(1))])),
              ("max_features_", self.v(nf))]
        init = self.obj("dummy", [("strategy", self.s("prior")), ("random_state", self.v(None)),
                                  ("constant", self.v(None)), ("_strategy", self.s("prior")),
                                  ("sparse_output_", self.v(False)), ("n_outputs_", self.v(1)),
                                  ("n_features_in_", self.v(None)), ("classes_", classes()),
                                  ("n_classes_", self.v(2)),
                                  ("class_prior_", self.arr(m.class_prior_, np.float64))] + self.version())
        p.append(("init_", init))
        rs = m.rng_state_ if isinstance(m.rng_state_, NpRandomState) else _rng_after(m.random_state, m.n_estimators_)
        rng_node = b.randomstate(rs)
        trees = [self.tree(m, t, rng_node, nf) for t in range(m.n_estimators_)]
        est = b.array(np.empty((m.n_estimators_, 1), dtype=object), obj_items=trees)
        p += [("estimators_", est), ("train_score_", self.arr(m.train_score_, np.float64)),
              ("_rng", rng_node), ("n_estimators_", self.v(int(m.n_estimators_)))]
        return self.obj("gbc", p + self.version())

    def tree(self, m, t, rng_node, nf):
        b = self.b
        c = int(m.tree_node_count_[t])
        depth = m.tree_max_depth_[t] if hasattr(m, "tree_max_depth_") else _depth(m, t)
        dtr = [("criterion", self.s(m.criterion)), ("splitter", self.s("best")),
               ("max_depth", self.v(m.max_depth)), ("min_samples_split", self.v(m.min_samples_split)),
               ("min_samples_leaf", self.v(m.min_samples_leaf)),
               ("min_weight_fraction_leaf", self.v(m.min_weight_fraction_leaf)),
               ("max_features", self.v(m.max_features)), ("max_leaf_nodes", self.v(m.max_leaf_nodes)),
               ("random_state", rng_node), ("min_impurity_decrease", self.v(m.min_impurity_decrease)),
               ("min_impurity_split", self.v(m.min_impurity_split)), ("class_weight", self.v(None)),
               ("presort", self.s(m.presort)), ("ccp_alpha", self.v(m.ccp_alpha)),
               ("n_features_", self.v(nf)), ("n_outputs_", self.v(1)), ("max_features_", self.v(nf))]
        order = _preorder(m, t, c)            # sklearn DepthFirstTreeBuilder node ids
        c = len(order)
        remap = {h: i for i, h in enumerate(order)}
        left = _np(m.tree_left_[t], np.int64)
        right = _np(m.tree_right_[t], np.int64)
        nodes = np.zeros(c, dtype=NODE_DTYPE)
        nodes["left_child"] = [remap[left[h]] if left[h] >= 0 else -1 for h in order]
        nodes["right_child"] = [remap[right[h]] if right[h] >= 0 else -1 for h in order]
        nodes["feature"] = _np(m.tree_feature_[t], np.int64)[order]
        nodes["threshold"] = _np(m.tree_threshold_[t], np.float64)[order]
        nodes["impurity"] = _np(m.tree_impurity_[t], np.float64)[order]
        nodes["n_node_samples"] = _np(m.tree_n_node_samples_[t], np.int64)[order]
        nodes["weighted_n_node_samples"] = _np(m.tree_weighted_n_node_samples_[t], np.float64)[order]
        values = _np(m.tree_value_[t], np.float64)[order].reshape(c, 1, 1)
        tree_state = sp.DictN([(self.s("max_depth"), sp.Prim(int(depth))),
                               (self.s("node_count"), sp.Prim(c)),
                               (self.s("nodes"), b.array(nodes)),
                               (self.s("values"), b.array(values))])
        tree = sp.Call(b.g(*_CLS["tree"]),
                       sp.TupleN([sp.Prim(nf), b.array(np.array([1], np.int64)), sp.Prim(1)]),
                       newobj=False, state=tree_state)
        dtr.append(("tree_", tree))
        return self.obj("dtr", dtr + self.version())

    def est(self, e, fitted, name=None):
        if isinstance(e, Pipeline):
            steps = []
            for n, s in e.steps:
                node = self.scaler(s, fitted) if isinstance(s, StandardScaler) else self.svc(s, fitted)
                if n not in self.step_names:
                    self.step_names[n] = sp.Str(n)
                steps.append(sp.TupleN([self.step_names[n], node]))
            return self.obj("pipe", [("steps", sp.ListN(steps)), ("memory", self.v(e.memory)),
                                     ("verbose", self.v(e.verbose))] + self.version())
        if isinstance(e, GradientBoostingClassifier):
            return self.gbc(e, fitted)
        if isinstance(e, LogisticRegression):
            return self.lr(e, fitted, liblinear_iter_dtype=(e.solver == "liblinear"))
        raise TypeError(type(e))


def _preorder(m, t, c):
    """Node order of sklearn's depth-first builder (parent, then left subtree, then right; ids in
    creation order) over the REACHABLE nodes.  A loaded checkpoint is already in that order (the
    identity); a fresh histogram-GBDT tree is a heap layout (children of node h at 2h+1, 2h+2,
    unreachable slots under leaves) and is compacted to sklearn's layout here."""
    left = _np(m.tree_left_[t], np.int64)
    right = _np(m.tree_right_[t], np.int64)
    order, stack = [], [0]
    while stack:
        h = stack.pop()
        order.append(h)
        if left[h] >= 0:
            stack.append(int(right[h]))
            stack.append(int(left[h]))
    if getattr(m, "tree_layout_", None) != "heap" and order != list(range(c)):
        raise ValueError(f"tree {t}: node order is not sklearn's depth-first order")
    return order


def _depth(m, t):
    feat = _np(m.tree_feature_[t])
    left = _np(m.tree_left_[t])
    right = _np(m.tree_right_[t])

    def d(i):
        return 0 if feat[i] < 0 else 1 + max(d(left[i]), d(right[i]))
    return d(0)


def _rng_after(random_state, n_draws) -> NpRandomState:
    """MT19937 state of ``RandomState(random_state)`` after the per-tree seed draws.
    The GBC shares one RandomState with its trees; sklearn 0.23.2 draws one
    ``randint(0, MAX_INT)`` per tree (observed: ``pos == n_estimators``)."""
    rs = np.random.RandomState(random_state if isinstance(random_state, int) else None)
    for _ in range(n_draws):
        rs.randint(np.iinfo(np.int32).max)
    st = rs.get_state()
    return NpRandomState(key=np.asarray(st[1], np.uint32), pos=int(st[2]), has_gauss=int(st[3]),
                         gauss=float(st[4]))


def checkpoint_graph(clf: StackingClassifier) -> sp.Node:
    w = _W()
    b = w.b
    templates = sp.ListN([sp.TupleN([sp.Str(n), w.est(e, fitted=False)]) for n, e in clf.estimators])
    # sklearn: the template names are the user's literals; the pipeline step name
    # 'svc' is a separate runtime string (make_pipeline lower-cases the class name).
    fitted = [w.est(e, fitted=True) for e in clf.estimators_]
    le_classes = w.arr(np.array([0.0, 1.0]))
    le = w.obj("le", [("classes_", le_classes)] + w.version())
    st = [("estimators", templates), ("final_estimator", w.est(clf.final_estimator, fitted=False)),
          ("cv", w.v(clf.cv)), ("stack_method", w.v(clf.stack_method)), ("n_jobs", w.v(clf.n_jobs)),
          ("verbose", w.v(clf.verbose)), ("passthrough", w.v(clf.passthrough)), ("_le", le),
          ("classes_", le_classes),
          ("final_estimator_", w.est(clf.final_estimator_, fitted=True)),
          ("estimators_", sp.ListN(fitted))]
    name_nodes = [t.items[0] for t in templates.items]
    bunch = sp.Call(b.g(*_CLS["bunch"]), sp.TupleN([]), newobj=True,
                    dictitems=list(zip(name_nodes, fitted)))
    sm = w.s("predict_proba")
    st += [("named_estimators_", bunch), ("stack_method_", sp.ListN([sm] * len(fitted)))]
    return w.obj("stack", st + w.version())


def save_checkpoint(clf: StackingClassifier, path: str) -> bytes:
    data = sp.emit(checkpoint_graph(clf))
    with open(path, "wb") as f:
        f.write(data)
    return data
