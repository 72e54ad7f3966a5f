"""Training surface (§8f "next" H6): ``partial_fit`` of FM, HHFM, DeepFM and
AFM on the gfx950 train-step kernels and the reference's epoch loops.

* FM / AFM / DFM loop — FM.py:221-282: each epoch NG=2 negatives per
  positive (label 0 for FM, -1 for AFM/DFM, FM.py:248 / AFM.py:317), shuffle,
  ``partial_fit`` over ``batch_size`` chunks, evaluation every ``verbose``
  epochs (or the loss-plateau rule when ``Result == 1``).
* HHFM loop — OurModel7.py:364-413: shuffle the train rows in place, NG=10
  negatives per row, BPR-max ``partial_fit``, evaluation every 10 epochs.
Result lines are printed and appended to ``args.result_file`` (the
reference's ``../result.txt``).
"""
from __future__ import annotations

from time import time

import numpy as np
import torch

from . import ops
from .harness import partition_all
from ._native import native

# --optimizer names (FM.py:129-136, AFM.py:151-158, OurModel7.py:186-193) -> the
# train kernels' optimizer codes (include/hhfm.h)
_OPT = {"AdagradOptimizer": 0, "GradientDescentOptimizer": 1, "MomentumOptimizer": 2,
        "AdamOptimizer": 3}
_SGD = 1


def _opt_code(model):
    try:
        return _OPT[model.optimizer_type]
    except KeyError:
        raise NotImplementedError(f"optimizer {model.optimizer_type!r} (the reference accepts "
                                  f"{', '.join(_OPT)})") from None


def _slots(opt, t):
    """The optimizer's slot array for variable ``t``: Adagrad's accumulator
    (TF initial_accumulator_value 0.1), Momentum's zeroed accumulator, Adam's
    zeroed m then v (2 × numel); SGD keeps none (a 1-element placeholder)."""
    if opt == 0:
        return torch.full_like(t, 0.1)
    if opt == 2:
        return torch.zeros_like(t)
    if opt == 3:
        return torch.zeros(2 * t.numel(), dtype=t.dtype, device=t.device)
    return torch.zeros(1, dtype=t.dtype, device=t.device)


def _state(model, names, opt):
    """Optimizer slots (``_slots``) + the zeroed gradient workspace (which also
    carries Adam's β1^t, β2^t), created on first use."""
    st = getattr(model, "_train_state", None)
    if st is not None and st.get("opt") != opt:
        raise ValueError("the optimizer changed after the first partial_fit")
    if st is None:
        if model.table_dtype != torch.float32:
            raise NotImplementedError("training runs on fp32 tables")
        st = {n: _slots(opt, model.weights[n]) for n in names}
        st["opt"] = opt
        k = model.weights["feature_embeddings"].shape[1]
        nbytes = native().train_workspace(model.features_M, k)
        st["ws"] = torch.zeros(nbytes, dtype=torch.uint8, device=model.device)
        st["loss"] = torch.zeros(1, dtype=torch.float32, device=model.device)
        model._train_state = st
    return st


def _grow(old, nbytes, state_bytes, dev):
    """A zero-filled train workspace of ``nbytes``; only the persistent prefix
    of the old one (``state_bytes``: include/hhfm.h hhfm_*_train_state_bytes —
    gradients, Adam's β powers, the touched mask) carried over, the per-batch
    scratch after it left zeroed."""
    ws = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    if old is not None:
        ws[:state_bytes].copy_(old[:state_bytes])
    return ws


def fm_partial_fit(model, data) -> float:
    """FM.partial_fit (FM.py:168-171): one optimizer step, returns the loss."""
    opt = _opt_code(model)
    if model.keep != 1:
        raise NotImplementedError("dropout keep < 1 is not implemented")
    W = model.weights
    st = _state(model, ["feature_embeddings", "feature_bias", "bias"], opt)
    X = model._idx(data["X"])
    y = torch.as_tensor(np.asarray(data["Y"], np.float32).reshape(-1)).to(model.device)
    B, F = X.shape
    M, k = W["feature_embeddings"].shape
    dev = model.device
    native().fm_train_step(X.data_ptr(), y.data_ptr(), B, F, W["feature_embeddings"].data_ptr(),
                           W["feature_bias"].data_ptr(), W["bias"].data_ptr(), M, k,
                           float(model.learning_rate), float(model.lamda_bilinear), opt,
                           st["feature_embeddings"].data_ptr(), st["feature_bias"].data_ptr(),
                           st["bias"].data_ptr(), st["ws"].data_ptr(), st["ws"].numel(),
                           st["loss"].data_ptr(), ops._stream(dev))
    return float(st["loss"].item())


def hhfm_partial_fit(model, data) -> float:
    """OUR.partial_fit (OurModel7.py:219-228): data X [B,2], Y [B,NG] negatives,
    F1 ctx columns, F2 time columns."""
    opt = _opt_code(model)
    W = model.weights
    st = _state(model, ["feature_embeddings"], opt)
    parts = [np.asarray(data["X"])]
    if model.context:
        parts.append(np.asarray(data["F1"]))
    if model.time:
        parts.append(np.asarray(data["F2"]))
    X = model._idx(np.concatenate(parts, axis=1))
    Neg = model._idx(np.asarray(data["Y"]))
    B, ncols = X.shape
    ctx, tim = model._ranges(ncols)
    M, k = W["feature_embeddings"].shape
    native().hhfm_train_step(X.data_ptr(), Neg.data_ptr(), B, ncols, ctx[0], ctx[1], tim[0],
                             tim[1], Neg.shape[1], W["feature_embeddings"].data_ptr(), M, k,
                             float(model.learning_rate), float(model.lamda_bilinear), opt,
                             st["feature_embeddings"].data_ptr(), st["ws"].data_ptr(),
                             st["ws"].numel(), st["loss"].data_ptr(),
                             ops._stream(model.device))
    return float(st["loss"].item())


def dfm_partial_fit(model, data) -> float:
    """DeepFM.partial_fit (DFM.py:214-217): one TF Adagrad step on every
    variable (DFM.py:155), loss l2_loss(y − out) + l2_reg on the concat
    projection and the layer weights (DFM.py:143-152)."""
    W = model.weights
    L = len(model.deep_layers)
    names = (["feature_embeddings", "feature_bias"] + [f"layer_{i}" for i in range(L)]
             + [f"bias_{i}" for i in range(L)] + ["concat_projection", "concat_bias"])
    st = getattr(model, "_train_state", None)
    if st is None:
        if model.table_dtype != torch.float32:
            raise NotImplementedError("training runs on fp32 tables")
        st = {n: _slots(0, W[n]) for n in names}
        st["loss"] = torch.zeros(1, dtype=torch.float32, device=model.device)
        st["ws"], st["ws_rows"] = None, 0
        model._train_state = st
    X = model._idx(data["X"])
    y = torch.as_tensor(np.asarray(data["Y"], np.float32).reshape(-1)).to(model.device)
    B, F = X.shape
    M, k = W["feature_embeddings"].shape
    dims = [int(d) for d in model.deep_layers]
    nat = native()
    if st["ws"] is None or st["ws_rows"] < B:
        nbytes = nat.dfm_train_workspace(B, F, k, M, dims)
        st["ws"] = _grow(st["ws"], nbytes, nat.dfm_train_state_bytes(F, k, M, dims),
                         model.device)
        st["ws_rows"] = B
    ptr = lambda n: W[n].data_ptr()  # noqa: E731
    nat.dfm_train_step(X.data_ptr(), y.data_ptr(), B, F, ptr("feature_embeddings"),
                       ptr("feature_bias"), M, k, dims, [ptr(f"layer_{i}") for i in range(L)],
                       [ptr(f"bias_{i}") for i in range(L)], ptr("concat_projection"),
                       ptr("concat_bias"), float(model.learning_rate), float(model.l2_reg), 0,
                       [st[n].data_ptr() for n in names], st["ws"].data_ptr(), st["ws"].numel(),
                       st["loss"].data_ptr(), ops._stream(model.device))
    model._prep = None   # the scoring path's prepared (transposed / bf16) weights are stale
    return float(st["loss"].item())


def afm_partial_fit(model, data) -> float:
    """AFM.partial_fit (AFM.py:205-207): one TF step on every variable, loss
    l2_loss(y − out) + l2_regularizer(λ)(attention_W) when λ > 0 (AFM.py:144-148)."""
    opt = _opt_code(model)
    if any(float(x) != 1.0 for x in np.ravel(model.keep)):
        raise NotImplementedError("dropout keep < 1 is not implemented")
    W = model.weights
    names = ["feature_embeddings", "feature_bias", "bias", "attention_W", "attention_b",
             "attention_p", "prediction"]
    st = getattr(model, "_train_state", None)
    if st is not None and st.get("opt") != opt:
        raise ValueError("the optimizer changed after the first partial_fit")
    if st is None:
        if model.table_dtype != torch.float32:
            raise NotImplementedError("training runs on fp32 tables")
        st = {n: _slots(opt, W[n]) for n in names}
        st["opt"] = opt
        st["loss"] = torch.zeros(1, dtype=torch.float32, device=model.device)
        st["ws"], st["ws_rows"] = None, 0
        model._train_state = st
    X = model._idx(data["X"])
    y = torch.as_tensor(np.asarray(data["Y"], np.float32).reshape(-1)).to(model.device)
    B, F = X.shape
    M, k = W["feature_embeddings"].shape
    A = W["attention_W"].shape[1]
    nat = native()
    if st["ws"] is None or st["ws_rows"] < B:
        nbytes = nat.afm_train_workspace(B, F, k, A, M)
        st["ws"] = _grow(st["ws"], nbytes, nat.afm_train_state_bytes(F, k, A, M), model.device)
        st["ws_rows"] = B
    lam = float(model.lamda_attention) if model.lamda_attention > 0 else 0.0
    ptr = lambda n: W[n].data_ptr()  # noqa: E731
    nat.afm_train_step(X.data_ptr(), y.data_ptr(), B, F, ptr("feature_embeddings"),
                       ptr("feature_bias"), ptr("bias"), M, k, A, ptr("attention_W"),
                       ptr("attention_b"), ptr("attention_p"), ptr("prediction"),
                       float(model.learning_rate), lam, opt,
                       [st[n].data_ptr() for n in names] if opt != _SGD else [],
                       st["ws"].data_ptr(), st["ws"].numel(), st["loss"].data_ptr(),
                       ops._stream(model.device))
    return float(st["loss"].item())


def _log(tr, line):
    print(line)
    path = getattr(tr.args, "result_file", None)
    if path:
        with open(path, "a") as f:
            f.write(line + "\n")


def _evaluate(tr):
    return (tr.evaluate_AUC(tr.data.Train_data), tr.evaluate_AUC(tr.data.Test_data),
            tr.evaluate_TopK(tr.data.Test_data))


def _report(tr, head, t_epoch, t_eval0, res):
    a1, a2, tk = res
    _log(tr, "%s [%.1f s]\ttrain=AUC:%.4f;test=AUC:%.4f,HR:%.4f,NDCG:%.4f,PRE:%.4f;[%.1f s]"
         % (head, t_epoch, a1, a2, tk[0], tk[1], tk[2], time() - t_eval0))


def run_training(tr, negatives=2, neg_label=0, plateau=-0.0075, epoch_cap=100):
    """FM.py:221-282 (also AFM.py:290-351, DFM.py:259-320).  The loss-plateau
    stop (Result == 1) is ``plateau`` = −0.0075 with a 100-epoch cap in FM
    (FM.py:261-262), −0.0075 without a cap in DFM (DFM.py:299-300) and −0.01
    without a cap in AFM (AFM.py:330-331)."""
    args = tr.args
    t2 = time()
    if args.Result == 0:
        res = _evaluate(tr)
        a1, a2, tk = res
        _log(tr, "Dataset=%s %s Init: \t train=AUC:%.4f;test=AUC:%.4f,HR:%.4f,NDCG:%.4f,PRE:%.4f;"
             "[%.1f s]" % (args.dataset, tr.method, a1, a2, tk[0], tk[1], tk[2], time() - t2))
    tr.loss_epoch = []
    for epoch in range(1, tr.epoch):
        loss = 0.0
        t1 = time()
        pos = tr.data.Train_data.values
        rep = np.repeat(np.array(pos, copy=True)[:, None, :], negatives, axis=1)
        rep = rep.reshape(-1, rep.shape[2])
        negs = tr.sample_negative(pos[:, 1:], negatives)
        rep[:, 2] = negs.reshape(-1)
        rep[:, 0] = neg_label
        dat = np.append(pos, rep, axis=0)
        np.random.shuffle(dat)
        for chunk in partition_all(tr.batch_size, range(len(dat))):
            X = np.array(dat[chunk][:, 1:], dtype=np.int64)
            Y = np.expand_dims(dat[chunk][:, 0], axis=1)
            loss = loss + tr.model.partial_fit({"X": X, "Y": Y})
        tr.loss_epoch.append(loss)
        t2 = time()
        if args.Result == 1 and epoch > 30:
            n = 3
            le = np.array(tr.loss_epoch)
            cond = np.sum((le[-1 - n:-1] / le[-2 - n:-2] - 1) > plateau)
            if cond == n or (epoch_cap is not None and epoch > epoch_cap):
                _report(tr, "%s%s Epoch %d" % (args.dataset, tr.method, epoch), t2 - t1, t2,
                        _evaluate(tr))
                break
        if args.Result == 0 and tr.verbose > 0 and epoch % tr.verbose == 0:
            _report(tr, "%s Epoch %d" % (tr.method, epoch), t2 - t1, t2, _evaluate(tr))
    return tr.loss_epoch


def run_training_hhfm(tr):
    """OurModel7.py:349-413."""
    args = tr.args
    t2 = time()
    if args.Result == 0:
        res = _evaluate(tr)
        a1, a2, tk = res
        _log(tr, "Dataset=%s %s Init: \t train=AUC:%.4f;test=AUC:%.4f,HR:%.4f,NDCG:%.4f,PRE:%.4f;"
             "[%.1f s]" % (args.dataset, tr.method, a1, a2, tk[0], tk[1], tk[2], time() - t2))
    tr.loss_epoch = []
    td = tr.time_dimension
    for epoch in range(1, tr.epoch):
        loss = 0.0
        t1 = time()
        pos = tr.data.Train_data.values[:, 1:]
        np.random.shuffle(pos)            # in place, like the reference (:369-370)
        NG = 10
        negs = tr.sample_negative(pos, NG)
        for chunk in partition_all(tr.batch_size, range(len(pos))):
            rows = pos[chunk]
            batch = {"X": np.array(rows[:, :2], dtype=np.int64),
                     "Y": np.array(negs[chunk], dtype=np.int64)}
            if tr.context and tr.time:
                batch["F1"] = np.array(rows[:, 2:-td], dtype=np.int64)
                batch["F2"] = np.array(rows[:, -td:], dtype=np.int64)
            elif tr.context:
                batch["F1"] = np.array(rows[:, 2:], dtype=np.int64)
            else:
                batch["F2"] = np.array(rows[:, 2:], dtype=np.int64)
            loss = loss + tr.model.partial_fit(batch)
        tr.loss_epoch.append(loss)
        t2 = time()
        if args.Result == 1 and epoch > 20:
            n = 3
            le = np.array(tr.loss_epoch)
            cond = np.sum((le[-1 - n:-1] / le[-2 - n:-2] - 1) > -0.0075)
            if cond == n or epoch > 100:
                _report(tr, "%s%s Epoch %d" % (args.dataset, tr.method, epoch), t2 - t1, t2,
                        _evaluate(tr))
                break
        if args.Result == 0 and epoch % 10 == 0:
            _report(tr, "%s Epoch %d" % (tr.method, epoch), t2 - t1, t2, _evaluate(tr))
    return tr.loss_epoch
