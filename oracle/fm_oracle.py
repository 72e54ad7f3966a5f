"""CPU oracle — TEST INFRASTRUCTURE ONLY.

A numpy restatement, op for op, of the reference's TensorFlow-1.x scoring
graphs (data-man-34/HHFM, Newcode/*.py).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use
this module, and only as the checker: the product path (``hhfm_amd``) never
imports it and fails loudly when its HIP extension is missing.

Third-party dependency restated: TensorFlow 1.x (unpinned in the reference —
no requirements file; ``Newcode/__pycache__`` is CPython 3.6 bytecode and the
code uses ``tf.contrib``/``keep_dims``/``tf.Session``, i.e. TF 1.5–1.15).
Ops restated with their published semantics: ``embedding_lookup`` (row
gather), ``reduce_sum``/``reduce_max``, elementwise ``square``/``multiply``/
``subtract``/``add_n``, ``matmul``, ``nn.relu``, ``nn.softmax``, ``exp``,
``concat`` and ``nn.top_k`` (sorted=True: descending values, equal values
keep the lower index first).  All arithmetic is float32 like the reference
graphs; reductions are numpy's (TF's Eigen reduction order is not
reproducible without TF — scores are compared with a tolerance, index sets
exactly where the score gap exceeds it).

Parity pinning: these functions are checked against golden vectors produced
by running the reference's own model classes (``Newcode/FM.py``,
``OurModel7.py``, ``AFM.py``, ``DFM.py``) on a numpy evaluation of the TF1
ops (``tests/golden/make_golden.py``), see ``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def _emb(E, ids):
    """tf.nn.embedding_lookup: row gather (E stays float32)."""
    return np.asarray(E, dtype=F32)[np.asarray(ids, dtype=np.int64)]


def top_k(score: np.ndarray, k: int):
    """tf.nn.top_k(score, k) on the last axis: values and indices sorted by
    value descending; ties broken by lower index first (stable sort)."""
    score = np.asarray(score, dtype=F32)
    order = np.argsort(-score, axis=-1, kind="stable")[..., :k]
    return np.take_along_axis(score, order, axis=-1), order.astype(np.int32)


# ---------------------------------------------------------------------------
# M1 — FM.out  (Newcode/FM.py:99-120)
# ---------------------------------------------------------------------------
def fm_out(X, E, w, w0=0.0):
    """out = Σ_k ½[(Σ_f e)² − Σ_f e²] + Σ_f w + w0, shape [B,1].

    FM.py:99   nonzero_embeddings = embedding_lookup(E, X)        [B,F,k]
    FM.py:100  summed = reduce_sum(., 1, keep_dims)               [B,1,k]
    FM.py:102  summed_square = square(summed)
    FM.py:105  squared = square(nonzero_embeddings)
    FM.py:106  squared_sum = reduce_sum(squared, 1, keep_dims)
    FM.py:109  FM = 0.5 * (summed_square - squared_sum)
    FM.py:113  FM_OUT = reduce_sum(FM, 1)                         [B,k]
    FM.py:114  dropout(keep=1) -> identity; batch_norm=0 (:111) -> skipped
    FM.py:117  Bilinear = reduce_sum(FM_OUT, 1, keep_dims)        [B,1]
    FM.py:118  Feature_bias = reduce_sum(embedding_lookup(w, X), 1)
    FM.py:119  Bias = w0 * ones_like(labels)
    FM.py:120  out = add_n([Bilinear, Feature_bias, Bias])
    """
    e = _emb(E, X)
    summed = e.sum(axis=1, keepdims=True, dtype=F32)
    sq_sum = np.square(e).sum(axis=1, keepdims=True, dtype=F32)
    fm = F32(0.5) * (np.square(summed) - sq_sum)
    fm_out_ = fm.sum(axis=1, dtype=F32)
    bil = fm_out_.sum(axis=1, keepdims=True, dtype=F32)
    if w is None:
        fb = np.zeros_like(bil)
    else:
        fb = _emb(np.asarray(w, F32).reshape(-1, 1), X).sum(axis=1, dtype=F32)
    return (bil + fb) + F32(w0)


# ---------------------------------------------------------------------------
# M2 — FM.topk  (Newcode/FM.py:172-198)
# ---------------------------------------------------------------------------
def fm_catalog_scores(A, E, w, n_user, n_item):
    """bias + score, shape [B, n_item] (FM.py:174-184).

    FM.py:174  user = lookup(E, A[:,0])
    FM.py:175  item = lookup(E, n_user .. n_user+n_item-1)
    FM.py:176  feature = reduce_sum(lookup(E, A[:,2:]), axis=1)
    FM.py:177  UserWithFeature = user + feature
    FM.py:178  ItemWithFeature = item[None] + feature[:,None]
    FM.py:180  mul = UserWithFeature[:,None] * ItemWithFeature
    FM.py:183  score = reduce_sum(mul, 2)
    FM.py:184  bias = transpose(lookup(w, items))   [1,N]
    FM.py:185  top_k(bias + score, tp)
    """
    A = np.asarray(A)
    user = _emb(E, A[:, 0])
    item = _emb(E, np.arange(n_user, n_user + n_item))
    feature = _emb(E, A[:, 2:]).sum(axis=1, dtype=F32)
    uwf = user + feature
    iwf = item[None, :, :] + feature[:, None, :]
    score = (uwf[:, None, :] * iwf).sum(axis=2, dtype=F32)
    if w is None:
        return score
    bias = np.asarray(w, F32).reshape(-1)[n_user:n_user + n_item][None, :]
    return bias + score


def fm_topk(A, E, w, n_user, n_item, tp=20):
    return top_k(fm_catalog_scores(A, E, w, n_user, n_item), tp)


# ---------------------------------------------------------------------------
# H1/H2 — HHFM (OurModel7), sum pooling (OurModel7.py:14-19)
# ---------------------------------------------------------------------------
def _hybrid(E, user_ids, ctx_ids=None, time_ids=None):
    """Σ over stack[user, Σctx, (Σtime)] (OurModel7.py:122-168, 244-292)."""
    stack = [_emb(E, user_ids)]
    if ctx_ids is not None:
        stack.append(_emb(E, ctx_ids).sum(axis=1, dtype=F32))   # :124 / :255
    if time_ids is not None:
        stack.append(_emb(E, time_ids).sum(axis=1, dtype=F32))  # :141 / :267
    out = stack[0]
    for s in stack[1:]:
        out = out + s                                            # :168 / :292
    return out


def hhfm_split(X, feature_dimension, time_dimension, context=True, time=False):
    """The reference's column split of a row [user, item, ctx..., time...]
    (partial_fit feeds, OurModel7.py:374-385; topk, :236-242)."""
    X = np.asarray(X)
    ctx = tim = None
    if context and time:
        ctx = X[:, 2:-time_dimension]
        tim = X[:, -time_dimension:]
    elif context:
        ctx = X[:, 2:]
    elif time:
        tim = X[:, 2:]
    return ctx, tim


def hhfm_positive_feedback(X, E, feature_dimension, time_dimension,
                           context=True, time=False):
    """PositiveFeadback = reduce_sum(hybrid * E[item], 1, keep_dims) [B,1]
    (OurModel7.py:171)."""
    X = np.asarray(X)
    ctx, tim = hhfm_split(X, feature_dimension, time_dimension, context, time)
    h = _hybrid(E, X[:, 0], ctx, tim)
    it = _emb(E, X[:, 1])
    return (h * it).sum(axis=1, keepdims=True, dtype=F32)


def hhfm_catalog_scores(A, E, n_user, n_item, feature_dimension,
                        time_dimension, context=True, time=False):
    """score = reduce_sum(hybrid[:,None] * items[None], 2) (OurModel7.py:294)."""
    A = np.asarray(A)
    ctx, tim = hhfm_split(A, feature_dimension, time_dimension, context, time)
    h = _hybrid(E, A[:, 0], ctx, tim)
    item = _emb(E, np.arange(n_user, n_user + n_item))
    return (h[:, None, :] * item[None, :, :]).sum(axis=2, dtype=F32)


def hhfm_topk(A, E, n_user, n_item, feature_dimension, time_dimension,
              context=True, time=False, tp=20):
    return top_k(hhfm_catalog_scores(A, E, n_user, n_item, feature_dimension,
                                     time_dimension, context, time), tp)


# ---------------------------------------------------------------------------
# helpers for comparing GPU results with the oracle
# ---------------------------------------------------------------------------
def topk_swaps(ref_scores, ref_idx, got_idx, tol):
    """Exactness check of a top-K index list against the oracle's.

    ``ref_scores`` [B, N] are the oracle's scores of every item, ``ref_idx``
    the oracle's top-K.  Every position where ``got_idx`` differs must be a
    tie in the oracle's own scores: |score(got) - score(ref)| <= tol (per
    query), i.e. two fp32 summation orders may legally order that pair either
    way.  Returns (n_unexplained, n_tie_swaps); callers assert the first is 0
    and report (and bound) the second."""
    ref_scores = np.asarray(ref_scores)
    ref_idx = np.asarray(ref_idx)
    got_idx = np.asarray(got_idx)
    B, K = ref_idx.shape
    tol = np.broadcast_to(np.asarray(tol, dtype=np.float64).reshape(-1, 1)
                          if np.ndim(tol) else np.float64(tol), (B, 1))
    unexplained = swaps = 0
    for b, p in np.argwhere(got_idx != ref_idx):
        g, r = int(got_idx[b, p]), int(ref_idx[b, p])
        if 0 <= g < ref_scores.shape[1] and \
                abs(float(ref_scores[b, g]) - float(ref_scores[b, r])) <= tol[b, 0]:
            swaps += 1
        else:
            unexplained += 1
    return unexplained, swaps


# ---------------------------------------------------------------------------
# A1/A2 — AFM (Newcode/AFM.py)
# ---------------------------------------------------------------------------
def _pairs(e):
    """element_wise_product_list over i<j (AFM.py:107-112) -> [B, P, k]."""
    F = e.shape[1]
    return np.stack([e[:, i, :] * e[:, j, :] for i in range(F) for j in range(i + 1, F)], 1)


def _att_logit(p, W, b, pvec):
    """Σ_A p * relu(reshape(p,[-1,k]) @ W + b)  (AFM.py:117-124, 221-224)."""
    shp = p.shape
    mul = np.matmul(p.reshape(-1, shp[-1]), W).astype(F32).reshape(*shp[:-1], W.shape[1])
    return (np.asarray(pvec, F32) * np.maximum(mul + np.asarray(b, F32).reshape(-1), 0)).sum(
        axis=-1, keepdims=True, dtype=F32)


def afm_out(X, E, w, w0, W, b, pvec, P):
    """AFM.out (AFM.py:103-142), attention=1, keep=[1,1] -> [B,1]."""
    e = _emb(E, X)
    pr = _pairs(e)                                           # [B,P,k]
    logit = _att_logit(pr, W, b, pvec)                       # [B,P,1]
    ex = np.exp(logit - logit.max(axis=1, keepdims=True))
    att = (ex / ex.sum(axis=1, keepdims=True)).astype(F32)   # softmax axis=1 (:125)
    afm = (att * pr).sum(axis=1, dtype=F32)                  # [B,k]      (:130)
    bil = np.matmul(afm, np.asarray(P, F32)).sum(axis=1, keepdims=True, dtype=F32)  # :138-139
    fb = _emb(np.asarray(w, F32).reshape(-1, 1), X).sum(axis=1, dtype=F32)          # :140
    return (bil + fb) + F32(w0)                                                     # :142


def afm_catalog_scores(A, E, w, W, b, pvec, P, n_user, n_item):
    """score3 + bias of AFM.topk (AFM.py:210-243) -> [B, N]."""
    A = np.asarray(A)
    uf = np.concatenate([_emb(E, A[:, 0])[:, None, :], _emb(E, A[:, 2:])], axis=1)  # :210-212
    ufp = _pairs(uf)                                                  # [B,C,k]  :214-220
    a_uf = np.exp(_att_logit(ufp, W, b, pvec))                        # [B,C,1]  :221-224
    item = _emb(E, np.arange(n_user, n_user + n_item))                # [N,k]    :226
    ufi = uf[:, None, :, :] * item[None, :, None, :]                  # [B,N,uf,k] :227
    a_ufi = np.exp(_att_logit(ufi, W, b, pvec))                       # [B,N,uf,1] :228-230
    ufw = (ufp * a_uf).sum(axis=1, dtype=F32)                         # [B,k]    :232
    iufw = (ufi * a_ufi).sum(axis=2, dtype=F32)                       # [B,N,k]  :233
    s1 = ufw[:, None, :] + iufw                                       # :234
    wt = a_uf.sum(axis=1, dtype=F32)[:, None, :] + a_ufi.sum(axis=2, dtype=F32)  # :235
    s2 = s1 / wt                                                      # :236
    s3 = (s2 * np.asarray(P, F32).T).sum(axis=2, dtype=F32)           # :239
    bias = np.asarray(w, F32).reshape(-1)[n_user:n_user + n_item][None, :]  # :240
    return s3 + bias                                                  # :243


# ---------------------------------------------------------------------------
# D1/D2 — DeepFM (Newcode/DFM.py)
# ---------------------------------------------------------------------------
def dfm_out(X, E, w, layers, biases, Wp, bp):
    """DeepFM.out (DFM.py:104-137), use_fm = use_deep = True, loss 'mse'."""
    X = np.asarray(X)
    e = _emb(E, X)                                                    # :104
    y1 = _emb(np.asarray(w, F32).reshape(-1, 1), X).sum(axis=2, dtype=F32)   # :109-110 [B,F]
    s = e.sum(axis=1, dtype=F32)                                      # :114
    y2 = F32(0.5) * (np.square(s) - np.square(e).sum(axis=1, dtype=F32))     # :115-122
    y = e.reshape(-1, e.shape[1] * e.shape[2])                        # :125
    for Wl, bl in zip(layers, biases):                                # :126-128 (relu on every layer)
        y = np.maximum(np.matmul(y, np.asarray(Wl, F32)).astype(F32) + np.asarray(bl, F32), 0)
    cat = np.concatenate([y1, y2, y], axis=1)                         # :132
    return np.matmul(cat, np.asarray(Wp, F32)).astype(F32) + F32(bp)  # :137


def dfm_catalog_rows(A, n_user, n_item):
    """DeepFM.topk's candidate rows (DFM.py:220-223): each query tiled over all
    items with column 1 replaced by the item id -> [B*N, F]."""
    A = np.asarray(A, dtype=np.int64)
    neg = np.repeat(A[:, None, :], n_item, axis=1)
    neg[:, :, 1] = np.arange(n_user, n_user + n_item)[None, :]
    return neg.reshape(-1, A.shape[1])


def dfm_catalog_scores(A, E, w, layers, biases, Wp, bp, n_user, n_item):
    rows = dfm_catalog_rows(A, n_user, n_item)
    return dfm_out(rows, E, w, layers, biases, Wp, bp).reshape(-1, n_item)  # :228


# ---------------------------------------------------------------------------
# H6 — one training step with TF-1.x semantics (loss + gradient + optimizer)
# ---------------------------------------------------------------------------
def tf_adagrad(var, grad, acc, lr):
    """tf.train.AdagradOptimizer (ApplyAdagrad): accum += g²; var -= lr·g·rsqrt(accum).
    Accumulators start at initial_accumulator_value = 0.1 (TF default)."""
    acc = (acc + grad * grad).astype(F32)
    return (var - F32(lr) * grad / np.sqrt(acc)).astype(F32), acc


MOMENTUM, BETA1, BETA2, ADAM_EPS = F32(0.95), F32(0.9), F32(0.999), F32(1e-8)


def _ftz(x):
    """float32 flush-to-zero: TF's CPU thread pools run every op with the
    FTZ/DAZ flags set (core/lib/core/threadpool.cc, EigenEnvironment::
    CreateThread: port::ScopedFlushDenormal), so a product below FLT_MIN is 0."""
    x = F32(x)
    return F32(0) if abs(x) < np.finfo(F32).tiny else x


def adam_powers(step):
    """TF AdamOptimizer's beta1_power / beta2_power at ``step`` (1-based):
    created at β1, β2 and multiplied by β in float32 after every step
    (_finish), under flush-to-zero: β1^t reaches exactly 0 at t = 829 and
    stays there (α = lr·√(1−β2^t) from then on)."""
    b1p, b2p = BETA1, BETA2
    for _ in range(step - 1):
        b1p, b2p = _ftz(b1p * BETA1), _ftz(b2p * BETA2)
    return b1p, b2p


def tf_apply(optimizer, var, grad, slot, lr, step=1, rows=None):
    """One TF-1.x optimizer update of ``var`` (FM.py:129-136, AFM.py:151-158,
    OurModel7.py:186-193).  ``rows``: None for a dense gradient, else the ids of
    the IndexedSlices an embedding_lookup produced (duplicates allowed; TF sums
    them first).  slot: Adagrad's accumulator, Momentum's accumulator, Adam's
    m and v stacked as a flat [2·n] array, None for SGD.  Returns (var, slot).
    * Adagrad (ApplyAdagrad; the sparse kernel is the same on touched rows and
      a no-op on the others): accum += g²; var -= lr·g/√accum.
    * Momentum(0.95) dense: accum = accum·0.95 + g; var -= lr·accum; sparse:
      the same on the touched rows only.
    * Adam(0.9, 0.999, 1e-8), α = lr·√(1−β2^t)/(1−β1^t): dense ApplyAdam
      m += (g−m)(1−β1), v += (g²−v)(1−β2); sparse (_apply_sparse_shared)
      m = m·β1 + g(1−β1), v = v·β2 + g²(1−β2) on every row; var -= α·m/(√v+ε)."""
    var = np.asarray(var, F32)
    g = np.asarray(grad, F32).reshape(var.shape)
    lr = F32(lr)
    if optimizer == "adagrad":
        return tf_adagrad(var, g, np.asarray(slot, F32).reshape(var.shape), lr)
    if optimizer == "sgd":
        return (var - lr * g).astype(F32), slot
    if optimizer == "momentum":
        acc = np.asarray(slot, F32).reshape(var.shape).copy()
        if rows is None:
            acc = (acc * MOMENTUM + g).astype(F32)
            return (var - acc * lr).astype(F32), acc
        var = var.copy()
        t = np.unique(np.asarray(rows, np.int64).reshape(-1))
        acc[t] = acc[t] * MOMENTUM + g[t]
        var[t] = var[t] - acc[t] * lr
        return var, acc
    if optimizer == "adam":
        mv = np.asarray(slot, F32).reshape(2, *var.shape)
        m, v = mv[0], mv[1]
        b1p, b2p = adam_powers(step)
        alpha = F32(lr * np.sqrt(F32(1) - b2p, dtype=F32) / (F32(1) - b1p))
        if rows is None:
            m = (m + (g - m) * (F32(1) - BETA1)).astype(F32)
            v = (v + (g * g - v) * (F32(1) - BETA2)).astype(F32)
        else:
            m = (m * BETA1 + g * (F32(1) - BETA1)).astype(F32)
            v = (v * BETA2 + (g * g) * (F32(1) - BETA2)).astype(F32)
        var = (var - (m * alpha) / (np.sqrt(v) + ADAM_EPS)).astype(F32)
        return var, np.stack([m, v]).reshape(-1)
    raise ValueError(f"optimizer {optimizer!r}")


def fm_train_step(X, y, E, w, w0, accE, accw, accw0, lr, lam, optimizer="adagrad", step=1):
    """FM partial_fit (FM.py:123-136, 168-171): loss = Σ(y−out)²/2 + λ·ΣE²/2.
    Returns (loss, E, w, w0, accE, accw, accw0) after one update."""
    X = np.asarray(X, np.int64)
    y = np.asarray(y, F32).reshape(-1)
    E = np.asarray(E, F32)
    w = np.asarray(w, F32).reshape(-1)
    out = fm_out(X, E, w, w0)[:, 0]
    r = y - out
    loss = F32(np.sum(r * r, dtype=np.float64) / 2 + lam * np.sum(E.astype(np.float64) ** 2) / 2)
    g = -r                                                     # d loss / d out
    e = E[X]
    s = e.sum(1)
    dE = np.zeros_like(E)
    for f in range(X.shape[1]):
        np.add.at(dE, X[:, f], g[:, None] * (s - e[:, f]))     # ∂out/∂e_f = Σe − e_f
    dE += F32(lam) * E                                         # l2_regularizer
    dw = np.zeros_like(w)
    for f in range(X.shape[1]):
        np.add.at(dw, X[:, f], g)
    dw0 = F32(g.sum())
    # E is an IndexedSlices unless the l2 term adds a dense gradient; w always is
    E, accE = tf_apply(optimizer, E, dE, accE, lr, step, X if lam == 0 else None)
    w, accw = tf_apply(optimizer, w, dw, accw, lr, step, X)
    w0n, accw0 = tf_apply(optimizer, np.float32(w0), dw0, accw0, lr, step)
    return loss, E, w, F32(w0n), accE, accw, accw0


def hhfm_train_step(X, Neg, E, accE, lr, lam, feature_dimension, time_dimension,
                    context=True, time=False, optimizer="adagrad", step=1):
    """OUR partial_fit (OurModel7.py:171-193): loss = −Σ log σ(pos − max_j neg_j)
    + λ·ΣE²/2; reduce_max's gradient is split equally between tied maxima."""
    X = np.asarray(X, np.int64)
    Neg = np.asarray(Neg, np.int64)
    E = np.asarray(E, F32)
    ctx, tim = hhfm_split(X, feature_dimension, time_dimension, context, time)
    h = _hybrid(E, X[:, 0], ctx, tim)
    it = E[X[:, 1]]
    pos = (h * it).sum(1, dtype=F32)
    neg = (h[:, None, :] * E[Neg]).sum(2, dtype=F32)
    mx = neg.max(1)
    z = pos - mx
    sg = (1.0 / (1.0 + np.exp(-z))).astype(F32)
    loss = F32(-np.sum(np.log(sg), dtype=np.float64) + lam * np.sum(E.astype(np.float64) ** 2) / 2)
    g = sg - F32(1)
    ind = (neg == mx[:, None]).astype(F32)
    ind /= ind.sum(1, keepdims=True)
    dh = g[:, None] * (it - (ind[:, :, None] * E[Neg]).sum(1))
    dE = np.zeros_like(E)
    np.add.at(dE, X[:, 1], g[:, None] * h)
    for j in range(Neg.shape[1]):
        np.add.at(dE, Neg[:, j], -(g * ind[:, j])[:, None] * h)
    np.add.at(dE, X[:, 0], dh)
    for cols in (ctx, tim):
        if cols is not None:
            for c in range(cols.shape[1]):
                np.add.at(dE, np.asarray(cols)[:, c].astype(np.int64), dh)
    dE += F32(lam) * E
    rows = np.concatenate([X.reshape(-1), Neg.reshape(-1)]) if lam == 0 else None
    E, accE = tf_apply(optimizer, E, dE, accE, lr, step, rows)
    return loss, E, accE


def dfm_train_step(X, y, E, w, layers, biases, Wp, bp, acc, lr, lam, optimizer="adagrad",
                   step=1):
    """DeepFM partial_fit (DFM.py:139-155, 214-217), use_fm = use_deep = True,
    loss_type "mse": loss = l2_loss(y − out) + λ·(‖Wp‖² + Σ_l ‖W_l‖²)/2
    (l2_regularizer on concat_projection and every layer_i; not on the
    embeddings, biases or concat_bias), one TF Adagrad step on every variable.
    acc: dict of accumulators keyed E, w, W0.., b0.., Wp, bp (updated copies
    are returned).  Returns (loss, E, w, layers, biases, Wp, bp, acc)."""
    X = np.asarray(X, np.int64)
    y = np.asarray(y, F32).reshape(-1)
    E = np.asarray(E, F32)
    w = np.asarray(w, F32).reshape(-1)
    layers = [np.asarray(W, F32) for W in layers]
    biases = [np.asarray(b, F32).reshape(-1) for b in biases]
    Wp = np.asarray(Wp, F32).reshape(-1)
    B, F = X.shape
    k = E.shape[1]
    e = E[X]                                                          # :104
    y1 = w[X]                                                         # :109-110
    s = e.sum(1, dtype=F32)
    y2 = F32(0.5) * (s * s - (e * e).sum(1, dtype=F32))               # :114-122
    hs = [e.reshape(B, F * k)]
    for W, b in zip(layers, biases):                                  # :125-128
        hs.append(np.maximum(np.matmul(hs[-1], W).astype(F32) + b, 0).astype(F32))
    cat = np.concatenate([y1, y2, hs[-1]], axis=1)                    # :132
    out = np.matmul(cat, Wp).astype(F32) + F32(bp)                    # :137
    r = y - out
    reg = np.sum(Wp.astype(np.float64) ** 2) + sum(np.sum(W.astype(np.float64) ** 2)
                                                     for W in layers)
    loss = F32(np.sum(r.astype(np.float64) ** 2) / 2 + lam * reg / 2)  # :143, :146-152
    g = -r                                                            # d loss / d out
    dWp = np.matmul(cat.T, g).astype(F32) + F32(lam) * Wp
    dbp = F32(g.sum(dtype=np.float64))
    dcat = g[:, None] * Wp[None, :]
    dh = dcat[:, F + k:]
    dWs, dbs = [None] * len(layers), [None] * len(layers)
    for i in range(len(layers) - 1, -1, -1):
        dz = (dh * (hs[i + 1] > 0)).astype(F32)                       # relu'
        dWs[i] = np.matmul(hs[i].T, dz).astype(F32) + F32(lam) * layers[i]
        dbs[i] = dz.sum(0, dtype=F32)
        dh = np.matmul(dz, layers[i].T).astype(F32)
    de = dh.reshape(B, F, k) + dcat[:, None, F:F + k] * (s[:, None, :] - e)
    dE = np.zeros_like(E)
    dw = np.zeros_like(w)
    for f in range(F):
        np.add.at(dE, X[:, f], de[:, f])
        np.add.at(dw, X[:, f], dcat[:, f])
    acc = {key: np.asarray(v, F32).copy() for key, v in acc.items()}

    def upd(var, grad, key, rows=None):
        var, acc[key] = tf_apply(optimizer, var, grad, acc.get(key), lr, step, rows)
        return var

    E = upd(E, dE, "E", X)
    w = upd(w, dw, "w", X)
    layers = [upd(W, dW, f"W{i}") for i, (W, dW) in enumerate(zip(layers, dWs))]
    biases = [upd(b, db, f"b{i}") for i, (b, db) in enumerate(zip(biases, dbs))]
    Wp = upd(Wp, dWp, "Wp")
    bp = upd(np.float32(bp), dbp, "bp")
    return loss, E, w, layers, biases, Wp, F32(bp), acc


def afm_train_step(X, y, E, w, w0, W, b, pvec, P, acc, lr, lam, optimizer="adagrad", step=1):
    """AFM partial_fit (AFM.py:144-156, 205-207), attention=1, keep=[1,1]:
    loss = l2_loss(y − out) + l2_regularizer(λ)(attention_W) = Σ(y−out)²/2
    + λ·ΣW²/2, one TF step on every variable (feature_embeddings,
    feature_bias, bias, attention_W/b/p, prediction).  Softmax backward
    dlogit = a ⊙ (da − Σ a·da); relu' where z = pW + b > 0 (TF ReluGrad).
    acc: dict of accumulators keyed E, w, w0, W, b, p, P.
    Returns (loss, E, w, w0, W, b, pvec, P, acc)."""
    X = np.asarray(X, np.int64)
    y = np.asarray(y, F32).reshape(-1)
    E = np.asarray(E, F32)
    w = np.asarray(w, F32).reshape(-1)
    W = np.asarray(W, F32)
    b = np.asarray(b, F32).reshape(-1)
    pvec = np.asarray(pvec, F32).reshape(-1)
    P = np.asarray(P, F32).reshape(-1)
    B, F = X.shape
    k, A = W.shape
    e = E[X]                                                          # :104
    pr = _pairs(e)                                                    # :107-112 [B,np,k]
    z = (np.matmul(pr.reshape(-1, k), W).astype(F32) + b).reshape(B, -1, A)   # :117
    r = np.maximum(z, 0)
    logit = (pvec * r).sum(-1, dtype=F32)                             # :121-124 [B,np]
    ex = np.exp(logit - logit.max(1, keepdims=True))
    att = (ex / ex.sum(1, keepdims=True)).astype(F32)                 # :125
    afm = (att[:, :, None] * pr).sum(1, dtype=F32)                    # :130 [B,k]
    out = np.matmul(afm, P).astype(F32) + w[X].sum(1, dtype=F32) + F32(w0)   # :138-142
    res = y - out
    loss = F32(np.sum(res.astype(np.float64) ** 2) / 2
               + lam * np.sum(W.astype(np.float64) ** 2) / 2)        # :146-149
    g = -res                                                          # d loss / d out
    dP = np.matmul(afm.T, g).astype(F32)
    dw0 = F32(g.sum(dtype=np.float64))
    s = np.matmul(pr, P).astype(F32)                                  # [B,np] = pr·P
    da = g[:, None] * s
    dlogit = att * (da - (att * da).sum(1, keepdims=True))
    dpvec = (dlogit[:, :, None] * r).sum((0, 1), dtype=F32)
    dz = (dlogit[:, :, None] * pvec * (z > 0)).astype(F32)            # [B,np,A]
    db = dz.sum((0, 1), dtype=F32)
    dW = np.matmul(pr.reshape(-1, k).T, dz.reshape(-1, A)).astype(F32) + F32(lam) * W
    dpr = att[:, :, None] * (g[:, None] * P[None, :])[:, None, :] + np.matmul(dz, W.T).astype(F32)
    de = np.zeros_like(e)
    p = 0
    for i in range(F):
        for j in range(i + 1, F):
            de[:, i] += dpr[:, p] * e[:, j]
            de[:, j] += dpr[:, p] * e[:, i]
            p += 1
    dE = np.zeros_like(E)
    dw = np.zeros_like(w)
    for f in range(F):
        np.add.at(dE, X[:, f], de[:, f])
        np.add.at(dw, X[:, f], g)
    acc = {key: np.asarray(v, F32).copy() for key, v in acc.items()}

    def upd(var, grad, key, rows=None):
        var, acc[key] = tf_apply(optimizer, var, grad, acc.get(key), lr, step, rows)
        return var

    return (loss, upd(E, dE, "E", X), upd(w, dw, "w", X), F32(upd(np.float32(w0), dw0, "w0")),
            upd(W, dW, "W"), upd(b, db, "b"), upd(pvec, dpvec, "p"), upd(P, dP, "P"), acc)
