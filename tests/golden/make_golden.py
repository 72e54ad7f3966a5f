#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ from the REFERENCE ITSELF.

Runs only in the builder container, where /root/reference exists (never on
the GPU box; the committed outputs are the fixtures).  It imports the
reference's unmodified modules — Newcode/NewLoadData.py, FM.py,
OurModel7.py, AFM.py, DFM.py — with:
  * ``tensorflow`` = tests/golden/tf1_numpy.py (numpy restatement of the
    TF-1.x ops those modules call; TF is not installed),
  * ``toolz.partition_all`` = a 3-line chunker (toolz is not installed),
  * ``np.int = int`` (removed in numpy >= 1.24, used by the reference),
and PYTHONDONTWRITEBYTECODE so nothing is written into the read-only tree.

Outputs (all synthetic, seeded — no Frappe rows are committed, since the
Frappe README forbids redistribution):
  synth_frappe.libfm / synth_jiaju.libfm   synthetic libfm inputs
  loaddata_*.npz        LoadData outputs for np.random.seed(2016)
  fm.npz hhfm_*.npz afm.npz dfm.npz        model-graph outputs (out / topk)
  losses.npz            each model's `self.loss` at seeded weights + batch
  harness.npz + harness.json               sample_negative / evaluate_TopK /
                                           evaluate_AUC outputs
  epoch_stream.json     the batches the reference's own Train.train feeds
                        partial_fit (FM and OurModel7, 2 epochs on
                        synth_frappe, seeded): per-batch sha256 of X/Y/F1
Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import types

sys.dont_write_bytecode = True
import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, HERE)
import tf1_numpy  # noqa: E402

tf1_numpy.install(sys.modules)
_toolz = types.ModuleType("toolz")
_toolz.partition_all = lambda n, seq: [list(seq)[i:i + n] for i in range(0, len(list(seq)), n)]
sys.modules["toolz"] = _toolz
np.int = int  # the reference uses np.int (removed in numpy 1.24)
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(REF, "Newcode"))

import Newcode.NewLoadData as NLD  # noqa: E402
import Newcode.FM as RFM  # noqa: E402
import Newcode.OurModel7 as RM7  # noqa: E402
import Newcode.AFM as RAFM  # noqa: E402
import Newcode.DFM as RDFM  # noqa: E402


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print("wrote", name, {k: getattr(v, "shape", v) for k, v in arrays.items()})


# ---------------------------------------------------------------------------
# synthetic libfm inputs (Frappe-like tokens; identical tokens across columns
# exercise quirk 1: one shared id, NewLoadData.py:29-34)
# ---------------------------------------------------------------------------
def write_synth_frappe(path, rows=7000, seed=5):
    rng = np.random.default_rng(seed)
    day = ["morning", "afternoon", "evening", "night", "sunrise", "sunset", "noon"]
    wk = ["weekend", "workday"]
    hw = ["home", "work", "unknown"]
    lines = []
    for _ in range(rows):
        u = int(rng.zipf(1.6)) % 120
        it = int(rng.zipf(1.3)) % 400
        item_tok = f"i{it}" if it % 37 else f"u{it % 120}"     # some items share a user token
        d = day[rng.integers(0, 7)]
        w = wk[rng.integers(0, 2)]
        h = hw[rng.integers(0, 3)] if rng.random() > 0.02 else "night"  # shared with daytime
        lines.append(f"1 u{u} {item_tok} {d} {w} {h}")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def write_synth_jiaju(path, rows=1500, seed=6):
    """jiaju-like layout: label user item ctx x5 time x3 (OurModel7.py:342-346)."""
    rng = np.random.default_rng(seed)
    lines = []
    for _ in range(rows):
        u = rng.integers(0, 40)
        it = rng.integers(0, 150)
        ctx = [f"TM{rng.integers(0, 25):03d}" for _ in range(5)]
        tim = [f"timeD{rng.integers(0, 150):03d}" for _ in range(3)]
        lines.append(" ".join(["1", f"{u:03d}.txt", f"I{it:03d}"] + ctx + tim))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def loaddata_fixture(dataset, tag):
    np.random.seed(2016)
    d = NLD.LoadData(HERE + "/", dataset)
    keys = sorted(d.positive_feedback.keys())
    pf_keys, pf_items = [], []
    for kk in keys:
        for it in sorted(d.positive_feedback[kk]):
            pf_keys.append(kk)
            pf_items.append(it)
    save(f"loaddata_{tag}.npz", train=d.Train_data.values.astype(np.int64),
         test=d.Test_data.values.astype(np.int64), n_user=d.n_user, n_item=d.n_item,
         features_M=d.features_M, columns=np.array(list(d.Train_data.columns)),
         pf_keys=np.array(pf_keys, dtype=np.int64), pf_items=np.array(pf_items, dtype=np.int64))
    return d


# ---------------------------------------------------------------------------
# model graphs
# ---------------------------------------------------------------------------
def vocab(n_user, n_item, ctx):
    return n_user + n_item + sum(ctx)


def rows(rng, B, n_user, n_item, ctx, ntime=0):
    cols = [rng.integers(0, n_user, B), rng.integers(n_user, n_user + n_item, B)]
    o = n_user + n_item
    for c in ctx:
        cols.append(rng.integers(o, o + c, B))
        o += c
    for _ in range(ntime):
        cols.append(rng.integers(n_user, n_user + n_item, B))
    return np.stack(cols, 1).astype(np.int32)


def gen_fm():
    rng = np.random.default_rng(101)
    nu, ni, ctx, k = 957, 4082, (7, 2, 3), 32
    M = vocab(nu, ni, ctx)
    m = RFM.FM(5, M, nu, ni, k, 0.1, 0.1, 1, "AdagradOptimizer", 0, 0)
    E = rng.normal(0, 0.01, (M, k)).astype(np.float32)
    w = rng.normal(0, 0.01, (M, 1)).astype(np.float32)
    w0 = np.float32(0.01)
    m.weights["feature_embeddings"].value = E
    m.weights["feature_bias"].value = w
    m.weights["bias"].value = w0
    X = rows(rng, 256, nu, ni, ctx)
    out = m.sess.run(m.out, feed_dict={m.train_features: X, m.train_labels: np.ones((256, 1)),
                                       m.dropout_keep: 1.0, m.train_phase: False})
    A = rows(rng, 24, nu, ni, ctx)
    tf1_numpy.LAST_TOPK_INPUT.clear()
    pred = m.topk(A, 20)
    save("fm.npz", E=E, w=w[:, 0], w0=w0, n_user=nu, n_item=ni, X=X, out=out[:, 0], A=A,
         topk_idx=pred, topk_scores=tf1_numpy.LAST_TOPK_INPUT[-1])


def gen_hhfm(tag, nu, ni, ctx, td, k, seed):
    rng = np.random.default_rng(seed)
    M = vocab(nu, ni, ctx)
    fd = len(ctx)
    m = RM7.OUR(fd, td, M, nu, ni, k, 0.1, 0.01, "AdagradOptimizer", True, td > 0)
    E = rng.normal(0, 0.01, (M, k)).astype(np.float32)
    m.weights["feature_embeddings"].value = E
    X = rows(rng, 256, nu, ni, ctx, td)
    feed = {m.Pos: X[:, :2], m.Fea: X[:, 2:2 + fd]}
    if td:
        feed[m.Tim] = X[:, 2 + fd:]
    out = m.sess.run(m.PositiveFeadback, feed_dict=feed)
    A = rows(rng, 24, nu, ni, ctx, td)
    tf1_numpy.LAST_TOPK_INPUT.clear()
    pred = m.topk(A, 20)
    save(f"hhfm_{tag}.npz", E=E, n_user=nu, n_item=ni, feature_dimension=fd,
         time_dimension=td, X=X, out=out[:, 0], A=A, topk_idx=pred,
         topk_scores=tf1_numpy.LAST_TOPK_INPUT[-1])


def gen_afm():
    rng = np.random.default_rng(303)
    np.random.seed(303)  # AFM draws attention weights from np.random (AFM.py:190-196)
    nu, ni, ctx, k = 100, 400, (7, 2, 3), 16
    M = vocab(nu, ni, ctx)
    m = RAFM.AFM(nu, ni, M, 1, [k, k], None, 0.1, 100.0, [1, 1], "AdagradOptimizer", 0.999, 5)
    E = rng.normal(0, 0.01, (M, k)).astype(np.float32)
    w = rng.normal(0, 0.01, (M, 1)).astype(np.float32)
    m.weights["feature_embeddings"].value = E
    m.weights["feature_bias"].value = w
    m.weights["bias"].value = np.float32(0.02)
    X = rows(rng, 128, nu, ni, ctx)
    out = m.sess.run(m.out, feed_dict={m.train_features: X, m.train_labels: np.ones((128, 1)),
                                       m.dropout_keep: [1.0, 1.0], m.train_phase: False})
    A = rows(rng, 12, nu, ni, ctx)
    tf1_numpy.LAST_TOPK_INPUT.clear()
    pred = m.topk(A, 20)
    W = m.weights
    save("afm.npz", E=E, w=w[:, 0], w0=np.float32(0.02), n_user=nu, n_item=ni,
         attention_W=W["attention_W"].value, attention_b=W["attention_b"].value,
         attention_p=W["attention_p"].value, prediction=W["prediction"].value,
         X=X, out=out[:, 0], A=A, topk_idx=pred, topk_scores=tf1_numpy.LAST_TOPK_INPUT[-1])


def gen_dfm():
    rng = np.random.default_rng(404)
    np.random.seed(404)  # DeepFM draws layer weights from np.random (DFM.py:185-208)
    nu, ni, ctx, k = 50, 300, (7, 2, 3), 16
    M = vocab(nu, ni, ctx)
    m = RDFM.DeepFM(nu, ni, M, 5, k, [150, 200, 150], tf1_numpy.nn.relu, 0.01, 0, 0.01)
    E = rng.normal(0, 0.01, (M, k)).astype(np.float32)
    w = rng.uniform(0, 1, (M, 1)).astype(np.float32)   # DFM.py:178-179 init U(0,1)
    m.weights["feature_embeddings"].value = E
    m.weights["feature_bias"].value = w
    X = rows(rng, 128, nu, ni, ctx)
    out = m.sess.run(m.out, feed_dict={m.feat_index: X, m.label: np.ones((128, 1))})
    A = rows(rng, 8, nu, ni, ctx)
    tf1_numpy.LAST_TOPK_INPUT.clear()
    pred = m.topk(A, 20)
    W = m.weights
    arrs = {f"layer_{i}": W[f"layer_{i}"].value for i in range(3)}
    arrs.update({f"bias_{i}": W[f"bias_{i}"].value for i in range(3)})
    save("dfm.npz", E=E, w=w[:, 0], n_user=nu, n_item=ni, X=X, out=out[:, 0], A=A,
         topk_idx=pred, topk_scores=tf1_numpy.LAST_TOPK_INPUT[-1],
         concat_projection=W["concat_projection"].value,
         concat_bias=np.float32(W["concat_bias"].value), **arrs)


# ---------------------------------------------------------------------------
# training objectives: each reference model's own `self.loss` graph
# (FM.py:123-126, OurModel7.py:172-184, AFM.py:144-148, DFM.py:139-152)
# evaluated at seeded weights on a seeded batch with negatives
# ---------------------------------------------------------------------------
def gen_losses():
    out = {}
    nu, ni, ctx = 40, 150, (7, 2, 3)
    M = vocab(nu, ni, ctx)

    # FM: MSE on positives (label 1) + sampled negatives (label 0, FM.py:248)
    rng = np.random.default_rng(701)
    k = 16
    m = RFM.FM(5, M, nu, ni, k, 0.1, 0.1, 1, "AdagradOptimizer", 0, 0)
    E = rng.normal(0, 0.01, (M, k)).astype(np.float32)
    w = rng.normal(0, 0.01, (M, 1)).astype(np.float32)
    m.weights["feature_embeddings"].value = E
    m.weights["feature_bias"].value = w
    m.weights["bias"].value = np.float32(0.03)
    X = rows(rng, 96, nu, ni, ctx)
    Y = np.concatenate([np.ones(48), np.zeros(48)]).reshape(-1, 1).astype(np.float32)
    loss = m.sess.run(m.loss, feed_dict={m.train_features: X, m.train_labels: Y,
                                         m.dropout_keep: 1.0, m.train_phase: True})
    out.update(fm_E=E, fm_w=w[:, 0], fm_w0=np.float32(0.03), fm_X=X, fm_Y=Y[:, 0],
               fm_lamda=np.float32(0.1), fm_loss=np.float32(loss))

    # HHFM (frappe layout): −Σ log σ(s⁺ − max_neg s⁻) + λ‖E‖²/2
    rng = np.random.default_rng(702)
    m = RM7.OUR(3, 0, M, nu, ni, k, 0.1, 0.01, "AdagradOptimizer", True, False)
    E = rng.normal(0, 0.3, (M, k)).astype(np.float32)   # wide: the sigmoid is not saturated at 0.5
    m.weights["feature_embeddings"].value = E
    X = rows(rng, 80, nu, ni, ctx)
    Neg = rng.integers(nu, nu + ni, (80, 10)).astype(np.int32)
    Neg[3, 4] = Neg[3, 7]                                   # a tie in reduce_max
    loss = m.sess.run(m.loss, feed_dict={m.Pos: X[:, :2], m.Fea: X[:, 2:], m.Neg: Neg})
    out.update(hhfm_E=E, hhfm_X=X, hhfm_Neg=Neg, hhfm_lamda=np.float32(0.01),
               hhfm_loss=np.float32(loss))

    # AFM: MSE with labels {1, -1} (AFM.py:317) + λ‖attention_W‖²/2
    rng = np.random.default_rng(703)
    np.random.seed(703)
    ka = 16
    m = RAFM.AFM(nu, ni, M, 1, [ka, ka], None, 0.1, 2.0, [1, 1], "AdagradOptimizer", 0.999, 5)
    E = rng.normal(0, 0.1, (M, ka)).astype(np.float32)
    w = rng.normal(0, 0.01, (M, 1)).astype(np.float32)
    m.weights["feature_embeddings"].value = E
    m.weights["feature_bias"].value = w
    m.weights["bias"].value = np.float32(0.02)
    X = rows(rng, 64, nu, ni, ctx)
    Y = np.concatenate([np.ones(32), -np.ones(32)]).reshape(-1, 1).astype(np.float32)
    loss = m.sess.run(m.loss, feed_dict={m.train_features: X, m.train_labels: Y,
                                         m.dropout_keep: [1.0, 1.0], m.train_phase: True})
    W = m.weights
    out.update(afm_E=E, afm_w=w[:, 0], afm_w0=np.float32(0.02), afm_X=X, afm_Y=Y[:, 0],
               afm_lamda=np.float32(2.0), afm_attention_W=W["attention_W"].value,
               afm_attention_b=W["attention_b"].value, afm_attention_p=W["attention_p"].value,
               afm_prediction=W["prediction"].value, afm_loss=np.float32(loss))

    # DeepFM: MSE with labels {1, -1} (DFM.py:286) + l2_reg on projection + layers
    rng = np.random.default_rng(704)
    np.random.seed(704)
    m = RDFM.DeepFM(nu, ni, M, 5, k, [32, 24], tf1_numpy.nn.relu, 0.01, 0, 0.05)
    E = rng.normal(0, 0.05, (M, k)).astype(np.float32)
    w = rng.uniform(0, 1, (M, 1)).astype(np.float32)
    m.weights["feature_embeddings"].value = E
    m.weights["feature_bias"].value = w
    X = rows(rng, 64, nu, ni, ctx)
    Y = np.concatenate([np.ones(32), -np.ones(32)]).reshape(-1, 1).astype(np.float32)
    loss = m.sess.run(m.loss, feed_dict={m.feat_index: X, m.label: Y})
    W = m.weights
    out.update(dfm_E=E, dfm_w=w[:, 0], dfm_X=X, dfm_Y=Y[:, 0], dfm_l2=np.float32(0.05),
               dfm_concat_projection=W["concat_projection"].value,
               dfm_concat_bias=np.float32(W["concat_bias"].value),
               **{f"dfm_layer_{i}": W[f"layer_{i}"].value for i in range(2)},
               **{f"dfm_bias_{i}": W[f"bias_{i}"].value for i in range(2)},
               dfm_loss=np.float32(loss))
    out.update(n_user=nu, n_item=ni)
    save("losses.npz", **out)
    print("losses", {kk: float(v) for kk, v in out.items() if kk.endswith("_loss")})


# ---------------------------------------------------------------------------
# harness (Train.* methods, unmodified, with a stand-in model)
# ---------------------------------------------------------------------------
class _OracleModel:
    """Stand-in for the TF model: FM.out / PositiveFeadback / topk computed by
    the numpy oracle with a fixed table (only the harness logic is under test)."""

    def __init__(self, E, w, n_user, n_item, fd):
        sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
        from oracle import fm_oracle
        self.o, self.E, self.w, self.nu, self.ni, self.fd = fm_oracle, E, w, n_user, n_item, fd
        self.train_features, self.train_labels = object(), object()
        self.dropout_keep, self.train_phase = object(), object()
        self.Pos, self.Fea = object(), object()
        self.out, self.PositiveFeadback = object(), object()
        model = self

        class _Sess:
            def run(self, fetch, feed_dict):
                if fetch is model.out:
                    return model.o.fm_out(feed_dict[model.train_features], model.E, model.w)
                X = np.concatenate([feed_dict[model.Pos], feed_dict[model.Fea]], axis=1)
                return model.o.hhfm_positive_feedback(X, model.E, model.fd, 0)
        self.sess = _Sess()

    def topk(self, A, tp):
        return self.o.hhfm_topk(A, self.E, self.nu, self.ni, self.fd, 0, tp=tp)[1]


class _PlantedModel(_OracleModel):
    """topk puts the row's target item at rank (7u + c1) % 24 (absent when
    >= 20) among filler items, so the metric walk hits every branch: hits at
    each rank, misses, and the target-in-positive_feedback skip (FM.py:354)."""

    def topk(self, A, tp):
        return planted_topk(np.asarray(A), self.nu, self.ni, tp)


def planted_topk(A, n_user, n_item, tp):
    out = np.empty((A.shape[0], tp), dtype=np.int32)
    for r, line in enumerate(A):
        tgt = int(line[1]) - n_user
        fill = [(tgt + 1 + 3 * j) % n_item for j in range(tp)]
        pos = (7 * int(line[0]) + int(line[2])) % 24
        if pos < tp:
            fill[pos] = tgt
        out[r] = fill
    return out


def gen_harness(d):
    rng = np.random.default_rng(505)
    E = rng.normal(0, 0.1, (d.features_M, 16)).astype(np.float32)
    w = rng.normal(0, 0.1, d.features_M).astype(np.float32)
    model = _OracleModel(E, w, d.n_user, d.n_item, 3)
    res = {}
    arr = {"E": E, "w": w}

    def trainer(mod, topk=10):
        t = object.__new__(mod.Train)
        t.data, t.n_user, t.n_item, t.TopK, t.model = d, d.n_user, d.n_item, topk, model
        t.context, t.time, t.time_dimension = True, False, 0
        return t

    t = trainer(RFM)
    np.random.seed(7)
    arr["neg_in"] = d.Train_data.values[:300, 1:].astype(np.int64)
    arr["neg_out"] = t.sample_negative(arr["neg_in"], 10)
    for topk in (5, 10):
        np.random.seed(11)
        res[f"fm_topk{topk}"] = [float(x) for x in trainer(RFM, topk).evaluate_TopK(d.Test_data)]
        np.random.seed(11)
        res[f"dfm_topk{topk}"] = [float(x) for x in trainer(RDFM, topk).evaluate_TopK(d.Test_data)]
    planted = _PlantedModel(E, w, d.n_user, d.n_item, 3)
    for topk in (1, 5, 10, 20):
        t = trainer(RFM, topk)
        t.model = planted
        np.random.seed(23)
        res[f"planted_fm_topk{topk}"] = [float(x) for x in t.evaluate_TopK(d.Test_data)]
        t = trainer(RDFM, topk)
        t.model = planted
        np.random.seed(29)
        res[f"planted_dfm_topk{topk}"] = [float(x) for x in t.evaluate_TopK(d.Test_data)]
    np.random.seed(13)
    res["fm_auc_test"] = float(trainer(RFM).evaluate_AUC(d.Test_data))
    np.random.seed(17)
    res["hhfm_auc_train"] = float(trainer(RM7).evaluate_AUC(d.Train_data))
    np.random.seed(19)
    res["fm_auc_train"] = float(trainer(RFM).evaluate_AUC(d.Train_data))
    save("harness.npz", **arr)
    with open(os.path.join(HERE, "harness.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("harness", res)


class _Recorder:
    """Stand-in model whose partial_fit records each batch it is fed (the
    epoch loop, not the model, is under test) and returns a fixed loss."""

    def __init__(self):
        self.batches = []

    def partial_fit(self, data):
        import hashlib
        h = hashlib.sha256()
        for key in sorted(data):
            a = np.ascontiguousarray(np.asarray(data[key], dtype=np.float64))
            h.update(key.encode())
            h.update(np.asarray(a.shape, np.int64).tobytes())
            h.update(a.tobytes())
        self.batches.append(h.hexdigest())
        return 1.0


def epoch_stream_case(mod, seed, epochs=2, batch=512):
    """The reference's Train.train (FM.py:221-282 / OurModel7.py:349-413),
    unmodified, with Result = 1 (no evaluation before epoch 30 / 20) and a
    recording model, on a fresh seeded LoadData of synth_frappe."""
    import argparse
    np.random.seed(2016)
    d = NLD.LoadData(os.path.join(HERE) + "/", "synth_frappe")
    t = object.__new__(mod.Train)
    t.args = argparse.Namespace(Result=1, dataset="synth_frappe", verbose=0)
    t.data, t.n_user, t.n_item = d, d.n_user, d.n_item
    t.epoch, t.batch_size, t.verbose, t.TopK = epochs + 1, batch, 0, 10
    t.context, t.time, t.time_dimension = True, False, 0
    t.model = _Recorder()
    np.random.seed(seed)
    t.train()
    return t.model.batches


def gen_epoch_stream():
    res = {"fm": epoch_stream_case(RFM, 41), "hhfm": epoch_stream_case(RM7, 43),
           "epochs": 2, "batch_size": 512, "seeds": {"fm": 41, "hhfm": 43},
           "loaddata_seed": 2016}
    with open(os.path.join(HERE, "epoch_stream.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("epoch_stream", {k: len(v) for k, v in res.items() if isinstance(v, list)})


def gen_frappe_real():
    """Real Frappe (builder container only): commit only derived numbers —
    split hashes and the reference harness's HR/NDCG/PRE@10 for a seeded
    random-weight HHFM scored by the oracle (no rows are redistributed)."""
    import hashlib
    path = os.path.join(REF, "data", "positive") + "/"
    if not os.path.exists(path + "frappe/frappe.libfm"):
        return
    np.random.seed(2016)
    d = NLD.LoadData(path, "frappe")
    res = {"sizes": [d.n_user, d.n_item, d.features_M],
           "train_sha256": hashlib.sha256(np.ascontiguousarray(d.Train_data.values, np.int64)).hexdigest(),
           "test_sha256": hashlib.sha256(np.ascontiguousarray(d.Test_data.values, np.int64)).hexdigest()}
    E = np.random.default_rng(606).normal(0, 0.01, (d.features_M, 64)).astype(np.float32)
    model = _OracleModel(E, None, d.n_user, d.n_item, 3)
    for topk in (5, 10):
        t = object.__new__(RM7.Train)
        t.data, t.n_user, t.n_item, t.TopK, t.model = d, d.n_user, d.n_item, topk, model
        np.random.seed(31)
        res[f"hhfm_random_w_topk{topk}"] = [float(x) for x in t.evaluate_TopK(d.Test_data)]
    with open(os.path.join(HERE, "frappe_real.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("frappe_real", res)


def main():
    os.makedirs(os.path.join(HERE, "synth_frappe"), exist_ok=True)
    os.makedirs(os.path.join(HERE, "synth_jiaju"), exist_ok=True)
    write_synth_frappe(os.path.join(HERE, "synth_frappe", "synth_frappe.libfm"))
    write_synth_jiaju(os.path.join(HERE, "synth_jiaju", "synth_jiaju.libfm"))
    d = loaddata_fixture("synth_frappe", "frappe")
    loaddata_fixture("synth_jiaju", "jiaju")
    gen_fm()
    gen_hhfm("frappe", 957, 4082, (7, 2, 3), 0, 32, 201)
    gen_hhfm("jiaju", 200, 600, (5, 4, 6, 3, 7), 3, 16, 202)
    gen_hhfm("resturant", 200, 600, (5, 4, 6, 3, 7), 5, 16, 203)
    gen_afm()
    gen_dfm()
    gen_losses()
    gen_harness(d)
    gen_epoch_stream()
    gen_frappe_real()


if __name__ == "__main__":
    main()
