"""H6 on the GPU: partial_fit steps vs the oracle's TF-semantics step
(hand-derived gradients pinned by finite differences in
tests/test_oracle_training.py), and the reference epoch loops end to end.
Gradients are summed with float atomics, so updates agree to ~1e-6
relative, not bitwise."""
import argparse
import os

import numpy as np
import pytest
import torch

from oracle import fm_oracle as orc

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _rows(rng, B, nu, ni, ctx, td=0):
    cols = [rng.integers(0, nu, B), rng.integers(nu, nu + ni, B)]
    o = nu + ni
    for c in ctx:
        cols.append(rng.integers(o, o + c, B))
        o += c
    for _ in range(td):
        cols.append(rng.integers(nu, nu + ni, B))
    return np.stack(cols, 1).astype(np.int64), o


def _close_update(got, ref, before):
    """Updated parameters agree to 1e-4 of the largest update (atomic
    summation order) and 1e-5 relative."""
    step = np.abs(ref - before).max()
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-4 * step + 1e-9)


OPTS = {"AdagradOptimizer": "adagrad", "GradientDescentOptimizer": "sgd",
        "MomentumOptimizer": "momentum", "AdamOptimizer": "adam"}


def _slot(o, v):
    """The oracle's initial slot for variable v (TF: Adagrad 0.1, Momentum 0,
    Adam m = v = 0 stacked flat)."""
    v = np.asarray(v, np.float32)
    return {"adagrad": np.full_like(v, 0.1), "momentum": np.zeros_like(v),
            "adam": np.zeros(2 * v.size, np.float32), "sgd": None}[o]


def _check_var(got, ref, before, o, grad):
    """_close_update, except under Adam: its early steps move an element by
    ≈ ±α whatever |g| is, so its update error is ≈ 3·α_t·δg/|g| for a
    gradient error δg (d(m̂/√v̂)/dg ≈ (1−β1)/√v̂, √v̂ ≥ √(1−β2)·|g|).  The
    float atomics' summation order gives δg up to ~1e-6 of the table row's
    largest |g| (a row's k elements sum over the same rows), so table
    elements with |g| ≥ 1e-2 of that are held to 1e-4 of the largest step (a
    1e-4 cut-off failed once among round 6's GPU runs); a vector's elements
    sum over different rows each (noise ∝ the element's own terms), so there
    the cut-off stays 1e-4 of the largest |g|.  The rest (~2 %) only to ≤ 2 ×
    the largest step."""
    got, ref, before = (np.asarray(x, np.float32) for x in (got, ref, before))
    if o != "adam":
        _close_update(got, ref, before)
        return
    g = np.abs(np.asarray(grad, np.float32).reshape(ref.shape))
    scale = g.max(axis=-1, keepdims=True) if g.ndim == 2 else g.max(initial=0.0)
    well = g >= (1e-2 if g.ndim == 2 else 1e-4) * scale
    step = np.abs(ref - before).max()
    off = well & ~np.isclose(got, ref, rtol=1e-5, atol=1e-4 * step + 1e-9)
    gs = g / np.maximum(scale, 1e-30)
    assert not off.any(), (f"{off.sum()} elements: |g|/row max {gs[off][:8]}, "
                           f"|got-ref| {np.abs(got - ref)[off][:8]}, step {step}")
    assert np.all(np.abs(got - ref) <= 2.01 * step + 1e-9)
    assert (well & (g > 0)).sum() >= 0.9 * (g > 0).sum()


def _check_slot(got, ref, o):
    if o == "sgd":
        return
    ref = np.asarray(ref, np.float32).reshape(-1)
    got = np.asarray(got, np.float32).reshape(-1)
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max() + 1e-12)


def _slots_of(m, names, o, cur):
    st = getattr(m, "_train_state", None)
    if st is None:
        return [_slot(o, v) for v in cur]
    return [None if o == "sgd" else st[n].cpu().numpy() for n in names]


FM_CASES = [("AdagradOptimizer", 0.1), ("GradientDescentOptimizer", 0.1),
            ("AdagradOptimizer", 0.0), ("MomentumOptimizer", 0.1), ("MomentumOptimizer", 0.0),
            ("AdamOptimizer", 0.1), ("AdamOptimizer", 0.0)]


@pytest.mark.parametrize("opt,lam", FM_CASES)
def test_fm_partial_fit_matches_oracle(opt, lam):
    """FM partial_fit (FM.py:123-136, 168-171) under each --optimizer, with
    the l2 term (E's gradient dense) and without it (E an IndexedSlices: the
    sparse Momentum / Adam rules).  Each step is replayed by the oracle from
    the GPU's own pre-step parameters and slots; Adam's β powers are the
    GPU's to carry (3 steps)."""
    from hhfm_amd.FM import FM
    rng = np.random.default_rng(0)
    nu, ni, k = 200, 500, 32
    X, M = _rows(rng, 5000, nu, ni, (7, 2, 3))
    m = FM(5, M, nu, ni, k, 0.1, lam, 1, opt, 0, 0)
    E = rng.normal(0, 0.01, (M, k)).astype(np.float32)
    w = rng.normal(0, 0.01, M).astype(np.float32)
    m.set_weights(feature_embeddings=E, feature_bias=w[:, None], bias=np.float32(0.02))
    o = OPTS[opt]
    names = ["feature_embeddings", "feature_bias", "bias"]
    for step in range(3):
        Wg = m.get_weights()
        cur = [Wg["feature_embeddings"], Wg["feature_bias"][:, 0], np.float32(Wg["bias"])]
        sl = _slots_of(m, names, o, cur)
        Xb = X[step * 1500:(step + 1) * 1500]
        y = rng.integers(0, 2, len(Xb)).astype(np.float32)[:, None]
        loss = m.partial_fit({"X": Xb, "Y": y})
        rl, E1, w1, w01, aE, aw, a0 = orc.fm_train_step(Xb, y, *cur, *sl, 0.1, lam, o, step + 1)
        _, Eg, wg, w0g, *_ = orc.fm_train_step(Xb, y, *cur, None, None, None, 1.0, lam, "sgd")
        assert np.isclose(loss, rl, rtol=1e-5)
        Wn = m.get_weights()
        _check_var(Wn["feature_embeddings"], E1, cur[0], o, cur[0] - Eg)
        _check_var(Wn["feature_bias"][:, 0], w1, cur[1], o, cur[1] - wg)
        _check_var(np.float32(Wn["bias"]).reshape(1), np.float32(w01).reshape(1),
                   np.float32(cur[2]).reshape(1), o, np.float32(cur[2] - w0g).reshape(1))
        for n, r in zip(names, (aE, aw, a0)):
            if o != "sgd":
                _check_slot(m._train_state[n].cpu().numpy(), r, o)


def _fm_adam_powers(m):
    """The FM train workspace's Adam scalars [β1^t, β2^t, started]
    (train.hip: scal = dE [M·k] + dw [M] floats in)."""
    M, k = m.weights["feature_embeddings"].shape
    o = M * k + M + 8
    return m._train_state["ws"].view(torch.float32)[o:o + 3]


def test_fm_adam_past_beta1_power_underflow():
    """β1^t = 0.9^t underflows to exactly 0 at t = 829 under TF's
    flush-to-zero and TF keeps using 0 (AdamOptimizer._finish multiplies the
    power each step), so a zero power must not read as "not started" (the
    round-4 kernels restarted the powers there: α jumped ~10×).  860 tiny
    Adam steps: the powers the GPU carries equal adam_powers(t + 1) bit for
    bit at every checked step, and each step from t = 822 on (across the
    underflow) is replayed by the oracle from the GPU's own pre-step
    parameters and slots."""
    from hhfm_amd.FM import FM
    rng = np.random.default_rng(5)
    nu, ni, k = 20, 30, 8
    X, M = _rows(rng, 64 * 860, nu, ni, (7, 2, 3))
    Y = rng.integers(0, 2, len(X)).astype(np.float32)[:, None]
    m = FM(5, M, nu, ni, k, 0.01, 0.1, 1, "AdamOptimizer", 0, 0)
    m.set_weights(feature_embeddings=rng.normal(0, 0.01, (M, k)).astype(np.float32),
                  feature_bias=rng.normal(0, 0.01, (M, 1)).astype(np.float32),
                  bias=np.float32(0.02))
    names = ["feature_embeddings", "feature_bias", "bias"]
    crossed = False
    for t in range(1, 861):
        Xb, yb = X[(t - 1) * 64:t * 64], Y[(t - 1) * 64:t * 64]
        if t < 822:
            m.partial_fit({"X": Xb, "Y": yb})
            if t % 97 == 0:
                b1, b2 = orc.adam_powers(t + 1)
                assert _fm_adam_powers(m).cpu().numpy().tolist() == [b1, b2, 1.0]
            continue
        Wg = m.get_weights()
        cur = [Wg["feature_embeddings"], Wg["feature_bias"][:, 0], np.float32(Wg["bias"])]
        sl = _slots_of(m, names, "adam", cur)
        loss = m.partial_fit({"X": Xb, "Y": yb})
        rl, E1, w1, w01, aE, aw, a0 = orc.fm_train_step(Xb, yb, *cur, *sl, 0.01, 0.1, "adam", t)
        _, Eg, wg, w0g, *_ = orc.fm_train_step(Xb, yb, *cur, None, None, None, 1.0, 0.1, "sgd")
        assert np.isclose(loss, rl, rtol=1e-5)
        Wn = m.get_weights()
        _check_var(Wn["feature_embeddings"], E1, cur[0], "adam", cur[0] - Eg)
        _check_var(Wn["feature_bias"][:, 0], w1, cur[1], "adam", cur[1] - wg)
        b1, b2 = orc.adam_powers(t + 1)
        assert _fm_adam_powers(m).cpu().numpy().tolist() == [b1, b2, 1.0]
        crossed |= b1 == 0.0
    assert crossed


HHFM_CASES = [("frappe", "AdagradOptimizer", 0.01), ("jiaju", "AdagradOptimizer", 0.01),
              ("frappe", "MomentumOptimizer", 0.0), ("jiaju", "MomentumOptimizer", 0.01),
              ("frappe", "AdamOptimizer", 0.0), ("jiaju", "AdamOptimizer", 0.01),
              ("frappe", "GradientDescentOptimizer", 0.0)]


@pytest.mark.parametrize("layout,opt,lam", HHFM_CASES)
def test_hhfm_partial_fit_matches_oracle(layout, opt, lam):
    """OUR partial_fit (OurModel7.py:171-193, 219-228) under each --optimizer;
    λ = 0 leaves the table's gradient an IndexedSlices over X and Neg."""
    from hhfm_amd.OurModel7 import OUR
    rng = np.random.default_rng(1)
    nu, ni, k = 300, 800, 32
    ctx, td = ((7, 2, 3), 0) if layout == "frappe" else ((5, 4, 6, 3, 7), 3)
    X, M = _rows(rng, 4500, nu, ni, ctx, td)
    fd = len(ctx)
    m = OUR(fd, td, M, nu, ni, k, 0.1, lam, opt, True, td > 0)
    m.set_weights(feature_embeddings=rng.normal(0, 0.01, (M, k)).astype(np.float32))
    o = OPTS[opt]
    for step in range(3):
        E = m.get_weights()["feature_embeddings"]
        (accE,) = _slots_of(m, ["feature_embeddings"], o, [E])
        Xb = X[step * 1500:(step + 1) * 1500]
        Neg = rng.integers(nu, nu + ni, (len(Xb), 10))
        data = {"X": Xb[:, :2], "Y": Neg, "F1": Xb[:, 2:2 + fd]}
        if td:
            data["F2"] = Xb[:, 2 + fd:]
        loss = m.partial_fit(data)
        rl, E1, acc1 = orc.hhfm_train_step(Xb, Neg, E, accE, 0.1, lam, fd, td, True, td > 0,
                                           o, step + 1)
        _, Eg, _ = orc.hhfm_train_step(Xb, Neg, E, None, 1.0, lam, fd, td, True, td > 0, "sgd")
        assert np.isclose(loss, rl, rtol=1e-5)
        _check_var(m.get_weights()["feature_embeddings"], E1, E, o, E - Eg)
        if o != "sgd":
            _check_slot(m._train_state["feature_embeddings"].cpu().numpy(), acc1, o)


def _args(tmp_path, **kw):
    a = dict(path=G + "/", dataset="synth_frappe", epoch=3, batch_size=5000, hidden_factor=32,
             lamda=0.1, keep=1, lr=0.1, optimizer="AdagradOptimizer", verbose=1, batch_norm=0,
             TopK=10, Result=0, result_file=str(tmp_path / "result.txt"))
    a.update(kw)
    return argparse.Namespace(**a)


def test_fm_train_loop_end_to_end(tmp_path):
    from hhfm_amd.FM import Train
    np.random.seed(2016)
    t = Train(_args(tmp_path))
    losses = t.train()
    assert len(losses) == 2 and losses[1] < losses[0]
    log = open(tmp_path / "result.txt").read()
    assert "Init" in log and "FM Epoch 1" in log


def test_hhfm_train_loop_end_to_end(tmp_path):
    from hhfm_amd.OurModel7 import Train
    np.random.seed(2016)
    t = Train(_args(tmp_path, lamda=0.01, epoch=11))
    losses = t.train()
    assert len(losses) == 10 and losses[-1] < losses[0]
    assert "M7 Epoch 10" in open(tmp_path / "result.txt").read()


@pytest.mark.parametrize("k,layers,B", [
    (16, [24, 40, 24], 301),        # ragged batch, widths not multiples of 8
    (32, [150, 200, 150], 1000),    # the reference's MLP (DFM.py:256)
    (8, [12], 7),                   # one layer, tiny batch
])
def test_dfm_partial_fit_matches_oracle(k, layers, B):
    """DeepFM partial_fit (DFM.py:139-155): every variable after two Adagrad
    steps vs the oracle's TF-semantics step."""
    from hhfm_amd.DFM import DeepFM
    rng = np.random.default_rng(k + B)
    nu, ni = 60, 200
    X, M = _rows(rng, 2 * B, nu, ni, (7, 2, 3))
    m = DeepFM(nu, ni, M, 5, k, layers, None, 0.01, 0, 0.01)
    W = m.get_weights()
    L = len(layers)
    E, w = W["feature_embeddings"], W["feature_bias"][:, 0]
    Ls = [W[f"layer_{i}"] for i in range(L)]
    bs = [W[f"bias_{i}"][0] for i in range(L)]
    Wp, bp = W["concat_projection"][:, 0], np.float32(W["concat_bias"])
    keys = ["E", "w"] + [f"W{i}" for i in range(L)] + [f"b{i}" for i in range(L)] + ["Wp", "bp"]
    vals = [E, w] + Ls + bs + [Wp, bp]
    acc = {kk: np.full_like(np.asarray(v, np.float32), 0.1) for kk, v in zip(keys, vals)}
    for step in range(2):
        Xb = X[step * B:(step + 1) * B]
        y = rng.choice([1.0, -1.0], B).astype(np.float32)[:, None]
        loss = m.partial_fit({"X": Xb, "Y": y})
        rl, E1, w1, L1, b1, Wp1, bp1, acc = orc.dfm_train_step(Xb, y, E, w, Ls, bs, Wp, bp, acc,
                                                               0.01, 0.01)
        assert np.isclose(loss, rl, rtol=1e-5)
        G = m.get_weights()
        _close_update(G["feature_embeddings"], E1, E)
        _close_update(G["feature_bias"][:, 0], w1, w)
        for i in range(L):
            _close_update(G[f"layer_{i}"], L1[i], Ls[i])
            _close_update(G[f"bias_{i}"][0], b1[i], bs[i])
        _close_update(G["concat_projection"][:, 0], Wp1, Wp)
        assert np.isclose(float(G["concat_bias"]), bp1, rtol=1e-5, atol=1e-4 * abs(bp1 - bp))
        E, w, Ls, bs, Wp, bp = E1, w1, L1, b1, Wp1, bp1
    # the scoring path sees the updated weights: the oracle forward on the
    # GPU's own trained weights (the training comparison above carries the
    # float-atomics noise; the forward alone is held to 1e-5)
    G = m.get_weights()
    Xs = X[:50]
    ref = orc.dfm_out(Xs, G["feature_embeddings"], G["feature_bias"][:, 0],
                      [G[f"layer_{i}"] for i in range(L)], [G[f"bias_{i}"] for i in range(L)],
                      G["concat_projection"], np.float32(G["concat_bias"]))[:, 0]
    got = m.score_rows(Xs)[:, 0]
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max())


def test_dfm_train_loop_end_to_end(tmp_path):
    from hhfm_amd.DFM import Train
    np.random.seed(2016)
    t = Train(_args(tmp_path, lamda=0.01, lr=0.01, epoch=3, hidden_factor=16))
    losses = t.train()
    assert len(losses) == 2 and losses[1] < losses[0]
    assert "DFM Epoch 1" in open(tmp_path / "result.txt").read()


@pytest.mark.parametrize("k,A,ctx,B,opt", [
    (64, 64, (7, 2, 3), 1000, "AdagradOptimizer"),       # Frappe F=5, the reference's k=A
    (16, 32, (5, 4, 6, 3, 7, 2, 2, 3, 4, 3), 301, "AdagradOptimizer"),   # F=12 (resturant/ml width), ragged
    (8, 4, (), 7, "GradientDescentOptimizer"),            # F=2: one pair, tiny batch
    (128, 128, (7, 2, 3), 600, "AdagradOptimizer"),       # main.py's factor 128
    (16, 32, (7, 2, 3), 301, "MomentumOptimizer"),        # AFM.py:157-158
    (32, 16, (5, 4, 6), 500, "AdamOptimizer"),            # AFM.py:151-152
])
def test_afm_partial_fit_matches_oracle(k, A, ctx, B, opt):
    """AFM partial_fit (AFM.py:144-156, 205-207): every variable after two
    steps vs the oracle's TF-semantics step."""
    from hhfm_amd.AFM import AFM
    rng = np.random.default_rng(k + A + B)
    nu, ni = 60, 200
    X, M = _rows(rng, 2 * B, nu, ni, ctx)
    F = X.shape[1]
    m = AFM(nu, ni, M, 1, [A, k], None, 0.1, 100.0, [1, 1], opt, 0.999, F)
    W = m.get_weights()
    W["feature_bias"] = rng.normal(0, 0.01, (M, 1)).astype(np.float32)
    W["prediction"] = rng.normal(1, 0.2, (k, 1)).astype(np.float32)
    m.set_weights(feature_bias=W["feature_bias"], prediction=W["prediction"])
    if opt in ("MomentumOptimizer", "AdamOptimizer"):
        # at the 0.01 init every pair's pre-activation has the sign of its
        # bias, so d attention_b = p · Σ_pairs dlogit = 0 exactly and both
        # sides hold only summation noise in that slot: spread the pairs
        m.set_weights(feature_embeddings=rng.normal(0, 0.3, (M, k)).astype(np.float32))
    names = ["feature_embeddings", "feature_bias", "bias", "attention_W", "attention_b",
             "attention_p", "prediction"]
    keys = ["E", "w", "w0", "W", "b", "p", "P"]
    o = OPTS[opt]
    for step in range(2):
        G = m.get_weights()
        cur = [np.asarray(G[n], np.float32) for n in names]
        cur[2] = cur[2].reshape(())
        acc = {kk: v for kk, v in zip(keys, _slots_of(m, names, o, cur)) if v is not None}
        Xb = X[step * B:(step + 1) * B]
        y = rng.choice([1.0, -1.0], B).astype(np.float32)[:, None]
        loss = m.partial_fit({"X": Xb, "Y": y})
        rl, *new, acc = orc.afm_train_step(Xb, y, *cur, acc, 0.1, 100.0, optimizer=o,
                                           step=step + 1)
        _, *gnew, _ = orc.afm_train_step(Xb, y, *cur, {}, 1.0, 100.0, optimizer="sgd")
        assert np.isclose(loss, rl, rtol=1e-5), (loss, rl)
        G = m.get_weights()
        for n, kk, v_new, v_old, v_g in zip(names, keys, new, cur, gnew):
            got = np.asarray(G[n], np.float32).reshape(np.shape(v_new))
            _check_var(got, np.asarray(v_new, np.float32), v_old, o,
                       np.asarray(v_old, np.float32) - np.asarray(v_g, np.float32).reshape(
                           np.shape(v_old)))
            if o != "sgd":
                _check_slot(m._train_state[n].cpu().numpy(), acc[kk], o)
    # the scoring path sees the updated weights
    G = m.get_weights()
    cur = [np.asarray(G[n], np.float32) for n in names]
    Xs = X[:50]
    ref = orc.afm_out(Xs, cur[0], cur[1], cur[2].reshape(()), cur[3], cur[4], cur[5],
                      cur[6])[:, 0]
    got = m.score_rows(Xs)[:, 0]
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max())


def test_afm_train_loop_end_to_end(tmp_path):
    from hhfm_amd.AFM import Train
    np.random.seed(2016)
    t = Train(_args(tmp_path, hidden_factor="[16,16]", keep="[1,1]", lamda_attention=100.0,
                    attention=1, decay=0.999, activation="relu"))
    losses = t.train()
    assert len(losses) == 2 and losses[1] < losses[0]
    assert "AFM Epoch 1" in open(tmp_path / "result.txt").read()


@pytest.mark.parametrize("entry", ["FM_main", "M7_main", "AFM_main", "DFM_main"])
def test_main_entry_points_through_argv(entry, tmp_path):
    """main.py's surface (Newcode/main.py:47-63 calls X_main(dataname, factor,
    TopK)): each entry point parses the reference's flags from argv, loads
    synth_frappe through LoadData, trains one epoch on the GPU (the loop
    whose batch stream test_epoch_stream.py pins) and appends the
    reference's result lines (Init + epoch 1 at --verbose 1; HHFM evaluates
    at init only before epoch 10, OurModel7.py:404) to --result_file."""
    import importlib
    mod = {"FM_main": "FM", "M7_main": "OurModel7", "AFM_main": "AFM", "DFM_main": "DFM"}[entry]
    fn = getattr(importlib.import_module(f"hhfm_amd.{mod}"), entry)
    out = tmp_path / "result.txt"
    argv = ["--path", G + "/", "--epoch", "2", "--batch_size", "4096",
            "--result_file", str(out)]
    if entry != "M7_main":
        argv += ["--verbose", "1"]
    np.random.seed(2016)
    session = fn("synth_frappe", 16, 5, argv)
    assert len(session.loss_epoch) == 1 and np.isfinite(session.loss_epoch[0])
    lines = out.read_text().splitlines()
    assert lines[0].startswith("Dataset=synth_frappe ") and "Init:" in lines[0]
    assert len(lines) == (1 if entry == "M7_main" else 2), lines
    for ln in lines:
        auc = float(ln.split("train=AUC:")[1].split(";")[0])
        hr = float(ln.split("HR:")[1].split(",")[0])
        assert 0.0 <= auc <= 1.0 and 0.0 <= hr <= 1.0, ln
