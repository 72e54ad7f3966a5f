"""The oracle's hand-written TF gradients (H6) vs finite differences of the
oracle's own loss (float64), and TF Adagrad semantics."""
import numpy as np

from oracle import fm_oracle as orc


def _fd(loss_fn, E, ids, eps=1e-3):
    E = E.astype(np.float64)
    out = []
    for (r, c) in ids:
        Ep, Em = E.copy(), E.copy()
        Ep[r, c] += eps
        Em[r, c] -= eps
        out.append((loss_fn(Ep) - loss_fn(Em)) / (2 * eps))
    return np.array(out)


def test_fm_gradient_matches_finite_differences():
    rng = np.random.default_rng(0)
    M, k, B, lam = 30, 4, 20, 0.1
    X = rng.integers(0, M, size=(B, 5))
    X[0, 3] = X[0, 2]                       # repeated id inside one row
    y = rng.integers(0, 2, B).astype(np.float64)
    E = rng.normal(0, 0.3, (M, k))
    w = rng.normal(0, 0.3, M)

    def loss(Ev):
        e = Ev[X]
        s = e.sum(1)
        out = (0.5 * (s * s - (e * e).sum(1))).sum(1) + w[X].sum(1)
        return ((y - out) ** 2).sum() / 2 + lam * (Ev ** 2).sum() / 2

    lr = 1e-3
    _, E1, *_ = orc.fm_train_step(X, y, E.astype(np.float32), w, 0.0, np.zeros((M, k), np.float32),
                                  np.zeros(M, np.float32), 0.0, lr, lam, optimizer="sgd")
    grad = (E.astype(np.float32) - E1) / lr
    ids = [(X[0, 2], 1), (X[3, 0], 0), (X[5, 4], 3), (int(np.setdiff1d(np.arange(M), X)[0]), 2)]
    fd = _fd(loss, E, ids)
    got = np.array([grad[r, c] for r, c in ids])
    assert np.allclose(got, fd, rtol=2e-3, atol=2e-4)


def test_hhfm_gradient_matches_finite_differences():
    rng = np.random.default_rng(1)
    M, k, B, lam = 40, 4, 12, 0.01
    X = np.stack([rng.integers(0, 10, B), rng.integers(10, 30, B), rng.integers(30, 35, B),
                  rng.integers(35, 40, B)], 1)
    Neg = rng.integers(10, 30, size=(B, 10))
    E = rng.normal(0, 0.5, (M, k))

    def loss(Ev):
        h = Ev[X[:, 0]] + Ev[X[:, 2:]].sum(1)
        pos = (h * Ev[X[:, 1]]).sum(1)
        neg = (h[:, None, :] * Ev[Neg]).sum(2)
        z = pos - neg.max(1)
        return -np.log(1 / (1 + np.exp(-z))).sum() + lam * (Ev ** 2).sum() / 2

    lr = 1e-3
    _, E1, _ = orc.hhfm_train_step(X, Neg, E.astype(np.float32), np.zeros((M, k), np.float32), lr,
                                   lam, 2, 0, optimizer="sgd")
    grad = (E.astype(np.float32) - E1) / lr
    ids = [(X[0, 0], 1), (X[1, 1], 2), (X[2, 2], 0), (Neg[0, 3], 3), (X[4, 3], 1)]
    fd = _fd(loss, E, ids, eps=1e-4)
    got = np.array([grad[r, c] for r, c in ids])
    assert np.allclose(got, fd, rtol=3e-3, atol=3e-4)


def test_dfm_gradient_matches_finite_differences():
    """DeepFM (DFM.py:139-155): every variable's gradient, incl. a repeated id."""
    rng = np.random.default_rng(2)
    M, k, B, F, lam = 30, 4, 16, 3, 0.05
    X = rng.integers(0, M, (B, F))
    X[0, 1] = X[0, 0]
    y = rng.choice([1.0, -1.0], B)
    E, w = rng.normal(0, 0.3, (M, k)), rng.normal(0, 0.3, M)
    Ls = [rng.normal(0, 0.5, (F * k, 6)), rng.normal(0, 0.5, (6, 5))]
    bs = [rng.normal(0, 0.3, 6), rng.normal(0.3, 0.1, 5)]
    Wp, bp = rng.normal(0, 0.5, F + k + 5), 0.01

    def loss(E, w, Ls, bs, Wp, bp):
        e = E[X]
        s = e.sum(1)
        h = e.reshape(B, -1)
        for W, b in zip(Ls, bs):
            h = np.maximum(h @ W + b, 0)
        out = np.concatenate([w[X], 0.5 * (s * s - (e * e).sum(1)), h], 1) @ Wp + bp
        return ((y - out) ** 2).sum() / 2 + lam * ((Wp ** 2).sum() + sum((W ** 2).sum() for W in Ls)) / 2

    lr = 1e-3
    l0, E1, w1, L1, b1, Wp1, bp1, _ = orc.dfm_train_step(X, y, E, w, Ls, bs, Wp, bp, {}, lr, lam,
                                                          optimizer="sgd")
    assert abs(l0 - loss(E, w, Ls, bs, Wp, bp)) < 1e-4 * abs(l0)

    def fd(fn, arr, i, eps=1e-5):
        a = arr.copy()
        a[i] += eps
        lp = fn(a)
        a[i] -= 2 * eps
        return (lp - fn(a)) / (2 * eps)

    checks = [
        ((E.astype(np.float32) - E1) / lr, (X[0, 0], 1), fd(lambda a: loss(a, w, Ls, bs, Wp, bp), E, (X[0, 0], 1))),
        ((w.astype(np.float32) - w1) / lr, (X[2, 1],), fd(lambda a: loss(E, a, Ls, bs, Wp, bp), w, (X[2, 1],))),
        ((Ls[0].astype(np.float32) - L1[0]) / lr, (3, 2), fd(lambda a: loss(E, w, [a, Ls[1]], bs, Wp, bp), Ls[0], (3, 2))),
        ((Ls[1].astype(np.float32) - L1[1]) / lr, (1, 4), fd(lambda a: loss(E, w, [Ls[0], a], bs, Wp, bp), Ls[1], (1, 4))),
        ((bs[1].astype(np.float32) - b1[1]) / lr, (2,), fd(lambda a: loss(E, w, Ls, [bs[0], a], Wp, bp), bs[1], (2,))),
        ((Wp.astype(np.float32) - Wp1) / lr, (F + k + 2,), fd(lambda a: loss(E, w, Ls, bs, a, bp), Wp, (F + k + 2,))),
        ((Wp.astype(np.float32) - Wp1) / lr, (F + 1,), fd(lambda a: loss(E, w, Ls, bs, a, bp), Wp, (F + 1,))),
    ]
    for grad, i, ref in checks:
        assert np.isclose(grad[i], ref, rtol=2e-3, atol=2e-4), (i, grad[i], ref)
    dbp = (np.float32(bp) - bp1) / lr
    assert np.isclose(dbp, fd(lambda a: loss(E, w, Ls, bs, Wp, a[0]), np.array([bp]), (0,)), rtol=2e-3)


def test_tf_adagrad_semantics():
    v, g, a = np.float32([1.0]), np.float32([0.5]), np.float32([0.1])
    v1, a1 = orc.tf_adagrad(v, g, a, 0.1)
    assert a1[0] == np.float32(0.35)
    assert np.isclose(v1[0], 1.0 - 0.1 * 0.5 / np.sqrt(0.35))


def test_afm_gradient_matches_finite_differences():
    """AFM (AFM.py:144-156): every variable's gradient, incl. a repeated id."""
    rng = np.random.default_rng(3)
    M, k, A, B, F, lam = 25, 4, 8, 10, 4, 0.3
    X = rng.integers(0, M, (B, F))
    X[0, 2] = X[0, 1]
    y = rng.choice([1.0, -1.0], B)
    E, w = rng.normal(0, 0.5, (M, k)), rng.normal(0, 0.3, M)
    W, b = rng.normal(0, 0.6, (k, A)), rng.normal(0, 0.3, (1, A))
    pv, P = rng.normal(0, 1, A), rng.normal(1, 0.3, (k, 1))
    w0 = 0.05
    pairs = [(i, j) for i in range(F) for j in range(i + 1, F)]

    def loss(E, w, w0, W, b, pv, P):
        e = E[X]
        pr = np.stack([e[:, i] * e[:, j] for i, j in pairs], 1)
        lg = (pv * np.maximum(pr @ W + b, 0)).sum(-1)
        a = np.exp(lg - lg.max(1, keepdims=True))
        a /= a.sum(1, keepdims=True)
        out = (a[:, :, None] * pr).sum(1) @ P[:, 0] + w[X].sum(1) + w0
        return ((y - out) ** 2).sum() / 2 + lam * (W ** 2).sum() / 2

    lr = 1e-3
    l0, E1, w1, w01, W1, b1, pv1, P1, _ = orc.afm_train_step(X, y, E, w, w0, W, b, pv, P, {},
                                                             lr, lam, optimizer="sgd")
    args = [E, w, np.array([w0]), W, b, pv, P]
    assert abs(l0 - loss(E, w, w0, W, b, pv, P)) < 1e-4 * abs(l0)

    def fd(which, i, eps=1e-5):
        def f(a):
            v = list(args)
            v[which] = a
            return loss(v[0], v[1], v[2][0], *v[3:])
        a = args[which].astype(np.float64).copy()
        a[i] += eps
        lp = f(a)
        a[i] -= 2 * eps
        return (lp - f(a)) / (2 * eps)

    new = [E1, w1, np.array([w01]), W1, b1.reshape(1, -1), pv1, P1.reshape(-1, 1)]
    for which, i in [(0, (X[0, 1], 2)), (0, (X[4, 3], 0)), (1, (X[2, 1],)), (2, (0,)),
                     (3, (1, 5)), (3, (3, 0)), (4, (0, 6)), (5, (2,)), (6, (1, 0))]:
        grad = (args[which].astype(np.float32)[i] - new[which][i]) / lr
        ref = fd(which, i)
        assert np.isclose(grad, ref, rtol=3e-3, atol=3e-4), (which, i, grad, ref)


def test_tf_momentum_dense_and_sparse():
    """MomentumOptimizer(0.95) (FM.py:135-136): ApplyMomentum on a dense
    gradient, SparseApplyMomentum (touched rows only) on an IndexedSlices."""
    v = np.float32([[1.0, 2.0], [3.0, 4.0], [5.0, 6.0]])
    g = np.float32([[0.5, -1.0], [0.0, 0.0], [2.0, 0.25]])
    acc = np.float32([[0.1, 0.2], [0.3, 0.4], [0.5, 0.6]])
    v1, a1 = orc.tf_apply("momentum", v, g, acc, 0.1)
    assert np.array_equal(a1, (acc * np.float32(0.95) + g).astype(np.float32))
    assert np.allclose(v1, v - 0.1 * a1)
    # ids [2, 0, 2]: row 1 untouched keeps var and accumulator; a touched row
    # with a zero gradient still decays
    v2, a2 = orc.tf_apply("momentum", v, g, acc, 0.1, rows=np.array([2, 0, 2]))
    assert np.array_equal(v2[1], v[1]) and np.array_equal(a2[1], acc[1])
    assert np.array_equal(a2[[0, 2]], a1[[0, 2]]) and np.allclose(v2[[0, 2]], v1[[0, 2]])
    g0 = np.zeros_like(g)
    v3, a3 = orc.tf_apply("momentum", v, g0, acc, 0.1, rows=np.array([1]))
    assert np.allclose(a3[1], acc[1] * 0.95) and np.allclose(v3[1], v[1] - 0.1 * a3[1])
    assert np.array_equal(v3[0], v[0])


def test_tf_adam_dense_and_sparse():
    """AdamOptimizer(0.9, 0.999, 1e-8) (FM.py:129-130): β powers start at β
    and advance after each step; the first step moves every coordinate with a
    gradient by ≈ lr·sign(g); sparse Adam decays m, v and moves untouched rows."""
    assert orc.adam_powers(1) == (np.float32(0.9), np.float32(0.999))
    b1p, b2p = orc.adam_powers(3)
    assert b1p == np.float32(np.float32(np.float32(0.9) * np.float32(0.9)) * np.float32(0.9))
    assert abs(b2p - 0.999 ** 3) < 1e-6
    v = np.float32([1.0, -2.0, 0.5, 3.0])
    g = np.float32([0.3, -0.02, 0.0, 5.0])
    slot = np.zeros(8, np.float32)
    v1, s1 = orc.tf_apply("adam", v, g, slot, 0.01, step=1)
    assert np.allclose(v - v1, 0.01 * np.sign(g), rtol=1e-4, atol=1e-7)
    assert np.allclose(s1[:4], 0.1 * g) and np.allclose(s1[4:], 0.001 * g * g, rtol=1e-4)  # f32 1−β2
    # float64 restatement of step 2 (dense)
    v2, s2 = orc.tf_apply("adam", v1, g, s1, 0.01, step=2)
    m = 0.9 * s1[:4].astype(np.float64) + 0.1 * g
    vv = 0.999 * s1[4:].astype(np.float64) + 0.001 * g.astype(np.float64) ** 2
    alpha = 0.01 * np.sqrt(1 - 0.999 ** 2) / (1 - 0.9 ** 2)
    assert np.allclose(v2, v1 - alpha * m / (np.sqrt(vv) + 1e-8), rtol=1e-6, atol=1e-7)
    # sparse: the id list touches 0 and 3 only, yet every row with m != 0 moves
    E = np.float32([[1.0], [2.0], [3.0], [4.0]])
    gs = np.float32([[0.5], [0.0], [0.0], [-0.5]])
    E1, t1 = orc.tf_apply("adam", E, gs, np.zeros(8, np.float32), 0.1, 1, rows=np.array([0, 3]))
    assert E1[1, 0] == E[1, 0] and E1[2, 0] == E[2, 0]     # m = 0 there: no move
    E2, t2 = orc.tf_apply("adam", E1, np.zeros_like(gs), t1, 0.1, 2, rows=np.array([1]))
    assert np.allclose(t2[:4], 0.9 * t1[:4]) and E2[0, 0] < E1[0, 0] and E2[3, 0] > E1[3, 0]


def test_tf_adam_powers_flush_to_zero():
    """TF multiplies beta1_power by β1 on FTZ/DAZ threads: the power falls
    from the smallest normal product straight to 0 at t = 829 and stays 0
    (never a denormal); α = lr·√(1 − β2^t) from then on."""
    b1_828, _ = orc.adam_powers(828)
    assert b1_828 >= np.finfo(np.float32).tiny
    for t in (829, 830, 1000, 2000):
        b1p, b2p = orc.adam_powers(t)
        assert b1p == 0.0 and 0.0 < b2p < 1.0
    v = np.float32([1.0, -2.0])
    g = np.float32([0.3, -0.02])
    slot = np.float32([0.01, -0.001, 1e-4, 1e-6])
    v1, s1 = orc.tf_apply("adam", v, g, slot, 0.01, step=900)
    alpha = np.float32(0.01 * np.sqrt(np.float32(1) - orc.adam_powers(900)[1], dtype=np.float32))
    assert np.allclose(v - v1, alpha * s1[:2] / (np.sqrt(s1[2:]) + 1e-8), rtol=1e-5)
