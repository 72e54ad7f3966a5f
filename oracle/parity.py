"""Parity checkers shared by tests/ and bench.py — TEST INFRASTRUCTURE ONLY.

These functions compare a GPU result with the oracle (fm_oracle.py /
cpu_oracle.c); they never produce a result the product path returns.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s checking legs use
them.

Contracts:
  * top-K index lists: a position may differ from the oracle's list only
    where the two items' float64 scores lie within TIE_WINDOW x the dot
    product's Σ|terms| — two fp32 summation orders may order such a pair
    either way.  Every such swap is counted and reported.
  * fp32 row scores: within 1e-5 relative of the float64 value for every
    row whose condition number Σ|terms| / |out| is at most KAPPA_MAX; rows
    above it are counted and held to the normwise bound.
"""
from __future__ import annotations

import numpy as np

TIE_WINDOW = 2e-6
KAPPA_MAX = 100.0


def bf16_round(x):
    """Round-to-nearest-even float32 -> bfloat16 -> float32 (what the GPU reads)."""
    import torch
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(torch.bfloat16).float().numpy()


# ---------------------------------------------------------------------------
# top-K lists
# ---------------------------------------------------------------------------
def hhfm_exact(A, E, n_user, ctx=(2, 5), time=(0, 0)):
    """float64 score of (query b, item offsets ids) for OurModel7.py:294 with
    the fp32 query vector h of :270-292, and Σ|h_e i_e|."""
    from oracle import fm_oracle as orc
    A = np.asarray(A)
    h = orc._hybrid(E, A[:, 0], A[:, ctx[0]:ctx[1]] if ctx[1] > ctx[0] else None,
                    A[:, time[0]:time[1]] if time[1] > time[0] else None).astype(np.float64)

    def exact(b, ids):
        it = E[n_user + np.asarray(ids, np.int64)].astype(np.float64)
        return it @ h[b], np.abs(it) @ np.abs(h[b])
    return exact


def fm_exact(A, E, w, n_user, ctx=(2, 5)):
    """float64 (u+f)·(i+f) + w_i of FM.py:176-185 and its Σ|terms|."""
    A = np.asarray(A, np.int64)
    f = E[A[:, ctx[0]:ctx[1]]].sum(1, dtype=np.float32)
    q = (E[A[:, 0]] + f).astype(np.float64)
    f = f.astype(np.float64)

    def exact(b, ids):
        rows = n_user + np.asarray(ids, np.int64)
        it = E[rows].astype(np.float64)
        s = (it + f[b]) @ q[b] + w[rows]
        return s, (np.abs(it) + np.abs(f[b])) @ np.abs(q[b]) + np.abs(w[rows])
    return exact


def topk_tie_count(got_i, ref_i, exact, window=TIE_WINDOW):
    """(unexplained, tie_swaps, duplicates) of ``got_i`` against the oracle's
    ``ref_i``: a differing position is a tie swap when the float64 gap of the
    two items is within ``window`` of Σ|terms|, unexplained otherwise."""
    got_i = np.asarray(got_i)
    ref_i = np.asarray(ref_i)
    if got_i.shape != ref_i.shape:
        return int(ref_i.size), 0, 0
    dup = sum(int(len(np.unique(r)) != len(r)) for r in got_i)
    bad = swaps = 0
    for b, p in np.argwhere(got_i != ref_i):
        s, mag = exact(b, [got_i[b, p], ref_i[b, p]])
        gap = abs(s[0] - s[1]) / max(float(np.max(mag)), 1e-300)
        if gap <= window:
            swaps += 1
        else:
            bad += 1
    return bad, swaps, dup


def topk_tie_swaps(got_i, ref_i, exact, window=TIE_WINDOW):
    """Number of positions where ``got_i`` differs from the oracle's ``ref_i``;
    raises unless every one is an fp32 tie (see TIE_WINDOW)."""
    got_i = np.asarray(got_i)
    ref_i = np.asarray(ref_i)
    assert got_i.shape == ref_i.shape, (got_i.shape, ref_i.shape)
    for row in got_i:
        assert len(np.unique(row)) == len(row), "duplicate item in a top-K list"
    bad = np.argwhere(got_i != ref_i)
    for b, p in bad:
        s, mag = exact(b, [got_i[b, p], ref_i[b, p]])
        gap = abs(s[0] - s[1]) / max(float(np.max(mag)), 1e-300)
        assert gap <= window, (f"query {b} position {p}: got item {got_i[b, p]}, oracle item "
                               f"{ref_i[b, p]}, float64 gap {gap:.3g} of Σ|terms| > {window}")
    return len(bad)


# ---------------------------------------------------------------------------
# FM.out rows (K1)
# ---------------------------------------------------------------------------
def fm_rows_exact(X, E, w, w0=0.0):
    """float64 FM.out of FM.py:99-120 and its Σ|terms| per row."""
    X = np.asarray(X, np.int64)
    e = np.asarray(E)[X].astype(np.float64)
    s = e.sum(1)
    q = (e * e).sum(1)
    out = (0.5 * (s * s - q)).sum(1) + float(w0)
    mag = (0.5 * (s * s + q)).sum(1) + abs(float(w0))
    if w is not None:
        wx = np.asarray(w, np.float64).reshape(-1)[X]
        out = out + wx.sum(1)
        mag = mag + np.abs(wx).sum(1)
    return out, mag


def row_check(got, exact, mag, rel=1e-5, kappa_max=KAPPA_MAX):
    """Elementwise check of fp32 row scores against their float64 values:
    every row with κ = Σ|terms| / |exact| <= kappa_max must be within ``rel``
    relative; rows above κ are counted and held to ``rel`` of Σ|terms|."""
    got = np.asarray(got, np.float64).reshape(-1)
    exact = np.asarray(exact, np.float64).reshape(-1)
    mag = np.asarray(mag, np.float64).reshape(-1)
    err = np.abs(got - exact)
    kappa = mag / np.maximum(np.abs(exact), 1e-300)
    well = kappa <= kappa_max
    relerr = err / np.maximum(np.abs(exact), 1e-300)
    normwise = err / np.maximum(mag, 1e-300)
    n_bad = int((relerr[well] > rel).sum()) + int((normwise[~well] > rel).sum())
    return {"rows": int(got.size), "rows_kappa_le_max": int(well.sum()),
            "rows_kappa_gt_max": int((~well).sum()), "kappa_max": kappa_max,
            "max_rel_err_kappa_le_max": float(relerr[well].max()) if well.any() else 0.0,
            "max_rel_err_normwise": float(normwise.max()) if got.size else 0.0,
            "rows_failing": n_bad, "tolerance": rel, "parity": n_bad == 0}


# ---------------------------------------------------------------------------
# DeepFM rows (K3)
# ---------------------------------------------------------------------------
def dfm_magnitude(X, E, w, layers, biases, Wp, bp):
    """Σ_j |concat_j · Wp_j| + |bp| in float64 (natural scale of DFM.py:137)."""
    X = np.asarray(X, np.int64)
    e = E[X].astype(np.float64)
    y1 = w[X].astype(np.float64)
    s = e.sum(1)
    y2 = 0.5 * (s * s - (e * e).sum(1))
    h = e.reshape(len(X), -1)
    for Wl, bl in zip(layers, biases):
        h = np.maximum(h @ Wl.astype(np.float64) + bl.astype(np.float64), 0)
    cat = np.concatenate([y1, y2, h], 1)
    return (np.abs(cat * Wp.reshape(1, -1))).sum(1) + abs(float(bp))


def dfm_rows_exact(X, E, w, layers, biases, Wp, bp):
    """float64 DeepFM.out of DFM.py:104-137 (ReLU after every layer, :128) and
    its natural magnitude Σ_j |concat_j · Wp_j| + |bp| per row."""
    X = np.asarray(X, np.int64)
    e = np.asarray(E, np.float64)[X]
    y1 = np.asarray(w, np.float64).reshape(-1)[X]
    s = e.sum(1)
    y2 = 0.5 * (s * s - (e * e).sum(1))
    h = e.reshape(len(X), -1)
    for Wl, bl in zip(layers, biases):
        h = np.maximum(h @ np.asarray(Wl, np.float64) + np.asarray(bl, np.float64).reshape(-1), 0)
    t = np.concatenate([y1, y2, h], 1) * np.asarray(Wp, np.float64).reshape(1, -1)
    return t.sum(1) + float(bp), np.abs(t).sum(1) + abs(float(bp))


def dfm_bf16_out(X, E, w, layers, biases, Wp, bp):
    """bf16 MLP mode of DFM.py:104-137: table rows, weights and stored hidden
    activations rounded to bf16; accumulation and the final dot in fp32; FM
    part in fp32."""
    X = np.asarray(X, np.int64)
    e = E[X]
    y1 = w[X]
    s = e.sum(1, dtype=np.float32)
    y2 = np.float32(0.5) * (s * s - (e * e).sum(1, dtype=np.float32))
    h = bf16_round(e.reshape(len(X), -1))
    L = len(layers)
    for i, (Wl, bl) in enumerate(zip(layers, biases)):
        h = np.maximum(h @ bf16_round(Wl) + bl, 0).astype(np.float32)
        if i < L - 1:
            h = bf16_round(h)
    cat = np.concatenate([y1, y2, h], 1)
    return (cat @ Wp.reshape(-1, 1))[:, 0] + np.float32(bp)


# ---------------------------------------------------------------------------
# AFM rows (K4)
# ---------------------------------------------------------------------------
def afm_rows_exact(X, E, w, w0, W, b, pvec, P):
    """float64 AFM.out of AFM.py:103-142 (attention on, keep = [1, 1]) and
    its natural magnitude Σ_pairs att·Σ_c |(e_i ⊙ e_j)_c P_c| + Σ|w| + |w0|."""
    X = np.asarray(X, np.int64)
    e = np.asarray(E, np.float64)[X]
    F = e.shape[1]
    pr = np.stack([e[:, i] * e[:, j] for i in range(F) for j in range(i + 1, F)], 1)
    z = pr @ np.asarray(W, np.float64) + np.asarray(b, np.float64).reshape(-1)
    logit = (np.maximum(z, 0) * np.asarray(pvec, np.float64).reshape(-1)).sum(-1)
    ex = np.exp(logit - logit.max(1, keepdims=True))
    att = ex / ex.sum(1, keepdims=True)
    t = att[:, :, None] * pr * np.asarray(P, np.float64).reshape(1, 1, -1)
    fb = np.asarray(w, np.float64).reshape(-1)[X]
    out = t.sum((1, 2)) + fb.sum(1) + float(w0)
    mag = np.abs(t).sum((1, 2)) + np.abs(fb).sum(1) + abs(float(w0))
    return out, mag
