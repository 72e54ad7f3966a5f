"""Shared test helpers: Frappe-shape synthetic data (seeded)."""
import numpy as np

# Frappe cardinalities measured by importing NewLoadData:
# 957 users, 4082 items, context columns with 7 / 2 / 3 values.
FRAPPE = dict(n_user=957, n_item=4082, ctx=(7, 2, 3))


def frappe_vocab(n_user=957, n_item=4082, ctx=(7, 2, 3)):
    """Global-id layout of LoadData: users, then items, then ctx values
    (NewLoadData.py:29-34). Returns (features_M, ctx_offsets)."""
    offs = []
    o = n_user + n_item
    for c in ctx:
        offs.append(o)
        o += c
    return o, offs


def synth_rows(rng, B, n_user, n_item, ctx, time_fields=0, time_card=0):
    """int32 rows [user, item, ctx..., time...] with global ids."""
    M, offs = frappe_vocab(n_user, n_item, ctx)
    cols = [rng.integers(0, n_user, B), rng.integers(n_user, n_user + n_item, B)]
    for o, c in zip(offs, ctx):
        cols.append(rng.integers(o, o + c, B))
    if time_fields:
        # time fields index previous items (OurModel7 jiaju/resturant layout)
        for _ in range(time_fields):
            cols.append(rng.integers(n_user, n_user + n_item, B))
    return np.stack(cols, axis=1).astype(np.int32), M


def table(rng, M, k, std=0.01):
    return rng.normal(0.0, std, size=(M, k)).astype(np.float32)


def bf16_round(x):
    """Round-to-nearest-even float32 -> bfloat16 -> float32 (what the GPU reads)."""
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).to(torch.bfloat16).float().numpy()


# ---------------------------------------------------------------------------
# Top-K exactness (north_star: bit-exact top-K index sets)
# ---------------------------------------------------------------------------
# A position may differ from the oracle's list only when the two items'
# float64 scores lie within TIE_WINDOW x the dot product's Σ|terms| (≈34 fp32
# ulps of accumulated rounding): two fp32 summation orders may legally order
# such a pair either way.  Every such swap is counted and reported; the
# golden fixtures and the seeded cases are held to zero.
TIE_WINDOW = 2e-6


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
