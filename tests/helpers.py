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


# bf16 rounding and the top-K tie contract live in oracle/parity.py (shared
# with bench.py's checking legs); re-exported here for the tests.
import os  # noqa: E402

from oracle import parity as _parity  # noqa: E402
from oracle.parity import TIE_WINDOW, bf16_round, fm_exact, hhfm_exact  # noqa: E402,F401

# Per-case parity record (tie swaps, ill-conditioned row counts), printed in
# the pytest terminal summary and written to $HHFM_PARITY_REPORT (conftest).
PARITY_LOG = []


def log_parity(kind, **fields):
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").rsplit(" (", 1)[0]
    PARITY_LOG.append(dict(test=test, kind=kind, **fields))


def topk_tie_swaps(got_i, ref_i, exact, window=TIE_WINDOW):
    """oracle/parity.topk_tie_swaps (raises unless every differing position
    is a float64-verified fp32 tie), with the count logged per case."""
    n = _parity.topk_tie_swaps(got_i, ref_i, exact, window)
    log_parity("topk_tie_swaps", swaps=int(n), positions=int(np.asarray(got_i).size))
    return n


def kappa_check(kind, got, ref32, exact, mag, rtol=1e-5, kappa_max=_parity.KAPPA_MAX):
    """north_star 1e-5 *relative*, elementwise: every row whose condition
    number κ = Σ|terms| / |exact| is at most ``kappa_max`` must be within
    ``rtol`` of its float64 value ``exact``; beyond that fp32 itself cannot
    promise 1e-5 relative, so those rows are held to ``rtol`` of Σ|terms|
    (normwise) and their error is logged beside the fp32 oracle's (``ref32``)
    own.  The per-case record goes to the parity report (conftest)."""
    got = np.asarray(got, np.float64).reshape(-1)
    ex = np.asarray(exact, np.float64).reshape(-1)
    mag = np.asarray(mag, np.float64).reshape(-1)
    den = np.maximum(np.abs(ex), 1e-300)
    kappa = mag / den
    rel_gpu = np.abs(got - ex) / den
    ok = kappa <= kappa_max
    rec = dict(rows=int(ok.size), rows_kappa_gt_100=int((~ok).sum()),
               max_rel_err_kappa_le_100=float(rel_gpu[ok].max()) if ok.any() else 0.0,
               max_rel_err_kappa_gt_100=float(rel_gpu[~ok].max()) if (~ok).any() else 0.0,
               oracle_max_rel_err_kappa_gt_100=0.0)
    if ref32 is not None and (~ok).any():
        r32 = np.asarray(ref32, np.float64).reshape(-1)
        rec["oracle_max_rel_err_kappa_gt_100"] = float((np.abs(r32 - ex) / den)[~ok].max())
    log_parity(kind, **rec)
    if ok.any():
        assert rel_gpu[ok].max() <= rtol, (kind, float(rel_gpu[ok].max()))
    norm = np.abs(got - ex) / np.maximum(mag, 1e-300)
    assert norm.max() <= rtol, (kind, "normwise", float(norm.max()))
    return rec
