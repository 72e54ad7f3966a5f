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
