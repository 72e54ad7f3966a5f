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
