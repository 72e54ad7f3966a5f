#!/usr/bin/env python3
"""Workload for the rocprofv3 --pmc passes of K1 (hhfm_fm_score_rows).

Two launches of the headline kernel on the bench table (16.8 M x 64 fp32):
  1. `calib`: user/item ids sequential (row r reads user r, item n_user+r),
     ctx ids Frappe-like — the table's user+item halves are streamed exactly
     once, so its HBM read bytes are known (B*(2*256+20+8)) and calibrate
     FETCH_SIZE for this access pattern (MI355X_MICROARCH.md §HBM: gfx950
     FETCH_SIZE under-counts wide coalesced reads by 2x);
  2. `bench`: the bench.py workload (uniform random ids), same B;
  3. `bench without w`: same rows with the bias gathers removed (isolates
     the cost of the two 4-byte w gathers per row).
Run under: rocprofv3 --pmc FETCH_SIZE ... -- python scripts/pmc_fm_rows.py
           rocprofv3 --pmc WRITE_SIZE ... -- python scripts/pmc_fm_rows.py
(bench.py's pmc_traffic runs both passes at the bench's row count)
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from hhfm_amd import ops  # noqa: E402

rows = int(os.environ.get("PMC_ROWS", 1 << 23))
k = int(os.environ.get("PMC_K", 64))
dev = torch.device("cuda", 0)
idx, E, w, M = bench.make_batch(rows, 8 << 20, 8 << 20, k, 1, dev)
out = torch.empty(rows, dtype=torch.float32, device=dev)
seq = idx.clone()
r = torch.arange(rows, device=dev, dtype=torch.int32)
seq[:, 0] = r % (8 << 20)
seq[:, 1] = (8 << 20) + r % (8 << 20)
torch.cuda.synchronize()
# two launches each; rocprof reports one row per dispatch, in order:
# calib, calib, bench, bench, bench-without-w, bench-without-w
for x, ww in ((seq, w), (seq, w), (idx, w), (idx, w), (idx, None), (idx, None)):
    ops.fm_score_rows(x, E, ww, 0.0, out=out)
torch.cuda.synchronize()
print("pmc workload done", rows)
