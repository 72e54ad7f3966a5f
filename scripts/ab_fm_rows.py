#!/usr/bin/env python3
"""Interleaved A/B of hhfm_fm_score_rows_ex flag variants in ONE process on
the bench workload (guide §5.4 rule 24): rounds x variants, median/min."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from hhfm_amd._native import native  # noqa: E402

rows = int(os.environ.get("AB_ROWS", 1 << 25))
variants = [int(v) for v in os.environ.get("AB_FLAGS", "0,1").split(",")]
rounds = int(os.environ.get("AB_ROUNDS", 8))
dev = torch.device("cuda", 0)
idx, E, w, M = bench.make_batch(rows, 8 << 20, 8 << 20, 64, 1, dev)
outs = {v: torch.empty(rows, dtype=torch.float32, device=dev) for v in variants}
nat = native()
st = torch.cuda.current_stream().cuda_stream


def run(v):
    nat.fm_score_rows_ex(idx.data_ptr(), rows, 5, E.data_ptr(), M, 64, 0, w.data_ptr(), 0.0,
                         outs[v].data_ptr(), v, 0, st)


for v in variants:
    run(v)
torch.cuda.synchronize()
times = {v: [] for v in variants}
for r in range(rounds):
    for v in variants:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            run(v)
        b.record()
        b.synchronize()
        times[v].append(a.elapsed_time(b) / 3)
ref = outs[variants[0]]
res = {}
for v in variants:
    t = np.array(times[v])
    res[v] = {"median_ms": float(np.median(t)), "min_ms": float(t.min()),
              "same_output": bool(torch.equal(outs[v], ref)),
              "GB_s_algorithmic": 1324 * rows / (np.median(t) * 1e-3) / 1e9}
print(json.dumps(res, indent=1))
