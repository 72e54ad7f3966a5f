"""Diagnostic: K1 at configs[1] (2^25 rows, 4.3 GB fp32 table) with the
shipped `w` gathers, with or without `w` (HAS_W off), timed with HIP events
over 20 back-to-back launches after warm-up.  Run under builds with
HHFM_K1_WMAP = 1 / 2 to see where the w lines come from."""
import json
import os
import sys

import torch

sys.path.append(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from hhfm_amd import ops  # noqa: E402  (a PYTHONPATH copy wins: appended path)

dev = torch.device("cuda", 0)
rows = 1 << 25
idx, E, w, M = bench.make_batch(rows, 8 << 20, 8 << 20, 64, 1, dev)
wbig = torch.zeros(M * 32, dtype=torch.float32, device=dev)   # room for the x32 map
wbig[: M] = w
out = torch.empty(rows, dtype=torch.float32, device=dev)


def timeit(fn, n=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / n


nat = ops.native()
st = torch.cuda.current_stream().cuda_stream


def run(wt):   # the C ABI directly: the diagnostic w buffer is larger than M
    nat.fm_score_rows_ex(idx.data_ptr(), rows, 5, E.data_ptr(), M, 64, 0,
                         0 if wt is None else wt.data_ptr(), 0.0, out.data_ptr(), 0, 0, st)


idx2 = idx[:, :2].contiguous()


def run2(wt):   # user and item columns only (F = 2): the gather floor
    nat.fm_score_rows_ex(idx2.data_ptr(), rows, 2, E.data_ptr(), M, 64, 0,
                         0 if wt is None else wt.data_ptr(), 0.0, out.data_ptr(), 0, 0, st)


res = {"with_w_ms": timeit(lambda: run(wbig)), "no_w_ms": timeit(lambda: run(None)),
       "ui_w_ms": timeit(lambda: run2(wbig)), "ui_only_ms": timeit(lambda: run2(None))}
print(json.dumps(res))
