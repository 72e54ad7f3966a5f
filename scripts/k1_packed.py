#!/usr/bin/env python3
"""K1 packed-row experiment on the bench workload (configs[1], HBM-roofline
variant): the table as [E | w | pad] rows at a 272-B or 384-B stride (w read
from the row's third 128-B line) against the default separate `w` array.
Times each variant with HIP events, alternating, and checks the outputs are
bit-identical to the default kernel's."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from hhfm_amd._native import native  # noqa: E402


def main():
    rows = int(os.environ.get("K1_ROWS", 1 << 25))
    reps = int(os.environ.get("K1_REPS", 10))
    dev = torch.device("cuda", 0)
    idx, E, w, M = bench.make_batch(rows, 8 << 20, 8 << 20, 64, 1, dev)
    st = torch.cuda.current_stream().cuda_stream
    tabs = {}
    for sel, stride in ((1, 272), (2, 384)):
        P = torch.zeros(M, stride // 4, dtype=torch.float32, device=dev)
        P[:, :64] = E
        P[:, 64] = w
        tabs[sel] = P
        torch.cuda.synchronize()
    outs = {v: torch.empty(rows, device=dev) for v in (0, 1, 2)}

    def run(v):
        T = E if v == 0 else tabs[v]
        native().fm_score_rows_ex(idx.data_ptr(), rows, 5, T.data_ptr(), M, 64, 0,
                                  w.data_ptr(), 0.0, outs[v].data_ptr(), v << 8, 0, st)
    for v in outs:
        run(v)
    torch.cuda.synchronize()
    ts = {v: [] for v in outs}
    for _ in range(reps):
        for v in outs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(v)
            e1.record()
            e1.synchronize()
            ts[v].append(e0.elapsed_time(e1))
    names = {0: "separate w (default)", 1: "packed 272-B rows", 2: "packed 384-B rows"}
    res = {names[v]: {"ms_median": float(np.median(ts[v])), "ms_min": float(min(ts[v])),
                      "bit_identical": bool(torch.equal(outs[v], outs[0])),
                      "frac_544B": 544 * rows / (np.median(ts[v]) * 1e-3) / 8e12}
           for v in outs}
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
