#!/usr/bin/env python3
"""K1 `w`-gather cache-policy variants on the bench workload (configs[1],
HBM-roofline variant): time each with HIP events and check the outputs are
bit-identical to the default kernel.  Run under rocprofv3 --pmc for the
per-variant HBM bytes (each variant is its own template instance, so the
kernel names tell them apart).

usage: python scripts/k1_wpolicy.py [--reps N]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from hhfm_amd._native import native  # noqa: E402

AUX = {0: "global (default)", 1: "buffer", 2: "buffer sc0", 3: "buffer nt", 4: "buffer sc0 nt",
       5: "buffer sc1", 6: "buffer sc0 sc1", 7: "buffer sc1 nt", 8: "buffer sc0 sc1 nt",
       -1: "table+ids+out nt (HHFM_FLAG_STREAM_TABLE), w default"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--rows", type=int, default=1 << 25)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    idx, E, w, M = bench.make_batch(a.rows, 8 << 20, 8 << 20, 64, 1, dev)
    st = torch.cuda.current_stream().cuda_stream
    ref = None
    res = {}
    for sel, name in AUX.items():
        out = torch.empty(a.rows, device=dev)

        def run():
            native().fm_score_rows_ex(idx.data_ptr(), a.rows, 5, E.data_ptr(), M, 64, 0,
                                           w.data_ptr(), 0.0, out.data_ptr(),
                                      1 if sel < 0 else sel << 4, 0, st)
        run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        if ref is None:
            ref = out.clone()
        res[name] = {"sel": sel, "ms_median": float(np.median(ts)), "ms_min": float(min(ts)),
                     "bit_identical": bool(torch.equal(out, ref))}
        print(json.dumps({name: res[name]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
