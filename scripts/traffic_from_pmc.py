#!/usr/bin/env python3
"""Turn the FETCH_SIZE / WRITE_SIZE passes of scripts/pmc_fm_rows.py into
profiles/traffic_fm_rows.json (HBM bytes per row of K1, calibrated).

The six fm_rows_fast dispatches are, in order: calib x2, bench x2,
bench-without-w x2 (see scripts/pmc_fm_rows.py).  FETCH_SIZE on gfx950
under-counts wide reads (MI355X_MICROARCH.md §HBM); the calib launch streams
a known byte count and gives the correction factor, applied to the others.

usage: python scripts/traffic_from_pmc.py gpurun_out/prof [profiles/traffic_fm_rows.json]
"""
import csv
import json
import os
import sys

ROWS = 1 << 23
K = 64
N_HALF = 8 << 20


def counters(path):
    vals = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "fm_rows_fast" in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    if len(vals) != 6:
        raise SystemExit(f"{path}: expected 6 fm_rows_fast dispatches, got {len(vals)}")
    return vals


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
        "traffic_fm_rows.json")
    fetch = counters(os.path.join(d, "fetch", "pmc_counter_collection.csv"))
    write = counters(os.path.join(d, "write", "pmc_counter_collection.csv"))
    # calib: user and item halves streamed once (rows r -> user r, item n_user+r),
    # 5 ids, w of user+item streamed, 3 ctx rows + their w cache-resident
    known = ROWS * (2 * K * 4 + 5 * 4 + 2 * 4)
    calib_fetch = 1024.0 * (fetch[0] + fetch[1]) / 2
    factor = known / calib_fetch

    def per_row(kb_a, kb_b):
        return 1024.0 * (kb_a + kb_b) / 2 * factor / ROWS

    def per_row_w(kb_a, kb_b):   # WRITE_SIZE is not corrected (no 2x under-count)
        return 1024.0 * (kb_a + kb_b) / 2 / ROWS

    rd, wr = per_row(fetch[2], fetch[3]), per_row_w(write[2], write[3])
    rd_now, wr_now = per_row(fetch[4], fetch[5]), per_row_w(write[4], write[5])
    res = {
        "kernel": "fm_rows_fast<5,16,f32,w> (K1, hhfm_fm_score_rows)",
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) on "
                  "scripts/pmc_fm_rows.py, gfx950; scripts/traffic_from_pmc.py",
        "pmc_rows": ROWS,
        "fetch_size_kb": fetch,
        "write_size_kb": write,
        "calibration": {
            "known_bytes_per_launch": known,
            "fetch_size_bytes": calib_fetch,
            "factor": factor,
            "note": "sequential user/item ids stream each table row once; FETCH_SIZE "
                    "reads 1/factor of the known bytes (MI355X_MICROARCH.md §HBM: gfx950 "
                    "counts 128-B requests as 64 B)",
        },
        "hbm_read_bytes_per_row": rd,
        "hbm_write_bytes_per_row": wr,
        "hbm_bytes_per_row": rd + wr,
        "no_w_hbm_bytes_per_row": rd_now + wr_now,
        "w_gather_bytes_per_row": rd - rd_now,
        "compulsory_bytes_per_row": 2 * K * 4 + 5 * 4 + 2 * 4 + 4,
        "k": K,
        "fields": 5,
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if "bytes_per_row" in k}, indent=1))


if __name__ == "__main__":
    main()
