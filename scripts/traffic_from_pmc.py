#!/usr/bin/env python3
"""Turn the FETCH_SIZE / WRITE_SIZE passes of scripts/pmc_fm_rows.py into
profiles/traffic_fm_rows.json (HBM bytes per row of K1, calibrated).

The six fm_rows_fast dispatches are, in order: calib x2, bench x2,
bench-without-w x2 (see scripts/pmc_fm_rows.py).  FETCH_SIZE on gfx950
under-counts wide reads (MI355X_MICROARCH.md §HBM); the calib launch streams
a known byte count and gives the correction factor, applied to the others.

usage: python scripts/traffic_from_pmc.py gpurun_out/prof [profiles/traffic_fm_rows.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

ROWS = 1 << 23
K = 64


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles",
                                                            "traffic_fm_rows.json")
    rows = int(os.environ.get("PMC_ROWS", ROWS))
    fetch = bench._pmc_column(os.path.join(d, "fetch", "pmc_counter_collection.csv"))
    write = bench._pmc_column(os.path.join(d, "write", "pmc_counter_collection.csv"))
    res = {"kernel": "fm_rows_fast<5,16,f32,w> (K1, hhfm_fm_score_rows)",
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) on "
                     "scripts/pmc_fm_rows.py, gfx950; scripts/traffic_from_pmc.py"}
    res.update(bench.pmc_bytes_per_row(fetch, write, rows, K))
    res.update({"compulsory_bytes_per_row": 2 * K * 4 + 5 * 4 + 2 * 4 + 4, "k": K, "fields": 5})
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if "bytes_per_row" in k}, indent=1))


if __name__ == "__main__":
    main()
