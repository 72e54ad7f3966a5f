#!/bin/bash
# round 6: AFM A1 with per-wave staging of narrow-span fields — AFM GPU tests, then the row table's A1/A2 legs
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/afm
timeout -k 10 600 python -u -m pytest tests/test_gpu_afm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/afm/pytest.txt 2>&1 || { tail -40 gpurun_out/r06/afm/pytest.txt; exit 1; }
tail -2 gpurun_out/r06/afm/pytest.txt
ROWS_ONLY=afm timeout -k 10 300 python3 scripts/rowtable.py > gpurun_out/r06/afm/rows.json 2> gpurun_out/r06/afm/rows.err || { tail -20 gpurun_out/r06/afm/rows.err; exit 1; }
grep -E '"gpu_ms"|"frac"' gpurun_out/r06/afm/rows.json
