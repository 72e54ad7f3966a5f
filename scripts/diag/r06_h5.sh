#!/bin/bash
# round 6: H5 sampler kernel trace at the row-table shape (86,583 rows x 50)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/h5
timeout -k 10 600 python -u -m pytest tests/test_gpu_harness.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/h5/pytest.txt 2>&1 || { tail -30 gpurun_out/r06/h5/pytest.txt; exit 1; }
tail -2 gpurun_out/r06/h5/pytest.txt
export ROWS_ONLY=h35
timeout -k 10 300 python3 scripts/rowtable.py > gpurun_out/r06/h5/rows.json 2> gpurun_out/r06/h5/rows.err || { tail -20 gpurun_out/r06/h5/rows.err; exit 1; }
tail -c 600 gpurun_out/r06/h5/rows.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/h5/kt -o h5 -- python3 scripts/rowtable.py > gpurun_out/r06/h5/kt.log 2>&1 || { tail -20 gpurun_out/r06/h5/kt.log; exit 1; }
find gpurun_out/r06/h5/kt -name '*kernel_stats.csv' | head -1 | xargs head -20
