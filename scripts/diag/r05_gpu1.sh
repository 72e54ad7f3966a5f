#!/bin/bash
# round-5 GPU step: full GPU suite, C3 fused A/B (timing + kernel trace), H5 row
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_pytest_gpu.txt 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/r05_pytest_gpu.txt
timeout -k 10 120 python scripts/diag/c3_fused_ab.py > gpurun_out/r05_c3_ab.json 2> gpurun_out/r05_c3_ab.err || { echo "c3 ab failed"; tail -20 gpurun_out/r05_c3_ab.err; exit 1; }
cat gpurun_out/r05_c3_ab.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_c3prof -o c3 -- python scripts/diag/c3_fused_ab.py > /dev/null 2> gpurun_out/r05_c3prof.err || { echo "rocprof failed"; exit 1; }
ROWS_ONLY=h35 timeout -k 10 300 python scripts/rowtable.py > gpurun_out/r05_rows_h5.json 2> gpurun_out/r05_rows_h5.err; echo "rows rc=$?"
cat gpurun_out/r05_rows_h5.json
