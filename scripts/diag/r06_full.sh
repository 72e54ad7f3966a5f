#!/bin/bash
# round 6 checkpoint: the whole GPU suite, then the default bench line
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/pytest_gpu.txt 2>&1
rc=$?
grep -E 'passed|failed|error' gpurun_out/r06/pytest_gpu.txt | tail -3
[ $rc -ne 0 ] && { tail -40 gpurun_out/r06/pytest_gpu.txt; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/r06/bench.json 2> gpurun_out/r06/bench.err || { tail -20 gpurun_out/r06/bench.err; exit 1; }
tail -c 3000 gpurun_out/r06/bench.json
