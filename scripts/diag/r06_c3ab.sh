#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "catalog" > gpurun_out/r06/c3_tests.txt 2>&1 || { tail -30 gpurun_out/r06/c3_tests.txt; exit 1; }
grep -E 'passed|failed' gpurun_out/r06/c3_tests.txt | tail -1
timeout -k 10 500 bash scripts/diag/c3_libs6.sh "$@" > gpurun_out/r06/c3ab.txt 2>&1; cat gpurun_out/r06/c3ab.txt
