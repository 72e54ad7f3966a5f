#!/bin/bash
# round 6: C3 merge rewrite — catalog GPU tests, then event-timed C3 calls
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -m gpu -x -q --timeout 300 --timeout-method thread -k "catalog or topk or fused" > gpurun_out/r06/c3m_tests.txt 2>&1 || { tail -30 gpurun_out/r06/c3m_tests.txt; exit 1; }
tail -2 gpurun_out/r06/c3m_tests.txt
for r in 1 2; do timeout -k 10 200 python scripts/diag/c3_ab6.py || exit 1; done
