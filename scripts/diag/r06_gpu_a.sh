#!/bin/bash
# round 6: C3 phases + PMC, K1 id-load A/B
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06
timeout -k 10 400 bash scripts/diag/k1_ab.sh k1old k1u6 > gpurun_out/r06/k1ab.txt 2>&1; cat gpurun_out/r06/k1ab.txt
bash scripts/diag/r06_c3b.sh
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multirank.py > gpurun_out/r06/multirank.txt 2>&1; tail -5 gpurun_out/r06/multirank.txt
