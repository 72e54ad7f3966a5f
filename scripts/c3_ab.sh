#!/bin/bash
# catalog parity tests, then the C3 call timed with each library variant
# (scripts/build_variants.sh into abw/<name>/), alternating twice
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c3ab_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/c3ab_pytest.log; exit 1; }
tail -1 gpurun_out/c3ab_pytest.log
for rnd in 1 2; do
for d in "$@"; do
  cp $d/*.so hhfm_amd/lib/ && echo -n "$d " && timeout -k 10 120 python scripts/c3_trace.py 2>/dev/null || exit 1
done
done
