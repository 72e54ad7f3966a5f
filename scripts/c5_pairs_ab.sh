#!/bin/bash
# DeepFM GPU tests, then C5 bf16 and fp32 with the FM part from the pair
# table (default) against without (HHFM_DFM_FM_PAIRS=0), alternating
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dfm.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/c5p_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/c5p_pytest.log; exit 1; }
tail -1 gpurun_out/c5p_pytest.log
for rnd in 1 2; do
  for v in 1 0; do
    echo -n "bf16 pairs=$v " && HHFM_DFM_FM_PAIRS=$v timeout -k 10 120 python scripts/k3w_time.py 12500000 5 || exit 1
  done
done
