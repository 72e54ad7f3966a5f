#!/bin/bash
# C5 fp32 leg: the FM part from the pair table (default) against the
# row-reading pre-kernel (HHFM_DFM_FM_PAIRS=0), alternating; parity tests first
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dfm.py -x -q -k "f32_split or projected or shapes or envelope or catalog" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pairs_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pairs_pytest.log; exit 1; }
tail -1 gpurun_out/pairs_pytest.log
for rnd in 1 2; do
  for v in 1 0; do
    echo -n "pairs=$v " && HHFM_DFM_FM_PAIRS=$v K3W_F32=1 timeout -k 10 120 python scripts/k3w_time.py 12500000 3 || exit 1
  done
done
