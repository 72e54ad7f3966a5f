#!/bin/bash
# C5 fp32 leg: the staged FM-part pre-kernel (default) against the
# grid-stride one (HHFM_DFM_FMB_STAGE=0), alternating; parity tests first
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dfm.py -x -q -k "f32_split or projected or shapes" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fmb_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/fmb_pytest.log; exit 1; }
tail -1 gpurun_out/fmb_pytest.log
for rnd in 1 2; do
  for v in 1 0; do
    echo -n "stage=$v " && HHFM_DFM_FMB_STAGE=$v K3W_F32=1 timeout -k 10 120 python scripts/k3w_time.py 12500000 3 || exit 1
  done
done
