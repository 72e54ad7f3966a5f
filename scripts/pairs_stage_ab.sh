#!/bin/bash
# FM pair-table pass: user rows of C staged in LDS (HHFM_DFM_PAIRS_STAGE=1)
# or gathered from the caches (default); DeepFM tests first, then C5 bf16 and
# fp32, alternating
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dfm.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pst_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pst_pytest.log; exit 1; }
tail -1 gpurun_out/pst_pytest.log
for rnd in 1 2; do
  for v in 0 1; do
    echo -n "bf16 stage=$v " && HHFM_DFM_PAIRS_STAGE=$v timeout -k 10 120 python scripts/k3w_time.py 12500000 5 || exit 1
    echo -n "f32 stage=$v " && HHFM_DFM_PAIRS_STAGE=$v K3W_F32=1 timeout -k 10 120 python scripts/k3w_time.py 12500000 3 || exit 1
  done
done
