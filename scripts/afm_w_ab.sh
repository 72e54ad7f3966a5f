#!/bin/bash
# AFM GPU tests (per-query A2 kernel on by default), then the A1/A2
# microbench legs with the per-query kernel (default) and afm_cat_fused
# (HHFM_AFM_CAT_W=0), alternating
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_afm.py tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/afmw_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/afmw_pytest.log; exit 1; }
tail -1 gpurun_out/afmw_pytest.log
for rnd in 1 2; do
  for v in 1 0; do
    echo -n "cat_w=$v " && HHFM_AFM_CAT_W=$v MB_ONLY=afm timeout -k 10 120 python scripts/microbench.py 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print({k: round(v['median_ms'],4) for k,v in d.items()})" || exit 1
  done
done
