#!/bin/bash
# AFM GPU tests with the current library, then the A1/A2 microbench legs for
# each library variant given (abw/<name>/), alternating twice
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_afm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/afml_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/afml_pytest.log; exit 1; }
tail -1 gpurun_out/afml_pytest.log
for rnd in 1 2; do
  for d in "$@"; do
    cp $d/*.so hhfm_amd/lib/ && echo -n "$d " && MB_ONLY=afm timeout -k 10 120 python scripts/microbench.py 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print({k: round(v['median_ms'],4) for k,v in d.items()})" || exit 1
  done
done
