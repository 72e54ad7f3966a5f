#!/bin/bash
# wide ITEM DeepFM kernel: parity tests, then the C5 forward timed for each
# library variant given (scripts/build_variants.sh into abw/<name>/)
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/k3w
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dfm.py -x -q -k "wide or item or projected" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
[ $# -gt 0 ] && K3W_ROWS=${K3W_ROWS:-12500000} bash scripts/k3w_ko.sh "$@"
exit 0
