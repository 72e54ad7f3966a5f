#!/bin/bash
# wide ITEM DeepFM kernel: parity tests, then the C5 A/B against the 128-row kernel
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/k3w
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dfm.py -x -q -k "wide or item or projected" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python scripts/c5_wide_ab.py 12500000 3 > $out/ab.json 2> $out/ab.err || { tail $out/ab.err; exit 1; }
cat $out/ab.json
