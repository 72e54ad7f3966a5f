#!/bin/bash
# K2 iteration on one MI355X: the catalog parity tests, then C4-shape timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/k2
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_bench.py -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider -k "catalog or sharded or topk or c4 or bench" > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python scripts/k2_c4.py ${K2_ARGS:---variants seed,seed_noring,noseed_noring} > $out/c4.json 2> $out/c4.err || { echo "k2_c4 failed"; tail $out/c4.err; exit 1; }
tail -1 $out/c4.json
