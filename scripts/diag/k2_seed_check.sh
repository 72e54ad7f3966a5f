#!/bin/bash
# K2 seed change check: C4-shape timing (seed / noseed / noring, checksums),
# kernel trace of the seeded call, then the catalog / AFM / DeepFM top-K tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
d=gpurun_out/k2seed2
mkdir -p $d
timeout -k 10 200 python scripts/k2_c4.py --variants seed,noseed,noring > $d/c4.json 2>&1 || { tail $d/c4.json; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d/kt -o kt --output-format csv -- python3 scripts/k2_c4.py --reps 10 --variants seed > $d/kt.log 2>&1 || { tail $d/kt.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_afm.py tests/test_gpu_dfm.py tests/test_gpu_models.py -k "catalog or topk or afm or seed" > $d/tests.txt 2>&1 || { tail -20 $d/tests.txt; exit 1; }
tail -2 $d/tests.txt
tail -1 $d/c4.json
