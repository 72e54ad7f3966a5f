#!/bin/bash
# DeepFM projected layer 0: GPU tests, C5 microbench (direct vs projected),
# rocprof kernel stats of the projected C5 leg.  Every GPU step time-limited.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/dfm
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dfm.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit 1; }
tail -1 $out/pytest.log
MB_ONLY=dfm timeout -k 10 300 python scripts/microbench.py > $out/mb.json 2> $out/mb.err || { echo "mb failed"; tail $out/mb.err; exit 1; }
cat $out/mb.json
MB_ONLY=dfm MB_DFM_LEGS=dfm_c5_bf16 MB_DFM_PROJ=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 scripts/microbench.py > $out/prof.log 2>&1 || { echo "rocprof failed"; tail $out/prof.log; exit 1; }
find $out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/kernel_stats.csv
head -12 $out/kernel_stats.csv
