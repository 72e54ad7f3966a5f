#!/bin/bash
# Parity tests of the catalog / dense top-K paths, then a kernel trace of the
# K2 microbenchmarks (C3, C4 shard).  Every GPU step time-limited; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c3
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_dfm.py tests/test_gpu_afm.py tests/test_gpu_models.py} -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c3/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/c3/pytest.log; exit 1; }
tail -2 gpurun_out/c3/pytest.log
MB_ONLY=${MB_ONLY:-k2} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c3 -o c3 --output-format csv -- python3 scripts/microbench.py > gpurun_out/c3/mb.json 2> gpurun_out/c3/err.log || { echo "microbench failed"; tail gpurun_out/c3/err.log; exit 1; }
cat gpurun_out/c3/mb.json
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/c3/c3_kernel_stats.csv')):
    if 'hhfm' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4} {r['Name'][:90]}")
PY
