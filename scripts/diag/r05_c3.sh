#!/bin/bash
# C3 fused-kernel A/B: catalog/model GPU tests, timing, kernel trace
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_c3_tests.txt 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/r05_c3_tests.txt
timeout -k 10 120 python scripts/diag/c3_fused_ab.py > gpurun_out/r05_c3_ab.json 2> gpurun_out/r05_c3_ab.err || { echo "c3 ab failed"; tail -20 gpurun_out/r05_c3_ab.err; exit 1; }
cat gpurun_out/r05_c3_ab.json
rm -rf gpurun_out/r05_c3prof
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_c3prof -o c3 --output-format csv -- python scripts/diag/c3_fused_ab.py > /dev/null 2> gpurun_out/r05_c3prof.err || { echo "rocprof failed"; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r05_c3prof/**/c3_kernel_stats.csv', recursive=True) + glob.glob('gpurun_out/r05_c3prof/c3_kernel_stats.csv')
for r in csv.DictReader(open(f[0])):
    if 'hhfm' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:8.2f} us x{r['Calls']:>4} {r['Name'][:100]}")
PY
