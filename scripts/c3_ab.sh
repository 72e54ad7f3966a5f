#!/bin/bash
# C3 small-catalog path: kernel tests, then the bench C3 leg (3,000 queries and
# the reference's 300-query call) with the query launch fused (default) and not.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/c3
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c3/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/c3/pytest.log; exit 1; }
tail -1 gpurun_out/c3/pytest.log
for f in 1 0; do
HHFM_CATALOG_FUSE_Q=$f timeout -k 10 300 python bench.py --legs c3 --cpu-seconds 0 --steps 2 --warmup 1 --rows 1048576 > gpurun_out/c3/b$f.json 2> gpurun_out/c3/b$f.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/c3/b$f.json'))['extra']['catalog_c3']
print('fuse=$f', round(d['ms_per_query_batch']*1e3,1), 'us/3000q', round(d['reference_call_300_queries_us'],1), 'us/300q', d['parity']['parity'])"
done
