#!/bin/bash
# Round 6: C3 fused kernel (one workgroup per 32 queries over the whole
# catalog) — catalog GPU tests, host/event call times, phase cycles (timing
# build abv/c3t), rocprofv3 kernel trace of the 300- and 3,000-query calls.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r06
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "catalog" > $out/c3_tests.txt 2>&1 || { tail -30 $out/c3_tests.txt; exit 1; }
tail -3 $out/c3_tests.txt
timeout -k 10 200 python scripts/diag/c3_host.py > $out/c3host2.json 2> $out/c3host2.err || { tail -5 $out/c3host2.err; exit 1; }
cat $out/c3host2.json
rm -rf /tmp/c3t && mkdir -p /tmp/c3t && cp -r hhfm_amd /tmp/c3t/ && cp abv/c3t/*.so /tmp/c3t/hhfm_amd/lib/ || exit 1
PYTHONPATH=/tmp/c3t timeout -k 10 200 python scripts/diag/c3_phases.py > $out/c3phases.json 2> $out/c3phases.err || { tail -5 $out/c3phases.err; exit 1; }
cat $out/c3phases.json
