#!/bin/bash
# Round 6: C3 fused kernel — catalog GPU tests, host/event call times, phase
# cycles (timing build abv/c3t), rocprofv3 kernel trace of 300/3,000 queries.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r06
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "catalog" > $out/c3_tests.txt 2>&1 || { tail -30 $out/c3_tests.txt; exit 1; }
tail -2 $out/c3_tests.txt
timeout -k 10 200 python scripts/diag/c3_host.py > $out/c3host.json 2> $out/c3host.err || { tail -5 $out/c3host.err; exit 1; }
cat $out/c3host.json
rm -rf /tmp/c3t && mkdir -p /tmp/c3t && cp -r hhfm_amd /tmp/c3t/ && cp abv/c3t/*.so /tmp/c3t/hhfm_amd/lib/ || exit 1
PYTHONPATH=/tmp/c3t timeout -k 10 200 python scripts/diag/c3_phases.py > $out/c3phases.json 2> $out/c3phases.err || { tail -5 $out/c3phases.err; exit 1; }
cat $out/c3phases.json
for b in 300 3000; do
  rm -rf $out/kt$b
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/kt$b -o kt --output-format csv -- python3 scripts/diag/c3_one.py $b > /dev/null 2> $out/kt$b.err || { tail -3 $out/kt$b.err; exit 1; }
  f=$(find $out/kt$b -name 'kt_kernel_stats.csv' | head -1); echo "== B=$b"; cut -d, -f1-8 $f | head -5
done
