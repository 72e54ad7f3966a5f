#!/bin/bash
# Round-6 final evidence in one GPU call: GPU tests (+ parity report), smoke,
# the full bench, the bench under rocprofv3 --kernel-trace --stats (and the
# timed launches' own statistics, scripts/timed_stats.py), a kernel trace of
# the C3 calls (300 / 3,000 queries, scripts/diag/c3_ab6.py), the row table.
# Every step time-limited; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/r06f
mkdir -p $o
HHFM_PARITY_REPORT=$o/parity_report.json timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $o/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 $o/pytest_gpu.txt; exit 1; }
tail -2 $o/pytest_gpu.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.txt 2>&1 || { echo "smoke failed"; tail $o/smoke.txt; exit 1; }
timeout -k 10 500 python bench.py > $o/bench_full.json 2> $o/bench_full.err || { echo "bench failed"; tail $o/bench_full.err; exit 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $o/trace -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-pmc > $o/bench_under_rocprof.json 2> $o/trace.err || { echo "trace failed"; tail $o/trace.err; exit 1; }
python3 scripts/timed_stats.py $(find $o/trace -name 'bench_kernel_trace.csv' | head -1) 3 20 $o/bench_kernel_stats_timed.csv || { echo "timed stats failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/c3 -o c3 --output-format csv -- python3 scripts/diag/c3_ab6.py > $o/c3_ab6.json 2> $o/c3.err || { echo "c3 trace failed"; tail $o/c3.err; exit 1; }
timeout -k 10 600 python scripts/rowtable.py > $o/rows.json 2> $o/rows.err || { echo "rowtable failed"; tail $o/rows.err; exit 1; }
echo done
