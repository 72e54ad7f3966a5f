#!/bin/bash
# rocprofv3 passes: kernel trace + stats of the bench and of the kernel
# microbenchmarks, then separate PMC passes (FETCH_SIZE, WRITE_SIZE) on the
# K1 calibration workload.  Every step is time-limited; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-pmc > gpurun_out/prof/bench_under_rocprof.json 2> gpurun_out/prof/trace.err || { echo "bench trace failed"; tail gpurun_out/prof/trace.err; exit 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/mb -o mb --output-format csv -- python3 scripts/microbench.py > gpurun_out/prof/mb.json 2> gpurun_out/prof/mb.err || { echo "microbench trace failed"; tail gpurun_out/prof/mb.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o pmc --output-format csv -- python3 scripts/pmc_fm_rows.py > gpurun_out/prof/fetch.log 2>&1 || { echo "fetch pmc failed"; tail gpurun_out/prof/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o pmc --output-format csv -- python3 scripts/pmc_fm_rows.py > gpurun_out/prof/write.log 2>&1 || { echo "write pmc failed"; tail gpurun_out/prof/write.log; exit 1; }
cat gpurun_out/prof/mb.json
