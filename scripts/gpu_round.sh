#!/bin/bash
# One gpurun session: GPU parity tests, then a short bench. Stops on a crash
# (rc other than 0 = pass / 1 = test failures).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest $TESTS -q -m gpu -p no:cacheprovider > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ -n "$NO_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --cpu-seconds 5} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
echo "bench rc=$brc"; cat gpurun_out/bench.json; tail -20 gpurun_out/bench.err
exit $brc
