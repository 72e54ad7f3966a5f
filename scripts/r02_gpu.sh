#!/bin/bash
# Round-2 validation on one MI355X: GPU tests, smoke, the bench line, the
# K1 w-policy PMC passes.  Every GPU step is time-limited; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r02
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider -rA > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest.log | head -20; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail $out/smoke.log; exit 1; }
cat $out/smoke.log
timeout -k 10 500 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail $out/bench.err; exit 1; }
cat $out/bench.json
