#!/bin/bash
# Round-end style validation on one MI355X: every GPU test, smoke(), the
# bench line, the rocprofv3 passes (scripts/gpu_profile.sh) and the per-row
# table (scripts/rowtable.py, one leg per process so progress stays visible).
# Every GPU step is time-limited; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/full
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail $out/smoke.log; exit 1; }
cat $out/smoke.log
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail $out/bench.err; exit 1; }
cat $out/bench.json
bash scripts/gpu_profile.sh > $out/profile.log 2>&1 || { echo "profile failed"; tail $out/profile.log; exit 1; }
echo "profiles done"
for leg in ${ROW_LEGS:-c2 c3 c4 c5 afm h6 h35}; do
  ROWS_ONLY=$leg timeout -k 10 400 python scripts/rowtable.py > $out/rows_$leg.json 2> $out/rows_$leg.err || { echo "rowtable $leg failed"; tail $out/rows_$leg.err; exit 1; }
  echo "rows $leg done"
done
