#!/bin/bash
# Round-3 validation on one MI355X: every GPU test (per-case parity record in
# gpurun_out/r03/parity_report.json), smoke(), and the bench line with every
# leg checked against the oracle.  Each GPU step is time-limited; the script
# stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${R03_OUT:-r03}
mkdir -p $out
export HHFM_PARITY_REPORT=$out/parity_report.json
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rA --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail $out/smoke.log; exit 1; }
cat $out/smoke.log
fi
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail $out/bench.err; exit 1; }
python -c "
import json,sys
d=json.load(open('$out/bench.json'))
print('value',d['value'],'ms',d['ms_per_step'],'frac',d['roofline']['frac'])
print('parity',json.dumps(d.get('parity')))
for k,v in d.get('extra',{}).items():
    print(k, {x:v.get(x) for x in ('ms_per_query_batch','ms_per_pass','kernel_ms','reference_call_300_queries_us','matches_n1')}, json.dumps(v.get('parity'))[:400], json.dumps(v.get('roofline',{}).get('frac')))
"
