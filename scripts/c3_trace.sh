#!/bin/bash
# kernel trace of the C3 call (scripts/c3_trace.py): per-kernel durations
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/c3t
mkdir -p $o
timeout -k 10 120 python3 scripts/c3_trace.py > $o/plain.json 2> $o/plain.err || { tail $o/plain.err; exit 1; }
cat $o/plain.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o -o c3 --output-format csv -- python3 scripts/c3_trace.py > $o/prof.json 2> $o/prof.err || { tail $o/prof.err; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/c3t/c3_kernel_stats.csv')):
    if 'hhfm' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:8.2f} us x{r['Calls']:>4} {r['Name'][:110]}")
PY
