#!/bin/bash
# kernel trace of the AFM microbench legs (A1 rows, A2 300-query catalog)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/afmt
mkdir -p $o
MB_ONLY=afm timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o -o afm --output-format csv -- python3 scripts/microbench.py > $o/mb.json 2> $o/err.log || { tail $o/err.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/afmt/afm_kernel_stats.csv')):
    if 'hhfm' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:9.2f} us x{r['Calls']:>4} {r['Name'][:100]}")
PY
