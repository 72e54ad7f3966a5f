#!/bin/bash
# Diagnostic: SQ counters of the fused C3 kernel (one pass, 8 SQ counters)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c3pmc
for B in 3000 300; do
  rm -rf gpurun_out/c3pmc/b$B
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/c3pmc/b$B -o p --output-format csv -- python scripts/diag/c3_one.py $B > /dev/null 2> gpurun_out/c3pmc/b$B.err || { echo "pmc $B failed"; tail -5 gpurun_out/c3pmc/b$B.err; exit 1; }
  python3 - $B <<'PY'
import csv, glob, sys, collections
f = glob.glob(f'gpurun_out/c3pmc/b{sys.argv[1]}/**/p_counter_collection.csv', recursive=True)
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    if 'catalog_fused' in r['Kernel_Name']:
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
print(sys.argv[1], {k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
done
