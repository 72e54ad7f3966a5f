#!/bin/bash
# Diagnostic: instruction-cache counters of the fused C3 kernel
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c3ic
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/c3ic/avail.txt 2>&1
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*" gpurun_out/c3ic/avail.txt | sort -u | head -20
rm -rf gpurun_out/c3ic/p
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES -d gpurun_out/c3ic/p -o p --output-format csv -- python scripts/diag/c3_one.py 300 > /dev/null 2> gpurun_out/c3ic/p.err || { echo "pmc failed"; tail -5 gpurun_out/c3ic/p.err; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/c3ic/p/**/p_counter_collection.csv', recursive=True)
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    if 'catalog_fused' in r['Kernel_Name']:
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
print({k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
