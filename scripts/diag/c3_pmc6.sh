#!/bin/bash
# Round 6 diagnostic: SQ / SQC counters of the C3 fused kernel (300 queries),
# three passes, each its own rocprofv3 run.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/r06/pmc
rm -rf $out && mkdir -p $out
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" \
           "SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $out/p$i -o p --output-format csv -- python3 scripts/diag/c3_one.py ${1:-300} > /dev/null 2> $out/p$i.err || { echo "pass $i failed"; tail -3 $out/p$i.err; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob('gpurun_out/r06/pmc/p*/**/p_counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'catalog_fused' in r['Kernel_Name']:
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
print({k: round(sum(v) / len(v)) for k, v in sorted(acc.items())})
PY
