#!/bin/bash
# Diagnostic: GPU kernel time per C3 call, fused (default) vs HHFM_PLAN_STORE,
# at 3,000 and 300 queries (kernel trace of 50 calls each)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c3paths
# CASES: "B:plan ..." (plan 16384 = HHFM_PLAN_FUSED, 8192 = HHFM_PLAN_STORE)
for case in ${CASES:-3000:0 3000:8192 300:16384 300:8192}; do
  B=${case%%:*}; plan=${case##*:}
  for once in 1; do
    rm -rf gpurun_out/c3paths/b${B}_p$plan
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c3paths/b${B}_p$plan -o k --output-format csv -- python scripts/diag/c3_one.py $B $plan > /dev/null 2> gpurun_out/c3paths/b${B}_p$plan.err || { echo "failed"; tail -3 gpurun_out/c3paths/b${B}_p$plan.err; exit 1; }
    python3 - $B $plan <<'PY'
import csv, glob, sys
f = glob.glob(f'gpurun_out/c3paths/b{sys.argv[1]}_p{sys.argv[2]}/**/k_kernel_stats.csv', recursive=True)
tot = 0.0
parts = []
for r in csv.DictReader(open(f[0])):
    if 'hhfm' in r['Name'] and 'check' not in r['Name']:
        per = float(r['TotalDurationNs']) / 50 / 1e3
        tot += per
        parts.append(f"{r['Name'].split('(')[0].split('::')[-1][:28]} {per:.1f}")
print(f"B={sys.argv[1]} plan={sys.argv[2]}: {tot:.1f} us/call  [{'; '.join(parts)}]")
PY
  done
done
