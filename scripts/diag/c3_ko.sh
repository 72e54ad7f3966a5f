#!/bin/bash
# Diagnostic: kernel durations of the fused C3 kernel under knock-out builds
# (abc/ko*/; each in a private copy of the package), kernel trace per build.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c3ko
for d in base abc/ko1 abc/ko2 abc/ko4; do
  n=$(basename $d)
  rm -rf /tmp/c3_$n && mkdir -p /tmp/c3_$n && cp -r hhfm_amd /tmp/c3_$n/ || exit 1
  [ "$d" != base ] && { cp $d/*.so /tmp/c3_$n/hhfm_amd/lib/ || exit 1; }
  rm -rf gpurun_out/c3ko/$n
  PYTHONPATH=/tmp/c3_$n timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c3ko/$n -o k --output-format csv -- python scripts/diag/c3_fused_ab.py > gpurun_out/c3ko/$n.json 2> gpurun_out/c3ko/$n.err || { echo "$n failed"; tail -5 gpurun_out/c3ko/$n.err; exit 1; }
  echo "== $n"
  python3 - "$n" <<'PY'
import csv, glob, sys
f = glob.glob(f'gpurun_out/c3ko/{sys.argv[1]}/**/k_kernel_stats.csv', recursive=True)
for r in csv.DictReader(open(f[0])):
    if 'catalog_fused' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:8.2f} us x{r['Calls']:>4} {r['Name'][:60]}")
PY
done
