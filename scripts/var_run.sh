#!/bin/bash
# Diagnostic A/B: run one command against prebuilt libhhfm variants
# (AB_DIR/<name>/ from scripts/build_variants.sh), one process per variant,
# in the order given; the shipped library is restored at the end.
#   AB_DIR=abdfm bash scripts/var_run.sh "python scripts/k3w_time.py 12500000 5" v1 v2 v1 v2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cmd=$1; shift
mkdir -p gpurun_out/.shipped && cp hhfm_amd/lib/*.so gpurun_out/.shipped/
for d in "$@"; do
  cp ${AB_DIR:-ab}/$d/*.so hhfm_amd/lib/ || exit 1
  r=$(timeout -k 10 300 $cmd 2>/dev/null | tail -1) || { echo "$d failed"; cp gpurun_out/.shipped/*.so hhfm_amd/lib/; exit 1; }
  echo "$d $r"
done
cp gpurun_out/.shipped/*.so hhfm_amd/lib/ && rm -rf gpurun_out/.shipped
