#!/bin/bash
# A/B of prebuilt libhhfm variants (AB_DIR/<name>/, scripts/build_variants.sh afm ...)
# on AFM A1 rows (scripts/afm_rows_ab.py), one process per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/afmlibs
mkdir -p $out
for d in "$@"; do
  cp ${AB_DIR:-ab}/$d/*.so hhfm_amd/lib/ || exit 1
  timeout -k 10 200 python scripts/afm_rows_ab.py 5 > $out/$d.json 2> $out/$d.err || { echo "$d failed"; tail $out/$d.err; exit 1; }
  echo "$d $(tail -1 $out/$d.json)"
done
