#!/bin/bash
# A/B of prebuilt libhhfm variants (AB_DIR/<name>/, scripts/build_variants.sh afm ...)
# on AFM A1 rows (scripts/afm_rows_ab.py), one process per variant; the
# shipped library is restored at the end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/afmlibs
mkdir -p $out gpurun_out/.shipped && cp hhfm_amd/lib/*.so gpurun_out/.shipped/
restore() { cp gpurun_out/.shipped/*.so hhfm_amd/lib/ && rm -rf gpurun_out/.shipped; }
for d in "$@"; do
  cp ${AB_DIR:-ab}/$d/*.so hhfm_amd/lib/ || { restore; exit 1; }
  timeout -k 10 200 python scripts/afm_rows_ab.py 5 > $out/$d.json 2> $out/$d.err || { echo "$d failed"; tail $out/$d.err; restore; exit 1; }
  echo "$d $(tail -1 $out/$d.json)"
done
restore
