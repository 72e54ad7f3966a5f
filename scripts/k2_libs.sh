#!/bin/bash
# A/B of prebuilt libhhfm variants (ab/<name>/, scripts/build_variants.sh) at the C4 shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/k2libs
mkdir -p $out
for d in "$@"; do
  cp ${AB_DIR:-ab}/$d/*.so hhfm_amd/lib/ || exit 1
  timeout -k 10 200 python scripts/k2_c4.py --variants seed,noring > $out/$d.json 2> $out/$d.err || { echo "$d failed"; tail $out/$d.err; exit 1; }
  echo "$d $(tail -1 $out/$d.json)"
done
