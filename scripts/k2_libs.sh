#!/bin/bash
# A/B of prebuilt libhhfm variants (ab/<name>/, scripts/build_variants.sh) at the C4 shape.
# Each variant runs from a private copy of the package (hhfm_amd/lib is never
# overwritten, so no variant can be left installed).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/k2libs
mkdir -p $out
for d in "$@"; do
  rm -rf /tmp/k2v_$d && mkdir -p /tmp/k2v_$d && cp -r hhfm_amd /tmp/k2v_$d/ || exit 1
  cp ${AB_DIR:-ab}/$d/*.so /tmp/k2v_$d/hhfm_amd/lib/ || exit 1
  PYTHONPATH=/tmp/k2v_$d timeout -k 10 200 python scripts/k2_c4.py --variants ${VARIANTS:-seed,noring} > $out/$d.json 2> $out/$d.err || { echo "$d failed"; tail $out/$d.err; exit 1; }
  echo "$d $(tail -1 $out/$d.json)"
done
