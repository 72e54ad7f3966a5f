#!/bin/bash
# C3 A/B of prebuilt libhhfm variants (ab dir ${AB_DIR:-ab}/<name>/), each from a private package copy
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/c3libs
mkdir -p $out
for d in "$@"; do
  rm -rf /tmp/c3v_$d && mkdir -p /tmp/c3v_$d && cp -r hhfm_amd /tmp/c3v_$d/ || exit 1
  cp ${AB_DIR:-ab}/$d/*.so /tmp/c3v_$d/hhfm_amd/lib/ || exit 1
  PYTHONPATH=/tmp/c3v_$d timeout -k 10 200 python scripts/diag/c3_ab.py > $out/$d.json 2> $out/$d.err || { echo "$d failed"; tail $out/$d.err; exit 1; }
  echo "$d $(tail -1 $out/$d.json)"
done
