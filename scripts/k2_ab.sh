#!/bin/bash
# A/B of catalog_ring settings at the C4 shape (env switches read per call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/k2ab
mkdir -p $out
for wv in 4 8; do
  HHFM_RING_WAVES=$wv timeout -k 10 200 python scripts/k2_c4.py --variants seed > $out/w$wv.json 2> $out/w$wv.err || { echo "w$wv failed"; tail $out/w$wv.err; exit 1; }
  echo "waves=$wv $(tail -1 $out/w$wv.json)"
done
