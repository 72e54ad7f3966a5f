#!/bin/bash
# Diagnostic (round 6): K1 at configs[1] — shipped kernel, the same kernel
# with the three context rows not loaded (ids and w kept: -DHHFM_K1_CTXKO=1),
# and the user+item-only kernel (F = 2, with and without w) — one box, one
# process per build (scripts/diag/k1_wmap.py).
cd "${GRAFT_REPO_ROOT:-.}"
for d in base abv/ctxko; do
  n=$(basename $d)
  rm -rf /tmp/k1_$n && mkdir -p /tmp/k1_$n && cp -r hhfm_amd /tmp/k1_$n/ || exit 1
  [ "$d" != base ] && { cp $d/*.so /tmp/k1_$n/hhfm_amd/lib/ || exit 1; }
  r=$(PYTHONPATH=/tmp/k1_$n timeout -k 10 200 python scripts/diag/k1_wmap.py 2>/tmp/k1_$n.err) || { tail -5 /tmp/k1_$n.err; exit 1; }; echo "== $n $r"
done
