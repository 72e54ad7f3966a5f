#!/bin/bash
# Diagnostic: K1 at configs[1] across library builds (base = the shipped
# tree, then abv/<name> variants), each in its own process, alternating twice.
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
for d in base "$@"; do
  n=$(basename $d)
  rm -rf /tmp/k1_$n && mkdir -p /tmp/k1_$n && cp -r hhfm_amd /tmp/k1_$n/ || exit 1
  [ "$d" != base ] && { cp abv/$d/*.so /tmp/k1_$n/hhfm_amd/lib/ || exit 1; }
  r=$(PYTHONPATH=/tmp/k1_$n timeout -k 10 200 python scripts/diag/k1_wmap.py 2>/tmp/k1_$n.err) || { tail -5 /tmp/k1_$n.err; exit 1; }; echo "== $n $r"
done
done
