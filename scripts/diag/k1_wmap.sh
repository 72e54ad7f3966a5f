#!/bin/bash
# Diagnostic: K1 time with w as shipped, folded into 1 MB, or one line per gather
cd "${GRAFT_REPO_ROOT:-.}"
for d in base abk1w/m1 abk1w/m2; do
  n=$(basename $d)
  rm -rf /tmp/k1_$n && mkdir -p /tmp/k1_$n && cp -r hhfm_amd /tmp/k1_$n/ || exit 1
  [ "$d" != base ] && { cp $d/*.so /tmp/k1_$n/hhfm_amd/lib/ || exit 1; }
  r=$(PYTHONPATH=/tmp/k1_$n timeout -k 10 200 python scripts/diag/k1_wmap.py 2>/tmp/k1_$n.err) || { tail -5 /tmp/k1_$n.err; exit 1; }; echo "== $n $r"
done
