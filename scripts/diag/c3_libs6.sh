#!/bin/bash
# Diagnostic: scripts/diag/c3_ab6.py across library builds (base = the tree,
# then abv/<name>), alternating twice, one process per build.
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
for d in base "$@"; do
  n=$(basename $d)
  rm -rf /tmp/c3_$n && mkdir -p /tmp/c3_$n && cp -r hhfm_amd /tmp/c3_$n/ || exit 1
  [ "$d" != base ] && { cp abv/$d/*.so /tmp/c3_$n/hhfm_amd/lib/ || exit 1; }
  r=$(PYTHONPATH=/tmp/c3_$n timeout -k 10 200 python scripts/diag/c3_ab6.py 2>/tmp/c3_$n.err) || { tail -5 /tmp/c3_$n.err; exit 1; }; echo "== $n $r"
done
done
