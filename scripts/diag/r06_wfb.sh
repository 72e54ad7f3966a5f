#!/bin/bash
# round 6: library builds abv/<name> given as arguments (e.g. wfb1: the
# PAIRS base formed in the wide kernel's prologue; sc8k / sc16k: 8 K / 16 K-row
# grouping scatter blocks) against the tree: wide_probe.py outputs bit for
# bit (incl. a PAIRS case), then the C5 bf16 leg of each build, twice
# (bench.py puts the repo first on sys.path: the build goes in by HHFM_AB_ROOT)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r06/wfb
mkdir -p $o
for n in base "$@"; do
  rm -rf /tmp/wv_$n && mkdir -p /tmp/wv_$n && cp -r hhfm_amd /tmp/wv_$n/ || exit 1
  [ $n != base ] && { cp abv/$n/*.so /tmp/wv_$n/hhfm_amd/lib/ || exit 1; }
  PYTHONPATH=/tmp/wv_$n timeout -k 10 200 python scripts/diag/wide_probe.py $o/$n.npz || exit 1
done
for n in "$@"; do python scripts/diag/wide_compare.py $o/base.npz $o/$n.npz; done
for rep in 1 2; do for n in base "$@"; do
  HHFM_AB_ROOT=/tmp/wv_$n timeout -k 10 300 python bench.py --legs c5 --no-pmc > $o/c5_$n.json 2> $o/c5_$n.err || { tail -20 $o/c5_$n.err; exit 1; }
  python3 -c "
import json
d = json.loads(open('$o/c5_$n.json').read().strip().splitlines()[-1]); ex = d.get('extra', d)
v = ex.get('dfm_c5', {}); print('$n', v.get('ms_per_pass'), v.get('kernel_ms'), (v.get('parity') or {}).get('parity'))"
done; done
