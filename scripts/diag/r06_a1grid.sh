#!/bin/bash
# round 6: A1 (afm_rows_pairs) grid = resident workgroups (the tree) vs the old
# 2,048-workgroup cap (abv/cap1): AFM GPU tests, then the row table's AFM legs
# of each build, alternating twice.  (Measured equal, profiles/r06_a1_grid_ab.txt;
# the resident-grid code was not kept — git history, round 6.)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r06/a1grid
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_afm.py -m gpu -q --timeout 200 --timeout-method thread > $o/pytest.txt 2>&1 || { tail -30 $o/pytest.txt; exit 1; }
tail -1 $o/pytest.txt
for n in base cap1; do
  rm -rf /tmp/a1_$n && mkdir -p /tmp/a1_$n && cp -r hhfm_amd /tmp/a1_$n/ || exit 1
  [ $n != base ] && { cp abv/$n/*.so /tmp/a1_$n/hhfm_amd/lib/ || exit 1; }
done
for rep in 1 2; do for n in base cap1; do
  HHFM_AB_ROOT=/tmp/a1_$n ROWS_ONLY=afm timeout -k 10 300 python scripts/rowtable.py > $o/rows_$n.json 2> $o/rows_$n.err || { tail -20 $o/rows_$n.err; exit 1; }
  python3 -c "
import json
d = json.load(open('$o/rows_$n.json'))
print('$n', 'A1 ms', d['A1_afm_rows']['gpu_ms'], 'frac', d['A1_afm_rows']['roofline']['frac'], 'A2 ms', d['A2_afm_catalog']['gpu_ms'])"
done; done
