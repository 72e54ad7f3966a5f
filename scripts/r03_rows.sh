#!/bin/bash
# the per-row table (scripts/rowtable.py), one leg per process
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/rows
for leg in ${ROW_LEGS:-c2 c3 c4 c5 afm h6 h35}; do
  ROWS_ONLY=$leg timeout -k 10 400 python scripts/rowtable.py > gpurun_out/rows/rows_$leg.json 2> gpurun_out/rows/rows_$leg.err || { echo "rowtable $leg failed"; tail gpurun_out/rows/rows_$leg.err; exit 1; }
  echo "rows $leg done"
done
