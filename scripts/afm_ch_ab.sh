#!/bin/bash
# A2 (300 queries x 4,082 items, k = A = 64) with the per-query kernel at
# different item-chunk counts per query (HHFM_AFM_W_CH), alternating
cd "${GRAFT_REPO_ROOT:-.}"
for rnd in 1 2; do
  for c in 1 2 3 4 6; do
    echo -n "ch=$c " && HHFM_AFM_W_CH=$c MB_ONLY=afm timeout -k 10 120 python scripts/microbench.py 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print(round(d['afm_topk_c300_k64']['median_ms'],4))" || exit 1
  done
done
