#!/bin/bash
# Diagnostic: C5 DeepFM forward time for each prebuilt library variant
# (scripts/build_variants.sh ... into ab/<name>/), alternating twice.
cd "${GRAFT_REPO_ROOT:-.}"
for rnd in 1 2; do
for d in "$@"; do
  cp $d/*.so hhfm_amd/lib/ && echo -n "$d " && timeout -k 10 120 python scripts/k3w_time.py ${K3W_ROWS:-4000000} 5 || exit 1
done
done
