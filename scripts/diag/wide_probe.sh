#!/bin/bash
# Diagnostic: run scripts/diag/wide_probe.py under every variant build in
# abw/*/ (a private copy of the package per variant, so hhfm_amd/lib is never
# overwritten), then compare each against abw/r2w8 (the shipped setting).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/wide
for d in abw/*/; do
  n=$(basename $d)
  rm -rf /tmp/wv_$n && mkdir -p /tmp/wv_$n && cp -r hhfm_amd /tmp/wv_$n/ && cp $d/*.so /tmp/wv_$n/hhfm_amd/lib/ || exit 1
  PYTHONPATH=/tmp/wv_$n timeout -k 10 120 python scripts/diag/wide_probe.py gpurun_out/wide/$n.npz || exit 1
done
python scripts/diag/wide_compare.py gpurun_out/wide/r2w8.npz gpurun_out/wide/*.npz
