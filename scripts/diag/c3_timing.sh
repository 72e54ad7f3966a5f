#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
rm -rf /tmp/c3t && mkdir -p /tmp/c3t && cp -r hhfm_amd /tmp/c3t/ && cp abt/t/*.so /tmp/c3t/hhfm_amd/lib/ || exit 1
PYTHONPATH=/tmp/c3t timeout -k 10 120 python scripts/diag/c3_timing.py
