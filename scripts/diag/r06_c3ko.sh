#!/bin/bash
# round 6: C3 in-kernel merge knock-outs (abv/ko1: no list loads, abv/ko2: no merge)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
AB_DIR=abv bash scripts/diag/c3_libs6.sh ko4 ko2 > gpurun_out/r06/c3ko.txt 2>&1 || { tail -20 gpurun_out/r06/c3ko.txt; exit 1; }
cat gpurun_out/r06/c3ko.txt
