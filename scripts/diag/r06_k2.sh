#!/bin/bash
# round 6: K2 ring with the deferred selection vs without (A/B, alternating), C4 shard shape
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/k2libs
AB_DIR=abv VARIANTS=seed bash scripts/k2_libs.sh defer nodefer defer nodefer
