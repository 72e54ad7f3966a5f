#!/bin/bash
# final-code profiles: rocprofv3 stats of the bench and the microbench + K1
# PMC passes (scripts/gpu_profile.sh), then the row table's C5 and AFM legs
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu_profile.sh > gpurun_out/prof_r03.log 2>&1 || { echo "profile failed"; tail gpurun_out/prof_r03.log; exit 1; }
echo "profiles done"
ROW_LEGS="c5 afm" bash scripts/r03_rows.sh
