#!/bin/bash
# Round-3 profiles of the final code: rocprofv3 kernel traces (bench,
# microbench) + K1 PMC traffic (scripts/gpu_profile.sh), then SQ counters of
# the C5 bf16 kernel (scripts/pmc_k3w.sh).  Each step time-limited.
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu_profile.sh > gpurun_out/prof_r03.log 2>&1 || { echo "profile failed"; tail gpurun_out/prof_r03.log; exit 1; }
echo "profiles done"
bash scripts/pmc_k3w.sh > gpurun_out/pmck3w.txt 2>&1 || { echo "pmc failed"; tail gpurun_out/pmck3w.txt; exit 1; }
cat gpurun_out/pmck3w.txt
