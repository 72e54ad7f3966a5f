#!/bin/bash
# round 6: dfm_fused_f32s phase timing (diag build abv/f32st)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/f32s
rm -rf /tmp/f32v && mkdir -p /tmp/f32v && cp -r hhfm_amd /tmp/f32v/ && cp abv/f32st/*.so /tmp/f32v/hhfm_amd/lib/ || exit 1
PYTHONPATH=/tmp/f32v timeout -k 10 300 python scripts/diag/f32s_phases.py > gpurun_out/r06/f32s/phases.json 2> gpurun_out/r06/f32s/phases.err || { tail -20 gpurun_out/r06/f32s/phases.err; exit 1; }
cat gpurun_out/r06/f32s/phases.json
