#!/bin/bash
# SQ counter passes (separate --pmc runs, no tracing) on a microbench leg.
# usage: MB_ONLY=k2 bash scripts/pmc_sq.sh <outdir-name>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
d=gpurun_out/pmc_${1:-sq}
mkdir -p $d
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES -d $d/a -o pmc --output-format csv -- python3 scripts/microbench.py > $d/a.log 2>&1 || { tail $d/a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $d/b -o pmc --output-format csv -- python3 scripts/microbench.py > $d/b.log 2>&1 || { tail $d/b.log; exit 1; }
echo done
