#!/bin/bash
# SQ counter passes (separate --pmc runs, no tracing) on the C4-shape K2 kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
d=gpurun_out/pmc_k2${1:-}
mkdir -p $d
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES -d $d/a -o pmc --output-format csv -- python3 scripts/k2_c4.py --reps 2 --variants seed > $d/a.log 2>&1 || { tail $d/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $d/b -o pmc --output-format csv -- python3 scripts/k2_c4.py --reps 2 --variants seed > $d/b.log 2>&1 || { tail $d/b.log; exit 1; }
echo pmc done
