#!/bin/bash
# AFM A1 / A2 kernels: times and SQ / LDS / L2 counters (scripts/afm_phases.py).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/pmcafm
mkdir -p $o
timeout -k 10 200 python3 scripts/afm_phases.py > $o/phases.json 2> $o/phases.err || { tail $o/phases.err; exit 1; }
cat $o/phases.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/kt -o kt --output-format csv -- python3 scripts/afm_phases.py > $o/kt.log 2>&1 || { tail $o/kt.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES -d $o/a -o pmc --output-format csv -- python3 scripts/afm_phases.py > $o/a.log 2>&1 || { tail $o/a.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $o/b -o pmc --output-format csv -- python3 scripts/afm_phases.py > $o/b.log 2>&1 || { tail $o/b.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum -d $o/c -o pmc --output-format csv -- python3 scripts/afm_phases.py > $o/c.log 2>&1 || { tail $o/c.log; exit 1; }
echo done
