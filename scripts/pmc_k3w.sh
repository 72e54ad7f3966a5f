#!/bin/bash
# SQ counters on the C5 DeepFM forward (scripts/k3w_time.py, 4 M rows): two
# passes, each time-limited; summary via scripts/pmc_summary.py
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/pmck3w
mkdir -p $o
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES -d $o/a -o pmc --output-format csv -- python3 scripts/k3w_time.py 4000000 3 > $o/a.log 2>&1 || { tail $o/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $o/b -o pmc --output-format csv -- python3 scripts/k3w_time.py 4000000 3 > $o/b.log 2>&1 || { tail $o/b.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SMEM -d $o/c -o pmc --output-format csv -- python3 scripts/k3w_time.py 4000000 3 > $o/c.log 2>&1 || { tail $o/c.log; exit 1; }
python3 scripts/pmc_summary.py $o dfm_fused_w
