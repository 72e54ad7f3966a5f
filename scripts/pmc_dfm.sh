#!/bin/bash
# DeepFM C5 kernels (scripts/microbench.py's dfm legs): SQ / LDS counters in
# two passes.  MB_DFM_LEGS / MB_DFM_PROJ select the legs (default: the bf16
# MLP leg, every layer-0 plan).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MB_ONLY=dfm MB_DFM_LEGS=${MB_DFM_LEGS:-dfm_c5_bf16}
mkdir -p gpurun_out/pmcdfm
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES -d gpurun_out/pmcdfm/a -o pmc --output-format csv -- python3 scripts/microbench.py > gpurun_out/pmcdfm/a.log 2>&1 || { tail gpurun_out/pmcdfm/a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmcdfm/b -o pmc --output-format csv -- python3 scripts/microbench.py > gpurun_out/pmcdfm/b.log 2>&1 || { tail gpurun_out/pmcdfm/b.log; exit 1; }
echo done
