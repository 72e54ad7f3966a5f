# DeepFM C5 direct kernel (bf16 MLP, fp32 table): L2 hit/miss and memory-side
# read requests (one rocprofv3 --pmc pass).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp MB_ONLY=dfm MB_DFM_LEGS=dfm_c5_bf16,dfm_c5_bf16_tbf16 MB_DFM_PROJ=0
mkdir -p gpurun_out/pmctcc
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum -d gpurun_out/pmctcc/a -o pmc --output-format csv -- python3 scripts/microbench.py > gpurun_out/pmctcc/a.log 2>&1 || { tail -5 gpurun_out/pmctcc/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr GRBM_GUI_ACTIVE -d gpurun_out/pmctcc/b -o pmc --output-format csv -- python3 scripts/microbench.py > gpurun_out/pmctcc/b.log 2>&1 || { tail -5 gpurun_out/pmctcc/b.log; exit 1; }
echo done
