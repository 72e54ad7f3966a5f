# K1 w-gather cache-policy variants: memory-side read requests by size
# (one rocprofv3 --pmc pass; scripts/k1_wpolicy.py runs each variant once).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcw
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum -d gpurun_out/pmcw/a -o pmc --output-format csv -- python3 scripts/k1_wpolicy.py --reps 1 > gpurun_out/pmcw/a.log 2>&1 || { tail -5 gpurun_out/pmcw/a.log; exit 1; }
echo done
