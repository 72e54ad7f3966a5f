#!/bin/bash
# K2 at the C4 shard: kernel stats + LDS bank-conflict / SQ counter passes
# of the in-tree library (separate rocprofv3 runs; no tracing with --pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
d=gpurun_out/k2r05${1:-}
mkdir -p $d
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d/kt -o kt --output-format csv -- python3 scripts/k2_c4.py --reps 10 --variants seed > $d/kt.log 2>&1 || { tail $d/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d $d/pmc -o pmc --output-format csv -- python3 scripts/k2_c4.py --reps 2 --variants seed > $d/pmc.log 2>&1 || { tail $d/pmc.log; exit 1; }
echo k2r05 done
