#!/bin/bash
# catalog_ring with the filter pipelined one tile late (default) vs not, at
# the C4 shape, after the ring/seed parity tests.
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/k2pipe
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "seed or c4_shard or streaming" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python scripts/k2_c4.py --variants seed,nopipe,seed,nopipe > $out/ab.json 2> $out/ab.err || { tail $out/ab.err; exit 1; }
head -8 $out/ab.json
