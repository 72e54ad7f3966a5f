#!/bin/bash
# round 6: persistent fp32 DeepFM kernel — DeepFM GPU tests, then the C5 legs
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/dfm32
timeout -k 10 600 python -u -m pytest tests/test_gpu_dfm.py tests/test_gpu_training.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/dfm32/pytest.txt 2>&1 || { tail -40 gpurun_out/r06/dfm32/pytest.txt; exit 1; }
tail -2 gpurun_out/r06/dfm32/pytest.txt
timeout -k 10 300 python bench.py --legs c5 --no-pmc > gpurun_out/r06/dfm32/bench_c5.json 2> gpurun_out/r06/dfm32/bench_c5.err || { tail -20 gpurun_out/r06/dfm32/bench_c5.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06/dfm32/bench_c5.json").read().strip().splitlines()[-1])
ex = d.get("extra", d)
for k in ("dfm_c5", "dfm_c5_f32"):
    v = ex.get(k, {})
    print(k, v.get("ms_per_pass"), v.get("kernel_ms"), (v.get("parity") or {}).get("parity"))
PY
