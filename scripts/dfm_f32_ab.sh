#!/bin/bash
# fp32-MLP DeepFM: GPU tests, then phase timings (2M rows) and the C5 bench
# leg for the split-bf16 kernel, and the exact-fp32 kernel for comparison.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/dfm
timeout -k 10 300 python -u -m pytest tests/test_gpu_dfm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dfm/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/dfm/pytest.log; exit 1; }
tail -1 gpurun_out/dfm/pytest.log
timeout -k 10 200 python3 scripts/dfm_f32_phases.py || exit 1
timeout -k 10 300 python bench.py --legs c5 --cpu-seconds 0 --steps 3 --warmup 1 > gpurun_out/dfm/split.json 2> gpurun_out/dfm/split.err || exit 1
python - <<'P'
import json
d=json.load(open("gpurun_out/dfm/split.json"))
for n in ("dfm_c5","dfm_c5_f32"):
    e=d["extra"][n]
    print(n, e.get("kernel_ms"), e.get("roofline",{}).get("frac"), json.dumps(e.get("parity")), e.get("error"))
P
