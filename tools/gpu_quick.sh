#!/bin/bash
# Quick GPU iteration: selected parity tests + bench without the CPU baseline. Usage: tools/gpu_quick.sh "<pytest -k expr>"
set -o pipefail
mkdir -p gpurun_out
K="${1:-ssao}"
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu -k "$K" -x > gpurun_out/quick_tests.log 2>&1
echo "TESTS EXIT $?" >> gpurun_out/quick_tests.log
tail -5 gpurun_out/quick_tests.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err
echo "BENCH EXIT $?"
python - <<'PY'
import json
d = json.load(open("gpurun_out/quick_bench.json"))
print("fps", d["value"], "ms/step", d["ms_per_step"], "north_star", d["north_star"])
print("ms_per_pass", d["ms_per_pass"])
print("gbs", d["gbs_per_pass"])
PY
