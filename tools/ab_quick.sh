#!/bin/bash
# A/B frame time: default bench vs extra flags. Usage: tools/ab_quick.sh "<flags B>" ["<pytest -k expr>"]
set -o pipefail
mkdir -p gpurun_out
if [ -n "$2" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -k "$2" -x --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab_a.json 2> gpurun_out/ab_a.err || exit 1
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline $1 > gpurun_out/ab_b.json 2> gpurun_out/ab_b.err || exit 1
python - <<'PY'
import json
for t in "ab":
    d = json.load(open(f"gpurun_out/ab_{t}.json"))
    print(t, "fps", d["value"], "ms/step", d["ms_per_step"], "comp_us", d["roofline"]["avg_launch_us"], "ns_us", d["north_star"]["us"])
print("passes", json.load(open("gpurun_out/ab_a.json"))["ms_per_pass"])
PY
