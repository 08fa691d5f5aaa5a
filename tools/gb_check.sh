#!/bin/bash
# G-buffer change check: the raster / C1 GPU tests, then two bench --raster lines (GBufferGeneration ms).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_raster.py tests/test_c1_helmet.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gb_tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/gb_tests.log | head; tail -20 gpurun_out/gb_tests.log; exit 1; }
tail -1 gpurun_out/gb_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --raster --steps 20 --warmup 5 --no-cpu-baseline ${GB_ARGS:-} > gpurun_out/gb_$i.json 2> gpurun_out/gb_$i.err || { tail -5 gpurun_out/gb_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/gb_$i.json'));print(d['value'], d['ms_per_pass']['GBufferGeneration'])"
done
