#!/bin/bash
# Raster GPU tests + end-to-end (--raster) bench lines for C3 and C4.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_raster.py tests/test_output.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/raster_tests.log 2>&1
rc=$?; echo "raster tests rc=$rc"; tail -3 gpurun_out/raster_tests.log; [ $rc -eq 0 ] || exit 1
for c in c3 c4; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --profile-frames 10 --raster --config $c --write-frame gpurun_out/frame_raster_$c.png --metrics-jsonl gpurun_out/metrics_raster_$c.jsonl > gpurun_out/raster_bench_$c.json 2> gpurun_out/raster_bench_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/raster_bench_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/raster_bench_$c.json')); print('$c', 'fps %.1f ms %.4f' % (d['value'], d['ms_per_step']), ' '.join('%s=%.1f' % (k[:16], 1e3 * v) for k, v in d['ms_per_pass'].items()))"
done
