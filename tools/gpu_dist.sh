#!/bin/bash
# The 2-rank GPU tests (shared device, gloo) and the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread > gpurun_out/dist_tests.log 2>&1
rc=$?; tail -15 gpurun_out/dist_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
