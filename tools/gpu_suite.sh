#!/bin/bash
# Full GPU test suite, smoke, then the default bench line (each step under its own limit; stops at the first failure).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/gpu_tests.log | head -20; tail -30 gpurun_out/gpu_tests.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
