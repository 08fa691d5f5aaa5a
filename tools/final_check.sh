#!/bin/bash
# Full GPU suite + smoke on one box (each step under its own limit; stops at the first failure).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 || { tail -40 gpurun_out/final_gpu_tests.log; exit 1; }
tail -3 gpurun_out/final_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -2 gpurun_out/final_smoke.log
