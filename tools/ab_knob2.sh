#!/bin/bash
# A/B of one tuning knob on the default bench line: tests matching $TESTS first (if set), then bench lines
# alternating KNOB=0 / KNOB=1, twice each.  Usage: KNOB=SOC_X [TESTS="pytest -k expression"] [BENCH_ARGS=...] tools/ab_knob2.sh
set -o pipefail
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$TESTS" > gpurun_out/ab2_tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/ab2_tests.log | head; tail -20 gpurun_out/ab2_tests.log; exit 1; }
  tail -1 gpurun_out/ab2_tests.log
fi
for rep in 1 2; do for v in 0 1; do
  env $KNOB=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab2_${v}_$rep.json 2> gpurun_out/ab2_${v}_$rep.err || { tail -5 gpurun_out/ab2_${v}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab2_${v}_$rep.json'));print('$KNOB=$v', d['value'], d['ms_per_pass'].get('CloudRendering'))"
done; done
