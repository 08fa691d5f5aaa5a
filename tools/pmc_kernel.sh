#!/bin/bash
# One PMC pass per counter group over a short bench run (kernel-trace only); summary per kernel.
# Usage: tools/pmc_kernel.sh <outdir> "<counters pass 1>" ["<counters pass 2>" ...]
set -o pipefail
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --profile-frames 1 ${BENCH_ARGS:-}"
i=0
for pass in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/p$i -o run -- python bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python tools/pmc_summary.py $OUT > $OUT/summary.json
