#!/bin/bash
# A/B a tuning knob: kernel trace of the serial-lane bench (c4 and c3) per knob value; prints the top kernels.
# Usage: tools/ab_knob.sh KNOB "v1 v2 ..." [bench args]
set -o pipefail
export TMPDIR=/tmp
K=$1; VALS=$2; shift 2
mkdir -p gpurun_out
for v in $VALS; do
  for cfg in c4 c3; do
    d=gpurun_out/ab_${K}_${v}_${cfg}
    env $K=$v timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-sky-lane "$@" > $d.json 2> $d.err || { echo "bench $v $cfg failed"; tail -5 $d.err; exit 1; }
    echo "$K=$v $cfg $(python -c "import json;d=json.load(open('$d.json'));print(d['value'], d['ms_per_group'])")"
  done
done
