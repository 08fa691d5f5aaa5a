#!/bin/bash
# per-pass raster times under knob variants: end-to-end (--raster) for the configs given (default c3 c4)
set -o pipefail
CONFIGS="${CONFIGS:-c3 c4}"
for c in $CONFIGS; do
  for v in "$@"; do
    vv="$v"; [ "$v" = "-" ] && vv=""
    env $vv timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-frames 5 --raster --config $c > gpurun_out/rs.json 2> gpurun_out/rs.err || { echo "fail $c $v"; tail -3 gpurun_out/rs.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/rs.json')); m=d['ms_per_pass']; print('%s %-24s fps %7.1f  prepass %.1f shadow %.1f gbuf %.1f' % ('$c', '$v', d['value'], 1e3*m['DepthPrepass'], 1e3*m['SunShadowDraw'], 1e3*m['GBufferGeneration']))"
  done
done
