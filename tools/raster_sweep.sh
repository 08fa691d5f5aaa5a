#!/bin/bash
# per-pass raster times under knob variants: C3 and C4 end-to-end (--raster)
set -o pipefail
for c in c3 c4; do
  for v in "-" "SOC_RASTER_PRECHECK=1" "SOC_RASTER_SMALL=16" "SOC_RASTER_SMALL=256" "SOC_RASTER_SMALL=1024"; do
    vv="$v"; [ "$v" = "-" ] && vv=""
    env $vv timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-frames 5 --raster --config $c > gpurun_out/rs.json 2> gpurun_out/rs.err || { echo "fail $c $v"; tail -3 gpurun_out/rs.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/rs.json')); m=d['ms_per_pass']; print('%s %-24s fps %7.1f  prepass %.1f shadow %.1f gbuf %.1f' % ('$c', '$v', d['value'], 1e3*m['DepthPrepass'], 1e3*m['SunShadowDraw'], 1e3*m['GBufferGeneration']))"
  done
done
