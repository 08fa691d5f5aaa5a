#!/bin/bash
# Round-end measurement set: bench lines (C3 default with the CPU baseline, C2, C3b, C4, raster C3/C4, a
# 960x540 raster frame PNG) and the C3 kernel-trace + FETCH/WRITE PMC traffic table. Usage: tools/round_profiles.sh <tag>
set -o pipefail
T=${1:-r02}
mkdir -p gpurun_out
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/${T}_bench_$n.json 2> gpurun_out/${T}_bench_$n.err || { echo "bench $n failed"; tail -5 gpurun_out/${T}_bench_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_bench_$n.json'));print('$n', d['value'], d['ms_per_step'], d['roofline']['frac'])"
}
run c3
run c2 --config c2 --no-cpu-baseline
run c3b --config c3b --no-cpu-baseline
run c4 --config c4 --no-cpu-baseline
run raster_c3 --raster --no-cpu-baseline
run raster_c4 --config c4 --raster --no-cpu-baseline
run frame_c3_960 --raster --no-cpu-baseline --width 960 --height 540 --steps 5 --warmup 2 --write-frame gpurun_out/${T}_frame_raster_c3_960x540.png
bash tools/profile_c3.sh $T || exit 1
