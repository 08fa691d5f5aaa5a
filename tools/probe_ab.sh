# Lane-probe decisions over repeated default bench runs per configuration (which queue the renderer keeps, and the fps).
set -o pipefail
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/$n.json 2> gpurun_out/$n.err || { echo "bench $n failed"; tail -5 gpurun_out/$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/$n.json'));print('$n', d['value'], 'fps', d['config'].get('sky_lane_queue'), d['config'].get('untimed_lane_probe_frames'), 'frac', d['roofline']['frac'])"
}
for i in 1 2 3 4; do run pw_c3_$i || exit 1; done
run pw_c2_1 --config c2 && run pw_c2_2 --config c2 && run pw_c4_1 --config c4 && run pw_c4_2 --config c4 || exit 1
run pw_rc4 --config c4 --raster && run pw_rc3 --raster && run pw_rc2 --config c2 --raster || exit 1
