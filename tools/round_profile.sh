#!/bin/bash
# Round-end evidence on the GPU box: full GPU test suite, default bench (with CPU baseline), the C4 bench,
# rocprofv3 kernel-trace stats of the bench, PMC FETCH_SIZE / WRITE_SIZE passes -> traffic table.
# Usage: tools/round_profile.sh <tag>   (outputs under gpurun_out/<tag>_*)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > gpurun_out/${T}_bench_c4.json 2> gpurun_out/${T}_bench_c4.err || { echo "c4 bench failed"; tail -5 gpurun_out/${T}_bench_c4.err; exit 1; }
for c in c3 c4; do
  timeout -k 10 300 python bench.py --config $c --raster --no-cpu-baseline --write-frame gpurun_out/${T}_frame_raster_$c.png --metrics-jsonl gpurun_out/${T}_metrics_raster_$c.jsonl > gpurun_out/${T}_bench_raster_$c.json 2> gpurun_out/${T}_bench_raster_$c.err || { echo "raster bench $c failed"; tail -5 gpurun_out/${T}_bench_raster_$c.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt_raster -o run -- python bench.py --raster --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_kt_raster.log 2>&1 || { echo "raster kernel trace failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_kt.log 2>&1 || { echo "kernel trace failed"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${T}_pmc/$c -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-frames 1 > gpurun_out/${T}_pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python tools/pmc_summary.py gpurun_out/${T}_pmc --traffic gpurun_out/${T}_pmc_traffic.json > gpurun_out/${T}_pmc_summary.json
echo done
