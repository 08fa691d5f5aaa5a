#!/bin/bash
# One parameterised driver for the GPU-box steps (run under gpurun from the repo root). Every GPU step runs under
# its own time limit; the script stops at the first failure (no retries). Outputs go to gpurun_out/.
#
#   tools/gpu.sh suite                          full -m gpu suite, smoke(), the default bench line
#   tools/gpu.sh tests "<pytest -k expr>"       selected GPU tests
#   tools/gpu.sh bench NAME [bench args]        one bench line -> gpurun_out/NAME.json (fps, ms/step, roofline frac)
#   tools/gpu.sh ab "K=V,K2=V2" "" "--flag,K=V" ... -- [bench args]
#                                               the bench line under variants: K=V items are environment
#                                               variables, "-..." items extra bench arguments ("" = none)
#   tools/gpu.sh kt TAG [bench args]            rocprofv3 --kernel-trace --stats of the default bench run (top kernels)
#   tools/gpu.sh pmc TAG "<counters>" ... [-- bench args]
#                                               one rocprofv3 --pmc pass per counter group (kernel trace only) + summary
#   tools/gpu.sh traffic TAG [bench args]       FETCH_SIZE / WRITE_SIZE passes -> per-kernel HBM traffic table
#   tools/gpu.sh round TAG                      the round-end measurement set (bench lines C3/C2/C3b/C4/raster C2/C3/C4, the RCCL
#                                               exchange line, frame PNG, kernel trace + same-run event check + traffic)
#   tools/gpu.sh valu TAG                       VALU issue calibration + the serial frame's SQ counters -> valu model
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cmd=${1:?usage: tools/gpu.sh suite|tests|bench|ab|kt|pmc|traffic|round ...}
shift

bench_line() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/$n.json 2> gpurun_out/$n.err || { echo "bench $n failed"; tail -5 gpurun_out/$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/$n.json'));pk=d['roofline'].get('per_kernel',{});print('$n', d['value'], 'fps', d['ms_per_step'], 'ms', 'frac', d['roofline']['frac'], {k[:11]: v['avg_launch_us'] for k, v in pk.items() if v}, d['ms_per_group'])"
}

kernel_trace() {   # tag, bench args...
  local t=$1; shift
  rm -rf gpurun_out/${t}_kt
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${t}_kt -o run -- python bench.py --no-cpu-baseline "$@" > gpurun_out/${t}_kt.log 2>&1 || { echo "kernel trace failed"; tail -5 gpurun_out/${t}_kt.log; exit 1; }
  local f; f=$(find gpurun_out/${t}_kt -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${t}_kernel_stats.csv
  python - "$t" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/{sys.argv[1]}_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:18]:
    print(f'{r["Name"].replace("(anonymous namespace)::", "")[:72]:72s} calls {r["Calls"]:>5s} avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
}

pmc_passes() {   # tag, counter groups..., [-- bench args]
  local t=$1; shift
  local groups=() args=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do groups+=("$1"); shift; done
  [ "$1" = "--" ] && shift && args=("$@")
  local i=0
  for c in "${groups[@]}"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${t}_pmc/p$i -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-frames 1 "${args[@]}" > gpurun_out/${t}_pmc_p$i.log 2>&1 || { echo "pmc pass $i ($c) failed"; tail -5 gpurun_out/${t}_pmc_p$i.log; exit 1; }
  done
}

case $cmd in
  suite)
    timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
    rc=$?; tail -1 gpurun_out/gpu_tests.log
    [ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests.log | head -20; exit 1; }
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
    tail -1 gpurun_out/smoke.log
    bench_line bench ;;
  tests)
    timeout -k 10 900 python -u -m pytest tests -v -m gpu -k "${1:?pytest -k expression}" --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_k.log 2>&1
    rc=$?; tail -1 gpurun_out/gpu_tests_k.log
    [ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR|Error" gpurun_out/gpu_tests_k.log | head -20; exit 1; } ;;
  bench)
    n=${1:?name}; shift; bench_line "$n" "$@" ;;
  ab)
    vars=()
    while [ $# -gt 0 ] && [ "$1" != "--" ]; do vars+=("$1"); shift; done
    [ "$1" = "--" ] && shift
    i=0
    for v in "${vars[@]}"; do
      i=$((i+1))
      echo "[$v]"
      # a variant is comma-separated: K=V items are exported, items starting with "-" are extra bench arguments
      ( extra=(); IFS=, read -ra items <<< "$v"
        for it in "${items[@]}"; do case $it in -*) extra+=("$it") ;; ?*) export "$it" ;; esac; done
        bench_line ab_$i --steps 40 --warmup 10 --no-cpu-baseline "${extra[@]}" "$@" ) || exit 1
    done ;;
  kt)
    t=${1:?tag}; shift; kernel_trace "$t" "$@" ;;
  pmc)
    t=${1:?tag}; shift; pmc_passes "$t" "$@"
    python tools/pmc_summary.py gpurun_out/${t}_pmc > gpurun_out/${t}_pmc_summary.json && echo "summary: gpurun_out/${t}_pmc_summary.json" ;;
  traffic)
    t=${1:?tag}; shift; pmc_passes "$t" FETCH_SIZE WRITE_SIZE -- "$@"
    python tools/pmc_summary.py gpurun_out/${t}_pmc --traffic gpurun_out/${t}_pmc_traffic.json --scene mesh > gpurun_out/${t}_pmc_summary.json && echo "traffic: gpurun_out/${t}_pmc_traffic.json" ;;
  round)
    t=${1:?tag}
    bench_line ${t}_bench
    bench_line ${t}_bench_c2 --config c2 --no-cpu-baseline
    bench_line ${t}_bench_c3b --config c3b --no-cpu-baseline
    bench_line ${t}_bench_c4 --config c4 --no-cpu-baseline
    bench_line ${t}_bench_raster_c2 --config c2 --raster --no-cpu-baseline
    bench_line ${t}_bench_raster_c3 --raster --no-cpu-baseline
    bench_line ${t}_bench_raster_c4 --config c4 --raster --no-cpu-baseline
    bench_line ${t}_frame_c3_960 --raster --no-cpu-baseline --width 960 --height 540 --steps 5 --warmup 2 --write-frame gpurun_out/${t}_frame_raster_c3_960x540.png
    bench_line ${t}_bench_exchange --exchange --no-cpu-baseline
    # the kernel trace of the default command, with the bench's per-frame pass events of the same run (event_trace_check)
    SOC_BENCH_EVENTS_OUT=gpurun_out/${t}_events.json kernel_trace $t
    python tools/roofline_check.py gpurun_out/${t}_bench.json gpurun_out/${t}_kt > gpurun_out/${t}_roofline_check.json
    python tools/event_trace_check.py compare gpurun_out/${t}_events.json "$(find gpurun_out/${t}_kt -name '*kernel_trace.csv' | head -1)" > gpurun_out/${t}_event_trace_check.json
    pmc_passes $t FETCH_SIZE WRITE_SIZE
    python tools/pmc_summary.py gpurun_out/${t}_pmc --traffic gpurun_out/${t}_pmc_traffic.json --scene mesh > gpurun_out/${t}_pmc_summary.json ;;
  valu)
    # VALU issue calibration: the microbenchmark, its counter check, the serial-lane frame's counters
    t=${1:?tag}
    hipcc --offload-arch=gfx950 -O3 -o gpurun_out/valu_rate tools/microbench/valu_rate.hip || exit 1
    timeout -k 10 120 ./gpurun_out/valu_rate > gpurun_out/${t}_valu_rate.txt 2>&1 || { echo valu_rate failed; exit 1; }
    rm -rf gpurun_out/${t}_vr_pmc
    timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/${t}_vr_pmc -o run -- ./gpurun_out/valu_rate > gpurun_out/${t}_vr_pmc.log 2>&1 || { echo valu pmc failed; exit 1; }
    pmc_passes ${t}sq "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" -- --no-sky-lane
    python tools/valu_calibrate.py gpurun_out/${t}_valu_rate.txt gpurun_out/${t}_vr_pmc gpurun_out/${t}sq_pmc > gpurun_out/${t}_valu_model.json && echo "valu model: gpurun_out/${t}_valu_model.json" ;;
  *)
    echo "unknown command $cmd"; exit 2 ;;
esac
