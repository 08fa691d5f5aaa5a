#!/bin/bash
# rocprofv3 kernel trace (+stats) of the default bench command and the FETCH_SIZE / WRITE_SIZE passes
# (separate runs, --kernel-trace only) -> per-kernel HBM traffic table. Usage: tools/profile_c3.sh <tag> [bench args]
set -o pipefail
export TMPDIR=/tmp
T=${1:-r02}
shift
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/${T}_kt.log 2>&1 || { echo "kernel trace failed"; tail -5 gpurun_out/${T}_kt.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${T}_pmc/$c -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-frames 1 "$@" > gpurun_out/${T}_pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/${T}_pmc_$c.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/${T}_pmc --traffic gpurun_out/${T}_pmc_traffic.json --scene mesh > gpurun_out/${T}_pmc_summary.json
f=$(find gpurun_out/${T}_kt -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_kernel_stats.csv
python - <<PY
import csv
rows = list(csv.DictReader(open("gpurun_out/${T}_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>5s} avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
echo done
