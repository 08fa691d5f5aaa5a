#!/bin/bash
# Kernel-trace stats of a short bench run: per-kernel average durations.
set -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/ktq
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktq -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --profile-frames 2 --no-sky-lane ${KT_ARGS:-} > gpurun_out/ktq.log 2>&1 || exit 1
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/ktq/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'].replace('(anonymous namespace)::', '')[:60]:60s} {r['Calls']:>5} {float(r['AverageNs'])/1000:8.1f} us")
PY
