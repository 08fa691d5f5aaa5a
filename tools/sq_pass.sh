#!/bin/bash
# One SQ PMC pass over a short serial bench run (kernel-trace only), summarised per kernel.
# Usage: tools/sq_pass.sh <tag> "<up to 8 SQ counters>"
set -o pipefail
export TMPDIR=/tmp
T=$1; C=$2; shift 2
rm -rf gpurun_out/$T
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/$T/p1 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-frames 1 --no-sky-lane "$@" > gpurun_out/$T.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/$T.log; exit 1; }
python tools/pmc_summary.py gpurun_out/$T > gpurun_out/$T.json
python - "$T" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/{sys.argv[1]}.json"))
keys = sorted({k for v in d.values() for k in v if k.startswith("SQ_")})
print(f"{'kernel':34s}" + "".join(f"{k[3:15]:>13s}" for k in keys))
for k, v in sorted(d.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    if k.startswith("soc::"):
        print(f"{k[5:39]:34s}" + "".join(f"{v.get(c, 0):13.4g}" for c in keys))
PY
