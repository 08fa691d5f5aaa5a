#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per kernel under an environment variant (separate PMC passes, kernel trace only).
# Usage: tools/pmc_ab.sh <tag> "K=V,K2=V2" [bench args]
set -o pipefail
export TMPDIR=/tmp
T=$1; V=$2; shift 2
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  env ${V//,/ } timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${T}_pmc/$c -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-frames 1 "$@" > gpurun_out/${T}_pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/${T}_pmc_$c.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/${T}_pmc --traffic gpurun_out/${T}_pmc_traffic.json --scene mesh > /dev/null
python - "$T" <<'PY'
import json, sys
t = json.load(open(f"gpurun_out/{sys.argv[1]}_pmc_traffic.json"))["kernels"]
for k, v in t.items():
    if any(s in k for s in ("bloomw", "taa", "composition", "ssao_kernel")):
        print(f"{sys.argv[1]:10s} {k[:36]:36s} {v['hbm_bytes'] / 1e6:8.1f} MB")
PY
